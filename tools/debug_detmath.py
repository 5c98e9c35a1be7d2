import sys, ctypes as C, numpy as np
sys.path[:0] = ['genetic-gaussian-splats_amd', 'oracle']
import ggs
from detmath import exp_f32, log_f32, sincos_f32
ggs.ensure_init()
fp = C.POINTER(C.c_float)
def dev(fn, x, y=None):
    x = np.ascontiguousarray(x, np.float32); out = np.empty_like(x)
    yy = None if y is None else np.ascontiguousarray(y, np.float32)
    rc = ggs.lib.ggs_detmath_eval(fn, x.ctypes.data_as(fp), None if yy is None else yy.ctypes.data_as(fp), len(x), out.ctypes.data_as(fp))
    assert rc == 0, ggs._lib.last_error()
    return out
rng = np.random.default_rng(0)
xs = {'exp': rng.uniform(-90, 90, 1_000_000), 'log': np.exp(rng.uniform(-40, 40, 1_000_000)),
      'sin': rng.uniform(-200, 200, 1_000_000)}
def report(name, a, b, x):
    bad = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0]
    print(name, 'mismatches', len(bad), [(float(x[i]), float(a[i]), float(b[i])) for i in bad[:5]])
x = xs['exp'].astype(np.float32); report('exp', dev(0, x), exp_f32(x), x)
x = xs['log'].astype(np.float32); report('log', dev(1, x), log_f32(x), x)
x = xs['sin'].astype(np.float32); s, c = sincos_f32(x); report('sin', dev(2, x), s, x); report('cos', dev(3, x), c, x)
x = np.abs(xs['sin']).astype(np.float32); report('sqrt', dev(4, x), np.sqrt(x), x)
y = rng.uniform(0.1, 100, len(x)).astype(np.float32); report('div', dev(5, x, y), x / y, x)
