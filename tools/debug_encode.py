import sys, os, numpy as np
sys.path[:0] = ['genetic-gaussian-splats_amd', 'oracle']
import ggs, ggs_oracle as O
from detmath import exp_f32, log_f32, sincos_f32
G = np.load('tests/golden/encode.npz')['edge_in']
a = ggs.encode(G)[0]; b = O.genome_to_renderer_batched(G)[0]
for col in range(9):
    bad = np.nonzero(a[:, col] != b[:, col])[0]
    print('col', col, 'nbad', len(bad))
    for i in bad[:6]:
        print('   ', i, G[0, i, :5], a[i, col], b[i, col], a[i,col].view(np.uint32), b[i,col].view(np.uint32))
# probe detmath pieces via render prep: exp through preprocess of renderer genome
x = np.linspace(-10, 10, 4001, dtype=np.float32)
g = np.zeros((len(x), 9), np.float32); g[:, 2] = x; g[:, 3] = x
p = ggs.preprocess(g, 64, 64, 3.0)
l11 = np.maximum(exp_f32(x), np.float32(1e-6))
i11 = np.float32(1) / l11
print('exp-probe sxx mismatches', int((p['syy'] != (i11 * i11)).sum()))
