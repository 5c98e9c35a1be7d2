"""Deterministic fp32 elementary functions — numpy half of a bit-exact pair.

TEST INFRASTRUCTURE (oracle). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product path never does.

Why this exists
---------------
The reference computes the splat bounds with torch elementwise ops
(``encode.py:5-22`` exp/cos/sin/sqrt/log, ``render.py:19-30`` exp then
floor/ceil).  torch-CPU, torch-GPU and numpy ``exp``/``log``/``sin``/``cos`` differ
by an ulp on a large fraction of inputs, and an ulp can flip an integer AABB
bound (SURVEY.md §0 "Parity hazard").  So the HIP prep stage and this oracle
both use *the same* fixed-operation-order float32 algorithms: every step is a
single IEEE-754 binary32 add/sub/mul/div/sqrt, rint/floor/ceil or an exact bit
manipulation, with NO fused multiply-add.  numpy float32 array arithmetic and
hipcc with ``-ffp-contract=off`` both round each such step identically, so the
two sides agree bit-for-bit.  The device mirror is
``genetic-gaussian-splats_amd/csrc/ggs_detmath.h``; every constant is given by
its binary32 bit pattern on both sides.

Algorithms: Cephes-style (S. L. Moshier) single-precision exp/log/sin/cos —
Cody-Waite range reduction + short polynomials, ≈1 ulp.  Domain conventions
(identical on both sides): ``exp(x) = 0`` for ``x < -87`` (no denormals),
``+inf`` above 88.7228; ``log`` of a subnormal is computed after a 2^23
pre-scale; NaN in → NaN out.
"""
from __future__ import annotations

import numpy as np

_f32 = np.float32


def _c(bits: int) -> np.float32:
    return np.array([bits], dtype=np.uint32).view(np.float32)[0]


# --- constants (binary32 bit patterns; mirrored in ggs_detmath.h) ----------
LOG2E = _c(0x3FB8AA3B)
EXP_C1 = _c(0x3F318000)      # 0.693359375   (ln2 high part, 9 bits)
EXP_C2 = _c(0xB95E8083)      # -2.12194440e-4 (ln2 low part)
EXP_P = [_c(0x39506967), _c(0x3AB743CE), _c(0x3C088908),
         _c(0x3D2AA9C1), _c(0x3E2AAAAA), _c(0x3F000000)]
EXP_HI = _c(0x42B17218)      # 88.72284
EXP_LO = _c(0xC2AE0000)      # -87.0
SQRTHF = _c(0x3F3504F3)
LOG_P = [_c(0x3D9021BB), _c(0xBDEBD1B8), _c(0x3DEF251A), _c(0xBDFE5D4F),
         _c(0x3E11E9BF), _c(0xBE2AAE50), _c(0x3E4CCEAC), _c(0xBE7FFFFC),
         _c(0x3EAAAAAA)]
LOG_Q1 = _c(0xB95E8083)
LOG_Q2 = _c(0x3F318000)
TWO_OVER_PI = _c(0x3F22F983)
PIO2_1 = _c(0x3FC90000)      # 1.5703125 (8 significant bits)
PIO2_2 = _c(0x39FDA000)
PIO2_3 = _c(0x33A22169)
SIN_S = [_c(0xB94CA1F9), _c(0x3C08839E), _c(0xBE2AAAA3)]
COS_C = [_c(0x37CCF5CE), _c(0xBAB6061A), _c(0x3D2AAAA5)]
EPS12 = _c(0x2B8CBCCC)       # float32(1e-12)  (encode.py:15)
EPS6 = _c(0x358637BD)        # float32(1e-6)   (render.py:19-20)
HALF = _f32(0.5)
ONE = _f32(1.0)
TWO = _f32(2.0)
QUARTER = _f32(0.25)
FOUR = _f32(4.0)
TWO23 = _f32(8388608.0)


def _arr(x) -> np.ndarray:
    return np.ascontiguousarray(x, dtype=np.float32)


def exp_f32(x) -> np.ndarray:
    """Deterministic float32 e^x (mirror: ``det_expf``)."""
    x = _arr(x)
    with np.errstate(all="ignore"):
        fk = np.rint(x * LOG2E)
        r = x - fk * EXP_C1
        r = r - fk * EXP_C2
        zz = r * r
        y = EXP_P[0]
        y = y * r + EXP_P[1]
        y = y * r + EXP_P[2]
        y = y * r + EXP_P[3]
        y = y * r + EXP_P[4]
        y = y * r + EXP_P[5]
        y = y * zz
        y = y + r
        y = y + ONE
        k = np.clip(np.nan_to_num(fk, nan=0.0), -126, 128).astype(np.int32)
        big = k > 127
        y = np.where(big, y * TWO, y).astype(np.float32)
        k = np.where(big, k - 1, k)
        p2 = ((k + 127).astype(np.uint32) << np.uint32(23)).view(np.float32)
        out = (y * p2).astype(np.float32)
        out = np.where(x < EXP_LO, _f32(0.0), out)
        out = np.where(x > EXP_HI, _f32(np.inf), out)
        out = np.where(np.isnan(x), x, out)
    return out.astype(np.float32)


def log_f32(x) -> np.ndarray:
    """Deterministic float32 natural log (mirror: ``det_logf``)."""
    x = _arr(x)
    with np.errstate(all="ignore"):
        sub = (x > 0) & (x < np.finfo(np.float32).tiny)
        xs = np.where(sub, x * TWO23, x).astype(np.float32)
        bits = xs.view(np.uint32)
        e = ((bits >> np.uint32(23)) & np.uint32(0xFF)).astype(np.int32) - 126
        e = np.where(sub, e - 23, e)
        m = ((bits & np.uint32(0x807FFFFF)) | np.uint32(0x3F000000)).view(np.float32)
        lo = m < SQRTHF
        e = np.where(lo, e - 1, e)
        m = np.where(lo, (m + m) - ONE, m - ONE).astype(np.float32)
        z = m * m
        y = LOG_P[0]
        for c in LOG_P[1:]:
            y = y * m + c
        y = y * m
        y = y * z
        fe = e.astype(np.float32)
        y = y + fe * LOG_Q1
        y = y - HALF * z
        r = m + y
        r = r + fe * LOG_Q2
        r = np.where(x == 0, _f32(-np.inf), r)
        r = np.where(x == np.inf, _f32(np.inf), r)
        r = np.where((x < 0) | np.isnan(x), _f32(np.nan), r)
    return r.astype(np.float32)


def sincos_f32(x):
    """Deterministic float32 (sin x, cos x) (mirror: ``det_sincosf``)."""
    x = _arr(x)
    with np.errstate(all="ignore"):
        j = np.rint(x * TWO_OVER_PI)
        r = x - j * PIO2_1
        r = r - j * PIO2_2
        r = r - j * PIO2_3
        q = j - FOUR * np.floor(j * QUARTER)
        qi = np.nan_to_num(q, nan=0.0).astype(np.int32) & 3
        zz = r * r
        t = SIN_S[0] * zz
        t = t + SIN_S[1]
        t = t * zz
        t = t + SIN_S[2]
        t = t * zz
        t = t * r
        s = t + r
        t = COS_C[0] * zz
        t = t + COS_C[1]
        t = t * zz
        t = t + COS_C[2]
        t = t * zz
        t = t * zz
        t = t - HALF * zz
        c = t + ONE
        sin = np.select([qi == 0, qi == 1, qi == 2], [s, c, -s], -c).astype(np.float32)
        cos = np.select([qi == 0, qi == 1, qi == 2], [c, -s, -c], s).astype(np.float32)
        bad = ~np.isfinite(x)
        sin = np.where(bad, _f32(np.nan), sin)
        cos = np.where(bad, _f32(np.nan), cos)
    return sin.astype(np.float32), cos.astype(np.float32)
