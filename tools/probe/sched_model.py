"""Dispatch-order model of one raster launch: per-(candidate, strip) work from
the raster's visit geometry (VALU ~HEAD per visit + PK per pair step + the cull
and epilogue per wave), waves placed on 1,024 SIMDs x 3 slots in block order
(each to a SIMD with the fewest resident waves), SIMDs sharing their VALU among
resident waves (aggregate issue rate TPUT[k] with k waves).  Prints the makespan
against the ideal (total work / (1,024 x TPUT[3])) for the shipped order
(centre-first strip groups, candidates rotating) and alternatives.

    python tools/probe/sched_model.py [--size 512 --splats 256 --pop 128]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
import ggs_oracle as O  # noqa: E402

TILE, TILE_H, NPK = 64, 128, 16
HEAD, PK, CULL, EPI = 30.0, 7.0, 12.0, 260.0       # VALU-equivalent slots
TPUT = {0: 0.0, 1: 0.80, 2: 0.95, 3: 1.0}


def strip_costs(pop, size, k=3.0):
    """[B, G] work per (candidate, strip), G = tiles x 4 (the raster's strip index t*4+wv)."""
    B, N = pop.shape[:2]
    nTX, nTY = -(-size // TILE), -(-size // TILE_H)
    G = nTX * nTY * 4
    cost = np.zeros((B, G))
    for b in range(B):
        p = O.preprocess(O.genome_to_renderer_batched(pop[b][None])[0], size, size, k)
        x0, x1, y0, y1 = (p[q].astype(np.int64) for q in ("x0", "x1", "y0", "y1"))
        c = np.full(G, EPI + CULL * -(-N // 64))
        for i in range(N):
            for ty in range(y0[i] // TILE_H, y1[i] // TILE_H + 1):
                ty0 = ty * TILE_H
                dy0, dy1 = y0[i] - ty0, y1[i] - ty0
                kA = (max(dy0, 0) >> 2) >> 1
                kB = NPK - 1 if dy1 >= TILE_H - 1 else (min(dy1, TILE_H - 1) >> 2) >> 1
                for sx in range(x0[i] // 16, x1[i] // 16 + 1):
                    t = ty * nTX + (sx >> 2)
                    c[t * 4 + (sx & 3)] += HEAD + PK * (kB - kA + 1)
        cost[b] = c
    return cost


def simulate(work, n_simd=1024, slots=3):
    """Makespan of `work` (in dispatch order) under processor sharing."""
    rem = np.zeros((n_simd, slots))
    live = np.zeros((n_simd, slots), bool)
    t, nxt, n = 0.0, 0, len(work)
    while True:
        while nxt < n:                      # fill free slots, fewest-resident SIMD first
            k = live.sum(1)
            s = int(np.argmin(np.where(k < slots, k, slots + 1)))
            if k[s] >= slots:
                break
            j = int(np.argmin(live[s]))
            rem[s, j], live[s, j] = work[nxt], True
            nxt += 1
        k = live.sum(1)
        if not k.any():
            return t
        rate = np.array([TPUT[int(x)] / x if x else 0.0 for x in range(slots + 1)])[k]
        tt = np.where(live, rem / np.maximum(rate[:, None], 1e-30), np.inf)
        dt = tt.min()
        t += dt
        rem = np.where(live, rem - dt * rate[:, None], 0.0)
        done = live & (rem <= 1e-9)
        live &= ~done


def centre_order(size):
    nTX, nTY = -(-size // TILE), -(-size // TILE_H)
    d = []
    for g in range(nTX * nTY * 4):
        t, s = g // 4, g % 4
        cx = (t % nTX) * TILE + (s + 0.5) * 16 - 0.5 * size
        cy = (t // nTX) * TILE_H + 0.5 * TILE_H - 0.5 * size
        d.append((cx * cx + cy * cy, g))
    return [g for _, g in sorted(d)]


def shipped(cost, size):
    B, G = cost.shape
    order = centre_order(size)
    return np.array([cost[(i + gi) % B, order[gi]] for gi in range(G) for i in range(B)])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--splats", type=int, default=256)
    ap.add_argument("--pop", type=int, default=128)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    pop = O.synthetic_population(a.pop, a.splats, a.size, a.size, seed=a.seed)
    cost = strip_costs(pop, a.size)
    ideal = cost.sum() / (1024 * TPUT[3])
    rows = {"shipped (centre-first groups)": shipped(cost, a.size),
            "exact LPT (per item)": np.sort(cost.ravel())[::-1],
            "random": np.random.default_rng(1).permutation(cost.ravel())}
    for name, w in rows.items():
        m = simulate(w)
        print(f"{name:32s} makespan {m:10.0f}  x ideal {m / ideal:.3f}")
    print(f"items {cost.size}, mean {cost.mean():.0f}, max {cost.max():.0f}, ideal {ideal:.0f}")


def split_model(pop, size, extra=300.0):
    """Depth split: each strip as two waves over the splat index halves (no
    duplicated visits; each half culls its own half), `extra` slots per half-wave
    for the state hand-off (store or load + compose of 32 px x 4 values/lane)."""
    N = pop.shape[1]
    cf = strip_costs(pop[:, N // 2:], size) + extra
    cb = strip_costs(pop[:, :N // 2], size) + extra
    return cf, cb


def simulate_fixed(work, n_simd=1024):
    """Single-round launch placed as the hardware does it (EXP §14: blocks r,
    r + 1,024, r + 2,048 share SIMD r): the makespan under processor sharing."""
    n = len(work)
    per = -(-n // n_simd)
    loads = np.zeros((n_simd, per))
    for i, w in enumerate(work):
        loads[i % n_simd, i // n_simd] = w
    t_end = np.zeros(n_simd)
    for s in range(n_simd):
        rem = sorted(x for x in loads[s] if x > 0)
        t, prev = 0.0, 0.0
        k = len(rem)
        for x in rem:                      # processor sharing: shortest finishes first
            rate = TPUT[k] / k
            t += (x - prev) / rate
            prev = x
            k -= 1
        t_end[s] = t
    return t_end.max()


def group_order_blocks(cost, order):
    """Block-order work of a launch whose strip groups run in `order` (candidates rotating)."""
    B, G = cost.shape
    return np.array([cost[(i + gi) % B, order[gi]] for gi in range(G) for i in range(B)])
