"""Dispatch-order experiment (probe build, GGS_PROBE_ORDER): strip-group orders for
rtime.py's 2048^2 SA configs from the model's per-strip costs (sched_model.py) of
the exact populations rtime.py renders, with the model's makespan per order.

    python tools/probe/order_exp.py --pop 2      -> tools/probe/orders/sa2_{lpt,centre}.bin
    python tools/probe/order_exp.py --pop 24 --size 512 --splats 512 --tag ga24
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, HERE, os.path.join(REPO, "oracle")]
import sched_model as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pop", type=int, default=2)
ap.add_argument("--size", type=int, default=2048)
ap.add_argument("--splats", type=int, default=4096)
ap.add_argument("--same", action="store_true", help="rtime.py --same populations")
ap.add_argument("--tag", default="")
a = ap.parse_args()
import bench  # noqa: E402
bench.H = bench.W = a.size
costs = []
for i in range(4):                       # rtime.py's four populations
    pop = bench.synthetic_population(a.pop, a.splats, 10_000 + (0 if a.same else i))
    if a.same:               # rtime.py --same: pop 0's first candidate, repeated
        pop = np.ascontiguousarray(np.broadcast_to(pop[:1], pop.shape))
    costs.append(M.strip_costs(pop, a.size))
avg = np.mean([c.mean(0) for c in costs], 0)
centre = np.array(M.centre_order(a.size))
orders = {"centre": centre, "lpt": np.argsort(-avg, kind="stable")}
for name, o in orders.items():
    ms = [M.simulate(M.group_order_blocks(c, list(o))) for c in costs]
    ideal = [c.sum() / 1024 for c in costs]
    print(f"{name:8s} model makespan x ideal " + " ".join("%.3f" % (m / i) for m, i in zip(ms, ideal)))
    o.astype(np.int32).tofile(os.path.join(HERE, "orders", f"{a.tag or 'sa%d' % a.pop}{'same' if a.same else ''}_{name}.bin"))
