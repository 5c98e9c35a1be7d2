#!/bin/bash
# Kernel trace of the SA device loop at configs[4] (start of run; SA_ARGS for the late regime).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sa_tr; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sa_tr -o run --output-format csv -- python3 tools/bench_sa.py --only device_loop_full --dev-iters 100 --repeat 1 ${SA_ARGS:-} > gpurun_out/sa_tr/log.txt 2>&1 || exit $?
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/sa_tr/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# the timed loop: the last 40 % of the trace
rows = rows[int(len(rows) * 0.6):]
import collections
d = collections.defaultdict(list)
for r in rows:
    d[r['Kernel_Name'][:40]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
span = (int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])) / 1e3
busy = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(k.ljust(40), len(v), '%8.2f us avg' % (sum(v) / len(v)))
print('span %.0f us, kernel-busy %.0f us, gaps %.0f us over %d launches' % (span, busy, span - busy, len(rows)))
PY
