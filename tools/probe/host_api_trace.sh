#!/bin/bash
# Timeline of host-API calls (ggs.fitness, 512^2/256/128): kernels and copies per call.
#   LIB=libggs bash tools/probe/host_api_trace.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
L=${LIB:-libggs}; OUT=gpurun_out/hat_$L; mkdir -p $OUT
GGS_HIP_RUNTIME=system GGS_LIB=$PWD/genetic-gaussian-splats_amd/$L.so timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace \
    -d $OUT -o run --output-format csv -- python3 tools/probe/host_api_probe.py > $OUT/log.txt 2>&1 || exit $?
python3 - $OUT <<'PY'
import csv, glob, sys
d = sys.argv[1]
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:28], r.get("Stream_Id", r.get("Queue_Id", ""))))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")[:12] + " %s B" % r.get("Bytes", "?"), r.get("Stream_Id", "")))
ev.sort()
ev = ev[-60:]
t0 = ev[0][0]
for a, b, n, s in ev:
    print("%9.1f %9.1f %7.1f  %-40s %s" % ((a - t0) / 1e3, (b - t0) / 1e3, (b - a) / 1e3, n, s))
PY
