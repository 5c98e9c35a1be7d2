#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the 512^2 raster for several libggs builds (one PMC pass
# per counter and build): LIBS="libggs libggs_x" under the package dir.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/traffic_ab; mkdir -p $OUT
P=genetic-gaussian-splats_amd
for L in ${LIBS:-libggs}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    GGS_LIB=$PWD/$P/$L.so timeout -k 10 120 rocprofv3 --pmc $C -d $OUT/${L}_$C -o run --output-format csv -- \
      python3 tools/probe/rtime.py --worker --config 512 --steps 40 --out /tmp/ta.npy > $OUT/${L}_$C.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$L $C rc=$rc"; tail -5 $OUT/${L}_$C.log; exit $rc; }
  done
  python3 - $OUT $L <<'PY'
import csv, sys, glob
out, L = sys.argv[1], sys.argv[2]
res = {}
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{out}/{L}_{C}/**/run_counter_collection.csv", recursive=True)[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "raster_kernel" in r["Kernel_Name"]]
    res[C] = sum(v[-40:]) / 40
print(f"{L}: FETCH_SIZE x2 {res['FETCH_SIZE'] * 2048 / 1e6:.1f} MB  WRITE {res['WRITE_SIZE'] * 1024 / 1e6:.2f} MB per launch")
PY
done
