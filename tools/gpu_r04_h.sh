#!/bin/bash
# Round-4 pass h: k_lsd_validate variants at 1536 frames (time_lsd): kernel
# time (trace) and FETCH / WRITE per frame: cur (best rectangle in LDS, 8
# waves), valold (in registers), valw6 (LDS, 6 waves: fewer spills).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1 || { tail -30 $O/lsd_tests.log; exit 1; }
tail -1 $O/lsd_tests.log
for v in cur valold valw6; do
  L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
  ORBPL_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/t_$v -o run --output-format csv -- python3 $R/tools/time_lsd.py 1536 > $O/t_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $O/t_$v.log; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    ORBPL_LIB=$L timeout -s KILL 180 rocprofv3 --pmc $c -d $O/p_${v}_$c -o run --output-format csv -- python3 $R/tools/time_lsd.py 1536 > $O/p_${v}_$c.log 2>&1 || { echo "pmc $v $c failed"; tail -5 $O/p_${v}_$c.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, collections, os, glob
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r04h"
for v in ("cur", "valold", "valw6"):
    fs = glob.glob(f"{O}/t_{v}/**/run_kernel_stats.csv", recursive=True)
    ms = None
    for r in csv.DictReader(open(fs[0])):
        if "k_lsd_validate" in r["Name"]:
            ms = float(r["AverageNs"]) / 1e6
    tot = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"{O}/p_{v}_{c}/**/run_counter_collection.csv", recursive=True)[0]
        acc = 0.0; disp = set()
        for r in csv.DictReader(open(f)):
            if "k_lsd_validate" in r["Kernel_Name"]:
                acc += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
        tot[c] = acc / len(disp) * 1024 * (2 if c == "FETCH_SIZE" else 1) / 1536 / 1e6
    print(f"{v}: validate {ms:.3f} ms per 1536 frames, fetch x2 {tot['FETCH_SIZE']:.2f} MB/frame, write {tot['WRITE_SIZE']:.3f} MB/frame, sum {tot['FETCH_SIZE'] + tot['WRITE_SIZE']:.2f}")
PY
exit 0
