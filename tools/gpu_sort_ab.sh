#!/bin/bash
# LSD introsort replay: stopper-mask global levels vs stopper positions.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_lsd_sort.log 2>&1
rc=$?
echo "lsd tests rc=$rc"; tail -3 gpurun_out/gpu_lsd_sort.log
if [ $rc -ne 0 ]; then grep -E "assert|Error|FAILED" gpurun_out/gpu_lsd_sort.log | head -20; exit 1; fi
for B in 1024 3072; do
  for m in 0 1; do
    ORBPL_SORT_MASKS=$m timeout -k 10 300 python -u tools/time_lsd.py $B > gpurun_out/time_sort_${B}_$m.log 2>&1 || { echo "time_lsd failed"; tail -5 gpurun_out/time_sort_${B}_$m.log; exit 1; }
    echo "masks=$m $(head -1 gpurun_out/time_sort_${B}_$m.log)"
  done
done
mkdir -p gpurun_out/sortprof
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
ORBPL_SORT_MASKS=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/sortprof/t$m -o run --output-format csv -- python3 $R/tools/time_lsd.py 3072 > $R/gpurun_out/sortprof/t$m.log 2>&1 || { echo "trace failed"; exit 1; }
python3 $R/tools/trace_summary.py $R/gpurun_out/sortprof/t$m/run_kernel_trace.csv | head -8
done
