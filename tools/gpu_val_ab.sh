#!/bin/bash
# LSD NFA validation A/B: a walk per evaluation vs merged p-halving walks
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/valab
cd $R
ORBPL_VAL_MERGED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_lsd_val.log 2>&1
rc=$?
echo "lsd tests (merged) rc=$rc"; tail -2 gpurun_out/gpu_lsd_val.log
if [ $rc -ne 0 ]; then grep -E "assert|Error|FAILED" gpurun_out/gpu_lsd_val.log | head -20; exit 1; fi
cd /tmp && export TMPDIR=/tmp
for m in 0 1 0 1; do
ORBPL_VAL_MERGED=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/valab/t$m -o run --output-format csv -- python3 $R/tools/time_lsd.py 3072 > $R/gpurun_out/valab/t$m.log 2>&1 || { echo "trace failed"; exit 1; }
echo "merged=$m $(python3 $R/tools/trace_summary.py $R/gpurun_out/valab/t$m/run_kernel_trace.csv | grep k_lsd_validate)"
done
