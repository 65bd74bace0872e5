#!/bin/bash
# small-batch seed loop: register budget A/B (ORBPL_SPEC_SMALL=0 = the bounded variant)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_lsd_small.log 2>&1
rc=$?
echo "lsd tests rc=$rc"; tail -2 gpurun_out/gpu_lsd_small.log
if [ $rc -ne 0 ]; then grep -E "assert|Error|FAILED" gpurun_out/gpu_lsd_small.log | head -20; exit 1; fi
for B in 1 16 64; do
  for v in 0 96; do
    ORBPL_SPEC_SMALL=$v timeout -k 10 300 python -u tools/time_lsd.py $B > gpurun_out/time_small_${B}_$v.log 2>&1 || { echo "time_lsd failed"; tail -5 gpurun_out/time_small_${B}_$v.log; exit 1; }
    echo "small=$v $(head -1 gpurun_out/time_small_${B}_$v.log)"
  done
done
