#!/bin/bash
# LSD balanced seed loop: bit-exactness, then A/B timing vs k_lsd_spec.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_lsd_bal.log 2>&1
rc=$?
echo "lsd tests rc=$rc"; tail -3 gpurun_out/gpu_lsd_bal.log
if [ $rc -ne 0 ]; then grep -E "assert|Error|FAILED" gpurun_out/gpu_lsd_bal.log | head -20; exit 1; fi
for B in 1 64 1024 3072; do
  for bal in 0 1; do
    ORBPL_LSD_BAL=$bal timeout -k 10 300 python -u tools/time_lsd.py $B > gpurun_out/time_lsd_${B}_$bal.log 2>&1 || { echo "time_lsd failed"; tail -5 gpurun_out/time_lsd_${B}_$bal.log; exit 1; }
    echo "bal=$bal $(head -2 gpurun_out/time_lsd_${B}_$bal.log | tr '\n' ' ')"
  done
done
