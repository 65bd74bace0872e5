#!/bin/bash
# map parity (incl. element-wise maps) + drop-in
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_dropin.py -v --timeout 300 --timeout-method thread > gpurun_out/gpu_map2.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "PASSED|FAILED|Error|assert " gpurun_out/gpu_map2.log | head -30
exit $rc
