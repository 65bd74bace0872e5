#!/bin/bash
# Round-4 pass i: the whole -m gpu suite on the current build, smoke(), then
# the LSD detector at 1 / 16 frames (sort_local spread over more blocks).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04i
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04i/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r04i/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r04i/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04i/smoke.log 2>&1 || { tail -20 gpurun_out/r04i/smoke.log; exit 1; }
tail -1 gpurun_out/r04i/smoke.log
export GPU_MAX_HW_QUEUES=16
for B in 1 16; do
  timeout -k 10 180 python3 tools/time_lsd.py $B > gpurun_out/r04i/time_lsd_$B.log 2>&1 || { tail -5 gpurun_out/r04i/time_lsd_$B.log; exit 1; }
  head -1 gpurun_out/r04i/time_lsd_$B.log
done
exit 0
