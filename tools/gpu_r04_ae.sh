#!/bin/bash
# Round-4 pass ae: k_lbd with its gradient loads batched 8 samples at a time
# (cur) against the per-sample loop (lbd1): LSD / LineExtractor parity, the
# kernel at 1536 frames, then the lines leg.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ae
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1 || { echo "parity FAILED"; tail -30 $O/lsd_tests.log; exit 1; }
echo "cur $(tail -1 $O/lsd_tests.log)"
cd $R
bash tools/ab_lines_lib.sh "cur lbd1" 2
