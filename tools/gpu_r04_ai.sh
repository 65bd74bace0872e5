#!/bin/bash
# Round-4 pass ai: the introsort test hook on the production configuration
# (1024 threads, segment table, chunk map) + all LSD parity, then the stereo
# and rig legs' kernel traces and FETCH / WRITE PMC for this build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ai
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1 || { echo "parity FAILED"; tail -30 $O/lsd_tests.log; exit 1; }
echo "lsd $(tail -1 $O/lsd_tests.log)"
MODE=kitti bash tools/prof.sh s2kitti && MODE=rig bash tools/prof.sh s2rig
