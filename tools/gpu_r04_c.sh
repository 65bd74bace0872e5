#!/bin/bash
# Round-4 pass c: LSD parity with the tiled degree plane, then kernel trace +
# FETCH / WRITE PMC + two SQ passes of the headline (points, 1024 streams) and
# trace + PMC of the lines leg (3072).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lsd.py tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04c_lsd.log 2>&1 || { tail -30 gpurun_out/r04c_lsd.log; exit 1; }
tail -2 gpurun_out/r04c_lsd.log
MODE=points SQ=1 SQ2=1 bash tools/prof.sh r04_points || exit 1
MODE=lines bash tools/prof.sh r04_lines || exit 1
exit 0
