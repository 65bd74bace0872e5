#!/bin/bash
# Round-2 profile set: LSD seed-loop shader-clock profile at batch 1 / 64 /
# 3072, then the lines (3072 streams) and points (256) trace + PMC passes.
set -o pipefail
mkdir -p gpurun_out
for b in 1 64 3072; do
  timeout -k 10 120 python tools/time_lsd.py $b >> gpurun_out/time_lsd.log 2>&1 || { echo "time_lsd $b failed"; exit 1; }
done
echo time_lsd ok; cat gpurun_out/time_lsd.log
MODE=lines bash tools/prof.sh lines_r02 || exit 1
MODE=points SQ=1 bash tools/prof.sh points_r02 || exit 1
