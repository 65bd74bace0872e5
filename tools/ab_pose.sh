#!/bin/bash
# k_pose configuration A/B (ORBPL_POSE_CFG="threads,waves") on the headline
# bench at the stream counts in $1 ("auto" = launch_pose's own choice).
set -o pipefail
mkdir -p gpurun_out/ab
SS=${1:-512 1024}
CS=${2:-auto 128,1 64,1 128,2 64,2}
for s in $SS; do
  for c in $CS; do
    E=""; [ "$c" != auto ] && E="$c"
    tag=$(echo "$c" | tr , x)
    ORBPL_POSE_CFG=$E timeout -k 10 200 python bench.py --streams $s --steps 10 --warmup 3 --no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --isolated-steps 3 --ingress-steps 0 > gpurun_out/ab/pose${tag}_$s.log 2>&1 || { echo "fail $c $s"; tail -n 5 gpurun_out/ab/pose${tag}_$s.log; exit 1; }
  done
done
