#!/bin/bash
# Round-3 pass m: hardware queues per process (GPU_MAX_HW_QUEUES 4 = the
# box default vs 8) x split LSD for the lines leg; stereo and points legs at
# 4 / 8 queues.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03m
mkdir -p $O
cd $R
C="--no-cpu-baseline --sweep 0 --isolated-steps 0 --ingress-steps 0"
run() {  # tag env... -- args
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS $C > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], 'parity', d['parity']['pass'])"
}
ARGS="--workload lines --streams 3072 --steps 5 --warmup 2"
for r in 1 2; do
  run l_q4_s0_$r GPU_MAX_HW_QUEUES=4 ORBPL_LSD_SPLIT=0 || exit 1
  run l_q8_s0_$r GPU_MAX_HW_QUEUES=8 ORBPL_LSD_SPLIT=0 || exit 1
  run l_q8_s1_$r GPU_MAX_HW_QUEUES=8 ORBPL_LSD_SPLIT=1 || exit 1
done
ARGS="--workload kitti --streams 1024 --steps 4 --warmup 2"
run k_q4 GPU_MAX_HW_QUEUES=4 || exit 1
run k_q8 GPU_MAX_HW_QUEUES=8 || exit 1
ARGS="--steps 20 --warmup 5 --secondary-steps 0 --stereo-steps 0 --rig-steps 0"
run p_q4 GPU_MAX_HW_QUEUES=4 || exit 1
run p_q8 GPU_MAX_HW_QUEUES=8 || exit 1
