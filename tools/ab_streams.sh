#!/bin/bash
# One workload at several stream counts and environment settings:
#   tools/ab_streams.sh <workload> "<streams...>" "<NAME=VALUE|- ...>" [steps]
# prints frames/s, ms per step and the LSD / extraction stage times per run
# (the bench's detail file); logs under gpurun_out/ab/.
set -o pipefail
mkdir -p gpurun_out/ab
W=$1; SS=$2; ES=${3:--}; K=${4:-3}
B="--workload $W --steps $K --warmup 1 --no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for s in $SS; do
  for e in $ES; do
    tag=$(echo "${W}_${s}_$e" | tr '=/,' '___')
    D=gpurun_out/ab/st_$tag.detail.json
    if [ "$e" = "-" ]; then
      timeout -k 10 400 python bench.py --streams $s $B --detail $D > gpurun_out/ab/st_$tag.log 2>&1 || { echo "fail $tag"; tail -3 gpurun_out/ab/st_$tag.log; exit 1; }
    else
      env "$e" timeout -k 10 400 python bench.py --streams $s $B --detail $D > gpurun_out/ab/st_$tag.log 2>&1 || { echo "fail $tag"; tail -3 gpurun_out/ab/st_$tag.log; exit 1; }
    fi
    python -c "import json; d=json.load(open('$D')); st=d['stage_ms']; print('$W', $s, '$e', round(d['value']), d['ms_per_step'], {k: round(st[k], 1) for k in ('pyramid', 'fast', 'lsd', 'lsd_seed', 'lsd_sort', 'lsd_validate', 'match', 'pose') if k in st})"
  done
done
