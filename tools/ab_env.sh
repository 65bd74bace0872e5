#!/bin/bash
# Headline bench A/B over an environment setting: for each stream count in $2
# (default "256 1024") runs the bench with each assignment in $1 (space-
# separated NAME=VALUE items, "-" = none) and prints frames/s per run.
set -o pipefail
mkdir -p gpurun_out/ab
ES=${1:--}
SS=${2:-256 1024}
B="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for s in $SS; do
  for e in $ES; do
    tag=$(echo "$e" | tr '=/,' '___')
    if [ "$e" = "-" ]; then
      timeout -k 10 200 python bench.py --streams $s --steps 10 --warmup 3 $B --detail gpurun_out/ab/env_${tag}_$s.detail.json > gpurun_out/ab/env_${tag}_$s.log 2>&1 || exit 1
    else
      env "$e" timeout -k 10 200 python bench.py --streams $s --steps 10 --warmup 3 $B --detail gpurun_out/ab/env_${tag}_$s.detail.json > gpurun_out/ab/env_${tag}_$s.log 2>&1 || exit 1
    fi
    python -c "import json; d=json.load(open('gpurun_out/ab/env_${tag}_$s.detail.json')); st=d['stage_ms']; print('$e', $s, round(d['value']), d['ms_per_step'], 'stages', {k: st[k] for k in ('pyramid', 'fast', 'octree', 'orient_desc', 'match', 'pose', 'local_map')})"
  done
done
