#!/bin/bash
# Round-4 pass ak: where the second LSD half starts on the lines leg
# (ORBPL_LSD_STAGGER 0 = step start, 1 = after the first half's sort (default),
# 2 = after its seed loop) with this session's faster sorts, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r04ak
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --isolated-steps 0"
for r in 1 2; do
  for st in 1 0 2; do
    ORBPL_LSD_STAGGER=$st timeout -k 10 300 python bench.py --workload lines --streams 3072 --steps 4 --warmup 1 $C > gpurun_out/r04ak/b_${st}_$r.log 2>&1 || { echo "fail $st"; exit 1; }
    grep '^{' gpurun_out/r04ak/b_${st}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r stagger $st lines', round(d['value']), d['ms_per_step'])"
  done
done
