#!/bin/bash
# Round-4 pass l: headline A/B of ORBPL_EXTRACT_CU_RESERVE (0 = all CUs for the
# extraction stream, k = the last k CUs of every 32 left to the tracking
# stream), 2 rounds, 20 timed steps.
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
A="--steps 20 --warmup 5 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --no-cpu-baseline --sweep 0 --trk-load 0 --isolated-steps 0 --no-parity"
for r in 1 2; do
  for k in 0 1 2 4; do
    ORBPL_EXTRACT_CU_RESERVE=$k timeout -k 10 300 python bench.py $A > $O/b_${k}_$r.json 2> $O/b_${k}_$r.err || { echo "fail $k"; tail -3 $O/b_${k}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${k}_$r.json')); print('$r reserve $k', d['value'], d['ms_per_step'])"
  done
done
exit 0
