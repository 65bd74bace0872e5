#!/bin/bash
# Round-3 pass p: hardware queues 8 vs 16 with both batch splits at their
# defaults, every leg, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03p
mkdir -p $O
cd $R
for r in 1 2; do
  for q in 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --no-cpu-baseline --sweep 0 --isolated-steps 0 > $O/b_${q}_$r.json 2> $O/b_${q}_$r.err || { echo "bench $q failed"; tail -5 $O/b_${q}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_${q}_$r.json').read().strip().splitlines()[-1])
print('q$q r$r points', d['value'], 'lines', d['secondary']['value'], 'stereo', d['stereo']['value'], 'rig', d['rig']['value'], 'ingress', d['ingress']['value'], 'parity', d['parity']['pass'])"
  done
done
