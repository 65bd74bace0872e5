#!/bin/bash
# Round-3 pass ab: where the second LSD half starts (ORBPL_LSD_STAGGER 0 =
# step start, 1 = after the first half's sort (default), 2 = after its seed
# loop) on the lines leg, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03ab
mkdir -p $O
cd $R
C="--workload lines --streams 3072 --steps 5 --warmup 2 --no-cpu-baseline --sweep 0 --isolated-steps 0 --ingress-steps 0"
for r in 1 2; do
  for v in 1 0 2; do
    ORBPL_LSD_STAGGER=$v timeout -k 10 300 python bench.py $C > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench $v failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('stagger $v r$r', d['value'], d['ms_per_step'], 'parity', d['parity']['pass'])"
  done
done
