#!/bin/bash
# Round-3 pass w: headline batch 1024 vs 2048 streams (and 2048 with the ORB
# split), two rounds, parity on.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03w
mkdir -p $O
cd $R
C="--no-cpu-baseline --sweep 0 --ingress-steps 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0"
run() {  # tag env... -- args
  tag=$1; s=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --streams $s $C > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], 'parity', d['parity']['pass'], 'dom', d['roofline']['kernel'], d['roofline']['frac'])"
}
for r in 1 2; do
  run p1024_$r 1024 ORBPL_ORB_SPLIT=0 || exit 1
  run p2048_$r 2048 ORBPL_ORB_SPLIT=0 || exit 1
  run p2048s_$r 2048 ORBPL_ORB_SPLIT=1 || exit 1
done
