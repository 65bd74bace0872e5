#!/bin/bash
# Round-4 pass ac: pyramid row bands per frame at 1024 frames (default 1 vs
# ORBPL_PYR_BANDS=2 / 4): headline leg with isolated stage times, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ac
mkdir -p $O
cd $R
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --trk-load 0"
for r in 1 2; do
  for nb in 0 2 4; do
    if [ $nb = 0 ]; then unset ORBPL_PYR_BANDS; else export ORBPL_PYR_BANDS=$nb; fi
    timeout -k 10 300 python bench.py $C > $O/b_${nb}_$r.log 2>&1 || { echo "bench $nb failed"; tail -5 $O/b_${nb}_$r.log; exit 1; }
    grep '^{' $O/b_${nb}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); i=d['roofline']['isolated']['stage_ms']; print('$r bands $nb', round(d['value']), d['ms_per_step'], 'iso pyr %.3f fast %.3f oct %.3f od %.3f' % (i['pyramid'], i['fast'], i['octree'], i['orient_desc']))"
  done
done
