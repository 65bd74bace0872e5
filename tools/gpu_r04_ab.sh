#!/bin/bash
# Round-4 pass ab: k_orient_desc with two keypoints per wave (cur) against one
# (ORBPL_OD_PAIR=0): ORB parity tests, then the headline leg (isolated stage
# times), two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ab
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > $O/orb_tests.log 2>&1 || { echo "parity FAILED"; tail -30 $O/orb_tests.log; exit 1; }
echo "cur $(tail -1 $O/orb_tests.log)"
C="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --trk-load 0"
for r in 1 2; do
  for v in cur one; do
    P=1; [ "$v" = one ] && P=0
    ORBPL_OD_PAIR=$P timeout -k 10 300 python bench.py $C > $O/b_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -5 $O/b_${v}_$r.log; exit 1; }
    grep '^{' $O/b_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); i=d['roofline']['isolated']['stage_ms']; print('$r $v', round(d['value']), d['ms_per_step'], 'iso pyr %.3f fast %.3f oct %.3f od %.3f' % (i['pyramid'], i['fast'], i['octree'], i['orient_desc']))"
  done
done
