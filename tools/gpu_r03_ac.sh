#!/bin/bash
# Round-3 pass ac: stereo + lines with the left image's LSD batch split
# (ORBPL_LSD_SPLIT=1): stereo tracker parity tests with it forced, then the
# KITTI leg (1024 pairs) without / with, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03ac
mkdir -p $O
cd $R
ORBPL_LSD_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_track.py -k "stereo" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/tests.log | head; exit $rc; }
C="--workload kitti --streams 1024 --steps 5 --warmup 2 --no-cpu-baseline --sweep 0 --isolated-steps 0 --ingress-steps 0"
for r in 1 2; do
  for v in 0 1; do
    ORBPL_LSD_SPLIT=$v timeout -k 10 300 python bench.py $C > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench $v failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('split $v r$r', d['value'], d['ms_per_step'], 'parity', d['parity']['pass'])"
  done
done
