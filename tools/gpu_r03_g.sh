#!/bin/bash
# Round-3 pass g (session 3): full -m gpu suite at HEAD, LSD stage times +
# seed-loop phase profile at batch 1 / 3072, then the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" $O/gpu_tests.log | head -20; exit $rc; }
for b in 1 3072; do
  timeout -k 10 120 python tools/time_lsd.py $b >> $O/time_lsd.log 2>&1 || { echo "time_lsd $b failed"; tail -5 $O/time_lsd.log; exit 1; }
done
cat $O/time_lsd.log
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; tail -c 300 $O/bench.json
exit $rc
