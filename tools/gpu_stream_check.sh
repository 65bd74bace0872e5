#!/bin/bash
# The round-free seed loop (k_lsd_stream): LSD parity tests, then LSD batch
# timings with the stream kernel (default for batches <= 96) and the round
# loop (ORBPL_LSD_STREAM=0). Each GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${1:-stream}
mkdir -p $O
cd $R
timeout -k 10 120 python tools/time_lsd.py 1 > $O/time_first.log 2>&1 || { echo "first stream run failed"; tail -5 $O/time_first.log; exit 1; }
cat $O/time_first.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_lsd.py -x -v --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1
rc=$?; echo "lsd tests exit $rc"; tail -3 $O/lsd_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/lsd_tests.log | head -20; exit $rc; }
for b in 1 16 64; do
  timeout -k 10 120 python tools/time_lsd.py $b >> $O/time_stream.log 2>&1 || { echo "stream $b failed"; tail -5 $O/time_stream.log; exit 1; }
  ORBPL_LSD_STREAM=0 timeout -k 10 120 python tools/time_lsd.py $b >> $O/time_round.log 2>&1 || { echo "round $b failed"; exit 1; }
done
echo "== stream"; cat $O/time_stream.log
echo "== round"; cat $O/time_round.log
