#!/bin/bash
# Round-3 pass o: split ORB extraction (two offset halves on two streams):
# tracker parity tests with the splits forced, the map tests, then points /
# lines / rig legs with ORBPL_ORB_SPLIT 0 / 1 (8 hardware queues).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03o
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_map.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/tests.log | head -20; exit $rc; }
C="--no-cpu-baseline --sweep 0 --isolated-steps 0 --ingress-steps 0"
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py $ARGS $C > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], 'parity', d['parity']['pass'])"
}
ARGS="--steps 20 --warmup 5 --secondary-steps 0 --stereo-steps 0 --rig-steps 0"
for r in 1 2; do
  run p_o0_$r ORBPL_ORB_SPLIT=0 || exit 1
  run p_o1_$r ORBPL_ORB_SPLIT=1 || exit 1
done
ARGS="--workload lines --streams 3072 --steps 5 --warmup 2"
run l_o0 ORBPL_ORB_SPLIT=0 || exit 1
run l_o1 ORBPL_ORB_SPLIT=1 || exit 1
ARGS="--workload rig --streams 256 --steps 10 --warmup 3"
run r_o0 ORBPL_ORB_SPLIT=0 || exit 1
run r_o1 ORBPL_ORB_SPLIT=1 || exit 1
