#!/bin/bash
# k_pose change check: the pose / tracker / map parity tests, stream 0's pose
# phase profile at 1024 streams, then the headline leg.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/poseab
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_map.py tests/test_gpu_dropin.py tests/test_gpu_errors.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "assert|Error" $O/tests.log | head -20; exit 1; fi
ORBPL_POSE_PROFILE=1 timeout -k 10 240 python3 tools/probe_track.py 1024 0 1 > $O/probe.log 2>&1 || { echo "probe failed"; tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
# A/B variants: "name:ENV=VAL[,ENV=VAL]" (lib from variants/<name>/ when it exists)
for v in $VARIANTS; do
  name=${v%%:*}; envs=${v#*:}; [ "$envs" = "$v" ] && envs=""
  (
    [ -f variants/$name/liborbpl.so ] && export ORBPL_LIB=$R/variants/$name/liborbpl.so
    for kv in ${envs//,/ }; do export "$kv"; done
    ORBPL_POSE_PROFILE=1 timeout -k 10 240 python3 tools/probe_track.py 1024 0 1 > $O/probe_$name.log 2>&1
  ) || { echo "probe $name failed"; tail -5 $O/probe_$name.log; exit 1; }
  echo "== $name"; cat $O/probe_$name.log
done
timeout -k 10 600 python -u bench.py --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --sweep 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - <<PY
import json
d = json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "parity", d["parity"]["pass"])
print("stages", d["stage_ms"])
print("isolated", d["roofline"].get("isolated", {}).get("stage_ms"))
PY
if [ -n "$BENCH2_ENV" ]; then
  env $BENCH2_ENV timeout -k 10 600 python -u bench.py --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --sweep 0 --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err || { echo "bench2 failed"; tail -20 $O/bench2.err; exit 1; }
  python3 - <<PY
import json
d = json.loads(open("$O/bench2.json").read().strip().splitlines()[-1])
print("bench2 ($BENCH2_ENV) value", d["value"], "ms", d["ms_per_step"], "parity", d["parity"]["pass"])
print("stages", d["stage_ms"])
PY
fi
