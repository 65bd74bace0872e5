#!/bin/bash
# Quick GPU check: map parity + the headline leg only (no secondary legs).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py -q --timeout 300 --timeout-method thread > gpurun_out/gpu_map_q.log 2>&1
rc=$?
echo "map tests rc=$rc"; tail -2 gpurun_out/gpu_map_q.log
if [ $rc -ne 0 ]; then grep -E "assert|Error" gpurun_out/gpu_map_q.log | head -20; exit 1; fi
timeout -k 10 600 python -u bench.py --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --sweep 0 --no-cpu-baseline $QUICK_ARGS > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { echo "bench failed"; tail -20 gpurun_out/bench_q.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_q.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "parity", d["parity"]["pass"])
print("stages", d["stage_ms"])
print("isolated", d["roofline"].get("isolated", {}).get("stage_ms"))
PY
