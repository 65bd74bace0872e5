#!/bin/bash
# the default bench (driver contract), output kept under gpurun_out/
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
start=$(date +%s)
timeout -k 10 1100 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -20 gpurun_out/bench_default.err; exit 1; }
echo "bench ok in $(( $(date +%s) - start )) s"
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_default.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"], d["parity"]["pass"], d["tracking"].get("sampled_streams_keyframes"))
for k in ("secondary", "stereo", "rig"):
    if k in d: print(k, d[k]["value"], d[k]["parity"]["pass"] if d[k]["parity"] else None)
print("ingress", d.get("ingress", {}).get("value"), "cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["reference_faithful"]["median_ms_per_frame"])
PY
