#!/bin/bash
# Round-3 GPU pass c: map parity, the -m gpu suite, smoke, default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_dropin.py -v --timeout 300 --timeout-method thread > gpurun_out/gpu_map.log 2>&1
rc=$?
echo "map+dropin tests rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/gpu_map.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --ignore tests/test_gpu_map.py --ignore tests/test_gpu_dropin.py > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -4 gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r03_c.json 2> gpurun_out/bench_r03_c.err || { echo "bench failed"; tail -20 gpurun_out/bench_r03_c.err; exit 1; }
echo bench ok
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_r03_c.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"], d["parity"]["pass"])
for k in ("secondary", "stereo", "rig"):
    if k in d: print(k, d[k]["value"], d[k]["parity"]["pass"] if d[k]["parity"] else None)
PY
