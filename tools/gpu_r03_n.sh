#!/bin/bash
# Round-3 pass n: full -m gpu suite, then the default bench (8 hardware
# queues, split LSD) and the default bench at 16 queues.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03n
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 $O/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "assert|Error|FAILED" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit $rc"; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
GPU_MAX_HW_QUEUES=16 timeout -k 10 420 python bench.py --no-cpu-baseline > $O/bench16.json 2> $O/bench16.err
rc=$?; echo "bench16 exit $rc"
python3 - <<PY
import json
for f in ["bench", "bench16"]:
    d = json.loads(open("$O/%s.json" % f).read().strip().splitlines()[-1])
    print(f, "points", d["value"], "lines", d["secondary"]["value"], "stereo", d["stereo"]["value"], "rig", d["rig"]["value"], "ingress", d.get("ingress", {}).get("value"), "parity", d["parity"]["pass"])
PY
exit $rc
