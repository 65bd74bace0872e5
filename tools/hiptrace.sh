#!/bin/bash
# HIP API + kernel trace of a short bench run (no PMC): host calls that block
# (long API durations) and the kernel timeline, under gpurun_out/hiptrace_<tag>/.
set -o pipefail
tag=${1:-run}; shift
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/hiptrace_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $out -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-parity --sweep 0 --ingress-steps 0 --isolated-steps 0 "$@" > $out/trace.log 2>&1 || { echo "trace failed"; tail -5 $out/trace.log; exit 1; }
python3 - "$out" <<'PY'
import csv, glob, sys
out = sys.argv[1]
f = glob.glob(out + "/**/*hip_api_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
with open(out + "/slow_api.txt", "w") as o:
    for r in rows[:60]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        o.write(f"{d:10.3f} ms  {r['Function']:32s} start {int(r['Start_Timestamp'])/1e6:.3f}\n")
PY
find $out -name '*.csv' -size +3M -delete
echo hiptrace ok
