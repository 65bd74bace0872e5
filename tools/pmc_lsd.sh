#!/bin/bash
# SQ counters of the LSD probe (tools/time_lsd.py <batch>) per env setting:
# gpurun_out/pmc_lsd_<tag>/counters.csv + a per-kernel summary.
# usage: tools/pmc_lsd.sh <batch> "<env|->" ...
set -o pipefail
B=${1:-1536}; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
PMC=${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY}
for e in "$@"; do
  tag=$(echo "$e" | tr '=/,:' '____')
  E=""; [ "$e" != "-" ] && E="$e"
  out=$R/gpurun_out/pmc_lsd_$tag; mkdir -p $out
  env $E timeout -s KILL 120 rocprofv3 --pmc $PMC -d $out -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $out/log.txt 2>&1 || { echo "pmc failed $e"; tail -3 $out/log.txt; exit 1; }
  f=$(find $out -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$e" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("orbpl::", "").replace("void ", "")
    if "lsd" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
print("==", sys.argv[2])
for k, c in acc.items():
    print("  %-28s " % k[:28] + " ".join("%s %.3g" % (n.replace("SQ_", ""), v) for n, v in sorted(c.items())))
PY
  find $out -name '*.csv' -size +2M -delete
done
