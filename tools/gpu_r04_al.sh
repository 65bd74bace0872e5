#!/bin/bash
# Round-4 pass al: VALU lane utilisation of the LSD kernels at 1 / 1536 frames
# on the session-2 build (100 x SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64)).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04al
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && export GPU_MAX_HW_QUEUES=16
for B in 1 1536; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES -d $O/lane_$B -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $O/lane_$B.log 2>&1 || { echo "lane $B failed"; tail -5 $O/lane_$B.log; exit 1; }
done
python3 - <<PY
import csv, collections
for B in (1, 1536):
    c = collections.defaultdict(lambda: collections.defaultdict(float))
    for x in csv.DictReader(open(f"$O/lane_{B}/run_counter_collection.csv")):
        c[x["Kernel_Name"].split("(")[0].replace("void ", "")][x["Counter_Name"]] += float(x["Counter_Value"])
    for k, v in c.items():
        if "lsd" in k and v["SQ_ACTIVE_INST_VALU"] > 0:
            print(f"lane util B={B} {k[:40]:40s} {100 * v['SQ_THREAD_CYCLES_VALU'] / (v['SQ_ACTIVE_INST_VALU'] * 64):6.1f} %  valu {v['SQ_INSTS_VALU']:.3g} waves {v['SQ_WAVES']:.0f}")
PY
