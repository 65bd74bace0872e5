#!/bin/bash
# k_pose anatomy at 1024 streams (points tracker, TrackLocalMap on):
# stream 0's phase stamps (ORBPL_POSE_PROFILE) and SQ counters of k_pose.
#   tools/gpu_pose_probe.sh [lib]   (lib: an A/B variant's liborbpl.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pose${TAG:-}
mkdir -p $O
[ -n "$1" ] && export ORBPL_LIB=$R/$1
ORBPL_POSE_PROFILE=1 timeout -k 10 240 python3 $R/tools/probe_track.py 1024 0 1 > $O/probe.log 2>&1 || { echo "probe failed"; tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $O/a -o run --output-format csv -- python3 $R/tools/probe_track.py 1024 0 1 > $O/a.log 2>&1 || { echo "pass a failed"; tail -3 $O/a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAVES -d $O/b -o run --output-format csv -- python3 $R/tools/probe_track.py 1024 0 1 > $O/b.log 2>&1 || { echo "pass b failed"; tail -3 $O/b.log; exit 1; }
O=$O python3 - <<'PY'
import csv, collections, os
O = os.environ["O"]
for part in "ab":
    v = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{O}/{part}/run_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in v:
        if "k_pose" in k:
            print(part, k, {c: int(sum(x) / len(x)) for c, x in v[k].items()})
PY
