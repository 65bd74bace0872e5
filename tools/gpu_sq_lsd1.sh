#!/bin/bash
# SQ counters of the LSD kernels at batch 1 (seed loop latency anatomy)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $R/gpurun_out/sq1/a -o run --output-format csv -- python3 $R/tools/time_lsd.py 1 > $R/gpurun_out/sq1/a.log 2>&1 || { echo "pass a failed"; tail -3 $R/gpurun_out/sq1/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAVES -d $R/gpurun_out/sq1/b -o run --output-format csv -- python3 $R/tools/time_lsd.py 1 > $R/gpurun_out/sq1/b.log 2>&1 || { echo "pass b failed"; tail -3 $R/gpurun_out/sq1/b.log; exit 1; }
python3 - <<'PY'
import csv, collections, os
R = os.environ["GRAFT_REPO_ROOT"]
for part in "ab":
    v = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{R}/gpurun_out/sq1/{part}/run_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in v:
        if "lsd_spec" in k:
            print(part, k, {c: int(sum(x) / len(x)) for c, x in v[k].items()})
PY
