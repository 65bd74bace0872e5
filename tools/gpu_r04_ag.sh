#!/bin/bash
# Round-4 pass ag: instruction-cache hits / misses of the LSD kernels at batch
# 1 (the seed loop's kernel is ~170 KB of code per instance).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && export GPU_MAX_HW_QUEUES=16
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $O/ic -o run --output-format csv -- python3 $R/tools/time_lsd.py 1 > $O/ic.log 2>&1 || { echo "ic failed"; tail -8 $O/ic.log; exit 1; }
python3 - <<PY
import csv, collections
r = collections.defaultdict(lambda: collections.defaultdict(float))
for x in csv.DictReader(open('$O/ic/run_counter_collection.csv')):
    r[x['Kernel_Name'].split('(')[0]][x['Counter_Name']] += float(x['Counter_Value'])
for k, v in r.items():
    print(k[:50], dict(v))
PY
