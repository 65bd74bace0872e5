#!/bin/bash
# One PMC pass (SQ counters) over the extraction probe: per-kernel VALU/LDS
# instruction counts and wave cycles under gpurun_out/pmc_<tag>/.
set -o pipefail
tag=${1:-run}
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
PMC=${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM}
B=${B:-256}
timeout -s KILL 90 rocprofv3 --pmc $PMC -d $out -o run --output-format csv -- python3 $R/tools/probe_extract.py $B > $out/log.txt 2>&1 || { echo "pmc failed"; tail -5 $out/log.txt; exit 1; }
find $out -name '*counter_collection.csv' -exec cp {} $out/counters.csv \;
echo pmc ok
