#!/bin/bash
# Round-3 pass j: fit phase anatomy (ORBPL_FIT_PROF variant, frame 0) at batch
# 1 / 3072, and SQ issue counters of the seed loop at 3072 frames.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03j
mkdir -p $O
cd $R
for b in 1 3072; do
  ORBPL_LIB=variants/fitprof/liborbpl.so timeout -k 10 120 python tools/time_lsd.py $b > $O/fitprof_$b.log 2>&1 || { echo "fitprof $b failed"; tail -3 $O/fitprof_$b.log; exit 1; }
  echo "batch $b: $(grep -m1 '^batch' $O/fitprof_$b.log)"; grep fitprof $O/fitprof_$b.log | tail -2
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES -d $O/sq -o run --output-format csv -- python3 $R/tools/time_lsd.py 3072 > $O/sq.log 2>&1 || { echo "sq failed"; tail -3 $O/sq.log; exit 1; }
python3 $R/tools/pmc_summary.py $(find $O/sq -name '*counter_collection.csv' | head -1) lsd
