#!/bin/bash
# SQ counters for the LSD kernels (time_lsd.py), one PMC pass.
set -o pipefail
out=gpurun_out/prof_lsd_sq
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/$out -o run --output-format csv -- python3 $R/tools/time_lsd.py 256 > $R/$out/log 2>&1 || { echo failed; tail -5 $R/$out/log; exit 1; }
echo ok
