#!/bin/bash
# PMC passes for the LSD kernels (time_lsd.py), one counter group per run.
set -o pipefail
out=gpurun_out/prof_lsd_${1:-sq}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU -d $R/$out/sq -o run --output-format csv -- python3 $R/tools/time_lsd.py 256 > $R/$out/sq.log 2>&1 || { echo sq failed; tail -5 $R/$out/sq.log; exit 1; }
echo sq ok
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum -d $R/$out/tcc -o run --output-format csv -- python3 $R/tools/time_lsd.py 256 > $R/$out/tcc.log 2>&1 || { echo tcc failed; tail -5 $R/$out/tcc.log; exit 1; }
echo tcc ok
