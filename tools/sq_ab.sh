#!/bin/bash
# SQ counters of the headline bench (short, no pipeline) for library variants:
# tools/sq_ab.sh <variant|cur> ... -> gpurun_out/sq_<variant>/
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16 ORBPL_LEVEL_PIPE=0
B="$R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --isolated-steps 0 --ingress-steps 0"
for v in "$@"; do
  L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
  out=$R/gpurun_out/sq_$v; mkdir -p $out
  ORBPL_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $out -o run --output-format csv -- python3 $B > $out/log.txt 2>&1 || { echo "sq failed $v"; tail -3 $out/log.txt; exit 1; }
  echo "sq ok $v"
done
