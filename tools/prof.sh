#!/bin/bash
# Profiling passes on the GPU box (rocprofv3). Kernel trace + stats first,
# then PMC passes, each counter group in its own run (no tracing domains
# combined with --pmc). Outputs under gpurun_out/prof_<tag>/.
#   MODE=points (default): the headline configs[1] leg of the default bench
#   MODE=lines: configs[2] at 4096 streams;  MODE=kitti: configs[3] at 3072
#   MODE=rig: configs[4] at 512 cameras
#   SQ=1 adds an SQ counter pass (VALU / wait / LDS instruction counts)
set -o pipefail
tag=${1:-run}
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
# the bench's hardware queue count, set before rocprofv3 starts the runtime
export GPU_MAX_HW_QUEUES=16
R=$GRAFT_REPO_ROOT
COMMON="--detail gpurun_out/prof_$tag/bench_detail.json --no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --isolated-steps 0 --ingress-steps 0"
case "$MODE" in
  lines) B="$R/bench.py --workload lines --streams 4096 --steps 3 --warmup 1 $COMMON" ;;
  kitti) B="$R/bench.py --workload kitti --streams 3072 --steps 3 --warmup 1 $COMMON" ;;
  rig)   B="$R/bench.py --workload rig --streams 512 --steps 3 --warmup 1 $COMMON" ;;
  *)     B="$R/bench.py --steps 20 --warmup 5 $COMMON" ;;
esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- python3 $B > $R/$out/trace.log 2>&1 || { echo "trace failed"; tail -5 $R/$out/trace.log; exit 1; }
echo trace ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/$out/fetch -o run --output-format csv -- python3 $B > $R/$out/fetch.log 2>&1 || { echo "fetch failed"; tail -5 $R/$out/fetch.log; exit 1; }
echo fetch ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/$out/write -o run --output-format csv -- python3 $B > $R/$out/write.log 2>&1 || { echo "write failed"; tail -5 $R/$out/write.log; exit 1; }
echo write ok
if [ -n "$SQ" ]; then
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES -d $R/$out/sq -o run --output-format csv -- python3 $B > $R/$out/sq.log 2>&1 || { echo "sq failed"; tail -5 $R/$out/sq.log; exit 1; }
echo sq ok
fi
if [ -n "$SQ2" ]; then
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD -d $R/$out/sq2 -o run --output-format csv -- python3 $B > $R/$out/sq2.log 2>&1 || { echo "sq2 failed"; tail -5 $R/$out/sq2.log; exit 1; }
echo sq2 ok
fi
