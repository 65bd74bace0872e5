#!/bin/bash
# Profiling passes on the GPU box (rocprofv3). Kernel trace + stats first,
# then PMC passes, each counter group in its own run (no tracing domains
# combined with --pmc). Outputs under gpurun_out/prof_<tag>/.
set -o pipefail
tag=${1:-run}
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
# points headline (256 streams) by default; MODE=lines profiles configs[2]
if [ "$MODE" = "lines" ]; then
  B="$R/bench.py --workload lines --streams 1536 --steps 3 --warmup 1 --ate-streams 0 --no-cpu-baseline"
else
  B="$R/bench.py --steps 20 --warmup 5 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ate-streams 0 --no-cpu-baseline"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- python3 $B > $R/$out/trace.log 2>&1 || { echo "trace failed"; tail -5 $R/$out/trace.log; exit 1; }
echo trace ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/$out/fetch -o run --output-format csv -- python3 $B > $R/$out/fetch.log 2>&1 || { echo "fetch failed"; tail -5 $R/$out/fetch.log; exit 1; }
echo fetch ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/$out/write -o run --output-format csv -- python3 $B > $R/$out/write.log 2>&1 || { echo "write failed"; tail -5 $R/$out/write.log; exit 1; }
echo write ok
if [ -n "$SQ" ]; then
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT -d $R/$out/sq -o run --output-format csv -- python3 $B > $R/$out/sq.log 2>&1 || { echo "sq failed"; tail -5 $R/$out/sq.log; exit 1; }
echo sq ok
fi
