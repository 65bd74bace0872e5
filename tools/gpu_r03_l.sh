#!/bin/bash
# Round-3 pass l: split LSD chain (two offset halves on two streams): the
# lines tracker parity tests (incl. the forced split case and the 1024-stream
# bench parity), then the lines leg at 3072 streams with ORBPL_LSD_SPLIT 0 / 1
# alternating, then a kernel trace of the split run.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03l
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_track.py -k "lines_matches_oracle_lvo" tests/test_gpu_multi.py::test_bench_lines_1024_streams_parity -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "assert|Error" $O/tests.log | head -20; exit $rc; }
B="--workload lines --streams 3072 --steps 5 --warmup 2 --no-cpu-baseline --sweep 0 --isolated-steps 0 --ingress-steps 0"
for r in 1 2; do
  for sp in 0 1; do
    ORBPL_LSD_SPLIT=$sp timeout -k 10 300 python bench.py $B > $O/b_${sp}_$r.json 2> $O/b_${sp}_$r.err || { echo "bench $sp failed"; tail -5 $O/b_${sp}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/b_${sp}_$r.json').read().strip().splitlines()[-1]); print('split $sp round $r', d['value'], d['ms_per_step'], 'parity', d['parity']['pass'])"
  done
done
cd /tmp && export TMPDIR=/tmp
ORBPL_LSD_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/bench.py --workload lines --streams 3072 --steps 4 --warmup 2 --no-cpu-baseline --sweep 0 --isolated-steps 0 --ingress-steps 0 --no-parity > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
find $O/trace -name '*kernel_trace.csv' -exec cp {} $O/kernel_trace.csv \;
echo done
