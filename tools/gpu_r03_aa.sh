#!/bin/bash
# Round-3 pass aa: the one-wave seed loop's register bound (ORBPL_SPEC_MINW 4
# in-tree vs 3 / 2) on the lines leg (3072 streams, split LSD), two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03aa
mkdir -p $O
cd $R
for v in minw3 minw2; do
  ORBPL_LIB=$R/variants/$v/liborbpl.so timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v tests exit $rc: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
C="--workload lines --streams 3072 --steps 5 --warmup 2 --no-cpu-baseline --sweep 0 --isolated-steps 0 --ingress-steps 0"
for r in 1 2; do
  for v in cur minw3 minw2; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 300 python bench.py $C > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench $v failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v r$r', d['value'], d['ms_per_step'], 'seed', d['stage_ms'].get('lsd_seed'), 'parity', d['parity']['pass'])"
  done
done
