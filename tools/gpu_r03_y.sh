#!/bin/bash
# Round-3 pass y: k_lsd_sort workgroup size 512 (in-tree) vs 256 / 1024
# (variants/st*): LSD parity tests per variant, then the lines leg (3072
# streams, split LSD) per variant, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03y
mkdir -p $O
cd $R
for v in cur st256 st1024; do
  L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
  ORBPL_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v tests exit $rc: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
C="--workload lines --streams 3072 --steps 5 --warmup 2 --no-cpu-baseline --sweep 0 --isolated-steps 0 --ingress-steps 0"
for r in 1 2; do
  for v in cur st256 st1024; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 300 python bench.py $C > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "bench $v failed"; tail -5 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v r$r', d['value'], d['ms_per_step'], 'sort', d['stage_ms'].get('lsd_sort'), 'parity', d['parity']['pass'])"
  done
done
