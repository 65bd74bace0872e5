#!/bin/bash
# Round-4 pass f: headline A/B (points, 1024 streams, 20 steps): the current
# build vs k_match_last with the frame's descriptors read from global memory
# (smaller LDS, placed sooner beside the next batch's extraction) vs the
# FAST score on two-input packed u16 ops (fastold) vs the pyramid with three
# barriers per level (pyrold), 2 rounds; ORB parity of the current build first.
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 200 --timeout-method thread > $O/orb_tests.log 2>&1 || { tail -30 $O/orb_tests.log; exit 1; }
tail -1 $O/orb_tests.log
A="--steps 20 --warmup 5 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --no-cpu-baseline --sweep 0 --trk-load 0 --isolated-steps 3 --no-parity"
for r in 1 2; do
  for v in cur mdg fastold pyrold; do
    L=""; [ "$v" != cur ] && L=variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 300 python bench.py $A > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "fail $v"; tail -3 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); st=d['roofline']['isolated']['stage_ms']; ex=sum(st[k] for k in ('pyramid','fast','octree','orient_desc')); print('$r $v', d['value'], d['ms_per_step'], 'isolated: extraction %.3f' % ex, 'pyr', st.get('pyramid'), 'fast', st.get('fast'), 'oct', st.get('octree'), 'desc', st.get('orient_desc'), 'match', st.get('match'))"
  done
done
exit 0
