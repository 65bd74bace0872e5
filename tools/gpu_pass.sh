#!/bin/bash
# One GPU pass (replaces the round-3/4 one-off lease scripts, which are in the
# git history before this file): the steps run in order, each under its own
# time limit, and the pass stops at the first failure. Outputs under
# gpurun_out/<tag>/.
#   usage: tools/gpu_pass.sh <tag> step [step ...]
#   host                host facts (CPU model, cgroup quota, affinity)
#   tests[=<expr>]      the -m gpu suite, or the -m gpu tests matching -k <expr> (commas = spaces)
#   smoke               __graft_entry__.smoke()
#   bench[=<args>]      bench.py <args> (commas become spaces), JSON in bench_<n>.json
#   prof=<MODE>         tools/prof.sh <tag> with MODE=points|lines|kitti|rig
#   faithful=<workload> tools/cpu_faithful.py <workload> (no GPU): the reference-
#                       faithful CPU loop, JSON appended to faithful.jsonl
#   env=<NAME=VALUE>    exported for the steps after it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
tag=$1; shift
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}; arg=""; [ "$step" != "$name" ] && arg=${step#*=}
  case $name in
    host)
      { nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket|NUMA"; cat /sys/fs/cgroup/cpu.max 2>/dev/null;
        python3 -c "import os; print('affinity', sorted(os.sched_getaffinity(0)))"; } > $O/host.txt 2>&1
      echo "host: $(grep 'Model name' $O/host.txt | head -1)" ;;
    tests)
      K=(); [ -n "$arg" ] && K=(-k "${arg//,/ }")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/gpu_tests_$n.log 2>&1
      rc=$?; echo "tests($arg) exit $rc: $(tail -1 $O/gpu_tests_$n.log)"
      if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/gpu_tests_$n.log | head -20; exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 1000 python -u bench.py --detail gpurun_out/$tag/bench_detail_$n.json ${arg//,/ } > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench failed"; tail -20 $O/bench_$n.err; exit 1; }
      tail -c 400 $O/bench_$n.json ;;
    prof)
      MODE=$arg bash tools/prof.sh ${tag}_$arg || exit 1 ;;
    faithful)
      timeout -k 10 600 python -u tools/cpu_faithful.py ${arg:-lines} 300 6 >> $O/faithful.jsonl 2> $O/faithful_$n.err || { echo "faithful failed"; tail -5 $O/faithful_$n.err; exit 1; }
      tail -1 $O/faithful.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('faithful', d['workload'], d['median_ms_per_frame'], d.get('stage_median_ms'), d['affinity'].get('pinned'))" ;;
    env)
      export "$arg"; echo "env $arg" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
