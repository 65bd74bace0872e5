#!/bin/bash
# Round-4 pass g: where the batch-1 lines step goes - kernel trace of the LSD
# detector alone (1 and 16 frames) and of the lines tracker at 1 stream.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_lsd.py -x -q --timeout 200 --timeout-method thread > $O/lsd_tests.log 2>&1 || { tail -30 $O/lsd_tests.log; exit 1; }
tail -1 $O/lsd_tests.log
for B in 1 16; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/lsd_$B -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $O/lsd_$B.log 2>&1 || { echo "lsd $B failed"; tail -5 $O/lsd_$B.log; exit 1; }
  head -2 $O/lsd_$B.log
done
COMMON="--no-cpu-baseline --no-parity --sweep 0 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --isolated-steps 0 --ingress-steps 0 --trk-load 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lines_1 -o run --output-format csv -- python3 $R/bench.py --workload lines --streams 1 --steps 10 --warmup 3 $COMMON > $O/lines_1.json 2> $O/lines_1.err || { echo "lines 1 failed"; tail -5 $O/lines_1.err; exit 1; }
# k_lsd_validate traffic at 1536 frames: frames of one XCD together (cur) or not (valnox)
for v in cur valnox; do
  L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
  for c in FETCH_SIZE WRITE_SIZE; do
    ORBPL_LIB=$L timeout -s KILL 180 rocprofv3 --pmc $c -d $O/val_${v}_$c -o run --output-format csv -- python3 $R/tools/time_lsd.py 1536 > $O/val_${v}_$c.log 2>&1 || { echo "val $v $c failed"; tail -5 $O/val_${v}_$c.log; exit 1; }
  done
  head -1 $O/val_${v}_FETCH_SIZE.log
done
# VALU lane utilisation of the LSD kernels (thread-cycles / (active VALU cycles x 64))
for B in 1 1536; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES -d $O/lane_$B -o run --output-format csv -- python3 $R/tools/time_lsd.py $B > $O/lane_$B.log 2>&1 || { echo "lane $B failed"; tail -5 $O/lane_$B.log; exit 1; }
done
python3 - <<'PY'
import csv, collections, os, glob
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r04g"
for d in ("lsd_1", "lsd_16", "lines_1"):
    fs = glob.glob(f"{O}/{d}/**/run_kernel_stats.csv", recursive=True)
    if not fs:
        print(d, "no stats"); continue
    rows = list(csv.DictReader(open(fs[0])))
    print("==", d)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e6:8.3f} ms max {float(r["MaxNs"])/1e6:8.3f}')
for v in ("cur", "valnox"):
    tot = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        fs = glob.glob(f"{O}/val_{v}_{c}/**/run_counter_collection.csv", recursive=True)
        if not fs:
            continue
        acc = collections.defaultdict(float); disp = collections.defaultdict(set)
        for r in csv.DictReader(open(fs[0])):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[k] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
        for k in acc:
            if "k_lsd_validate" in k:
                tot[c] = acc[k] / len(disp[k]) * 1024 * (2 if c == "FETCH_SIZE" else 1)
    if tot:
        print(f"validate {v}: fetch x2 {tot.get('FETCH_SIZE', 0) / 1536 / 1e6:.2f} MB/frame, write {tot.get('WRITE_SIZE', 0) / 1536 / 1e6:.3f} MB/frame")
for B in (1, 1536):
    fs = glob.glob(f"{O}/lane_{B}/**/run_counter_collection.csv", recursive=True)
    if not fs:
        print("lane", B, "no counters"); continue
    v = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        v[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in v.items():
        if "lsd" in k and c.get("SQ_ACTIVE_INST_VALU"):
            print(f"lane util B={B} {k[:40]:40s} {100 * c['SQ_THREAD_CYCLES_VALU'] / (c['SQ_ACTIVE_INST_VALU'] * 64):6.1f} %  "
                  f"valu {c['SQ_INSTS_VALU']:.3g} waves {c['SQ_WAVES']:.0f}")
PY

# headline A/B: k_match_local descriptors in LDS (cur) or from global memory (locglob)
cd $R
A="--steps 20 --warmup 5 --secondary-steps 0 --stereo-steps 0 --rig-steps 0 --ingress-steps 0 --no-cpu-baseline --sweep 0 --trk-load 0 --isolated-steps 3 --no-parity"
for r in 1 2; do
  for v in cur locglob; do
    L=""; [ "$v" != cur ] && L=$R/variants/$v/liborbpl.so
    ORBPL_LIB=$L timeout -k 10 300 python bench.py $A > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "fail $v"; tail -3 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); st=d['roofline']['isolated']['stage_ms']; print('$r $v', d['value'], d['ms_per_step'], 'isolated match_local', st.get('match_local'), 'local_map', st.get('local_map'), 'match', st.get('match'))"
  done
done

exit 0
