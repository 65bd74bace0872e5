"""The bench's reference-faithful CPU timing in a process of its own (no GPU
work).
  python tools/cpu_faithful.py --npz <file>: the child of
      bench.cpu_reference_faithful (frames, vocabulary and settings from the
      file), prints one JSON line;
  python tools/cpu_faithful.py [workload] [frames] [vocab_levels]: the same
      measurement standalone on the bench's synthetic loop and vocabulary
      (one JSON line: latency, per-thread stage times, the CPUs used)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import bench  # noqa: E402
from _pkg import load_oracle, load_pkg  # noqa: E402


def main():
    import json
    if len(sys.argv) >= 3 and sys.argv[1] == "--npz":
        load_pkg()
        print(json.dumps(bench.faithful_run(sys.argv[2], pin="--no-pin" not in sys.argv)))
        return
    wname = sys.argv[1] if len(sys.argv) > 1 else "lines"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    load_pkg()
    import orbpl.synth as synth
    from _vocab import training_descriptors
    O = load_oracle()
    wl = bench.WORKLOADS[wname]
    g, dep = bench.render_loop(32, seed=1, workers=16, cam_name=wl["cam"])
    lay = bench.Layout(synth.loop_trajectory(32, seed=1), 1)
    if L > 0:
        t = synth.vocabulary_tree(training_descriptors(8), k=10, L=L, seed=3)
        bench.VOCAB["arrays"] = dict(parent=t["parent"], leaf=t["leaf"], desc=t["desc"],
                                     weight=t["weight"], k=10, L=L, scoring=0, weighting=0)
    # the bench's reference-faithful leg: the map model, TrackLocalMap +
    # TrackReferenceKeyFrame, 20 warm-up frames, a child process of its own
    r = bench.cpu_reference_faithful(g, dep, lay, wname, O.TRACK_LOCAL_MAP | O.TRACK_REFKF,
                                     20, frames, True)
    r["workload"] = wname
    r["vocab_levels"] = L
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
