"""bench.cpu_reference_faithful runs the oracle's one-stream loop in a child
process of its own (tools/cpu_faithful.py --npz): the frames the stream reads,
its start pose and the bench vocabulary travel through the file, and the
child's JSON line comes back (CPU only, no GPU call)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def test_faithful_child_process():
    import bench
    from _pkg import load_oracle, load_pkg
    load_pkg()
    import orbpl.synth as synth
    from _vocab import training_descriptors
    g, dep = bench.render_loop(4, seed=1, workers=4, cam_name="TUM1")
    lay = bench.Layout(synth.loop_trajectory(4, seed=1), 1)
    t = synth.vocabulary_tree(training_descriptors(2), k=10, L=3, seed=3)
    old = bench.VOCAB["arrays"]
    bench.VOCAB["arrays"] = dict(parent=t["parent"], leaf=t["leaf"], desc=t["desc"],
                                 weight=t["weight"], k=10, L=3, scoring=0, weighting=0)
    try:
        O = load_oracle()
        r = bench.cpu_reference_faithful(g, dep, lay, "points", O.TRACK_LOCAL_MAP | O.TRACK_REFKF,
                                         2, 5, True)
    finally:
        bench.VOCAB["arrays"] = old
    assert r["frames"] == 5 and r["threads_per_frame"] == 1
    assert r["median_ms_per_frame"] > 0 and np.isfinite(r["mean_ms_per_frame"])
    assert "process of its own" in r["sample"]
