"""ASan + UBSan build of the CPU oracle (SURVEY.md §5 "sanitizers"): the
driver oracle/sanitize_main.cpp pushes a short synthetic RGB-D sequence and a
stereo pair sequence through ORB, LSD/LBD, the points+lines VO loop (plain,
with the local map, with the analytic line Jacobian) and the stereo
points+lines loop. Any out-of-bounds access, leak or undefined arithmetic in
the checker aborts the run."""
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def test_oracle_under_asan_ubsan(tmp_path):
    from _pkg import load_pkg
    load_pkg()
    import orbpl.synth as synth
    from _scenes import stereo_sequence
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "sanitize"], check=True, timeout=600)
    cfg = dict(synth.TUM1)
    W, H, F = cfg["width"], cfg["height"], 3
    traj = synth.trajectory(F, seed=71)
    room = synth.default_room(71)
    frames = [synth.render(cfg, T, room, seed=710 + i) for i, T in enumerate(traj)]
    # a rectified pair sequence of the same size (right camera at +mb)
    shift = np.eye(4)
    shift[0, 3] = cfg["bf"] / cfg["fx"]
    rights = [synth.render(cfg, T @ shift, room, seed=710 + i)[0] for i, T in enumerate(traj)]
    f = tmp_path / "frames.bin"
    with open(f, "wb") as fh:
        fh.write(np.array([W, H, F], np.int32).tobytes())
        for g, _ in frames:
            fh.write(np.ascontiguousarray(g, np.uint8).tobytes())
        for _, d in frames:
            fh.write(np.ascontiguousarray(d, np.float32).tobytes())
        for r in rights:
            fh.write(np.ascontiguousarray(r, np.uint8).tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(ROOT / "oracle" / "_build" / "oracle_sanitize"), str(f)], env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitize ok" in r.stdout
    assert "runtime error" not in r.stderr
