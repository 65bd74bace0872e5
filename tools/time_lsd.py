"""Time the GPU LSD stages on a batch of synthetic 640x480 frames (GPU box)."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from _pkg import load_pkg  # noqa: E402


def main():
    pkg = load_pkg()
    import orbpl.synth as synth
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    cfg = synth.TUM1
    room = synth.default_room(1)
    traj = synth.loop_trajectory(16, seed=1)
    frames = np.stack([synth.render(cfg, traj[i % 16], room, seed=i)[0] for i in range(16)])
    imgs = frames[np.arange(B) % 16]
    det = pkg.LineSegmentDetector(640, 480, max_batch=B)
    buf = pkg.DeviceBuffer.from_array(imgs)
    det.detect_batch_device(buf.ptr, B)
    det.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        det.detect_batch_device(buf.ptr, B)
    det.synchronize()
    dt = (time.perf_counter() - t0) / reps
    n = [len(det.lines(f)) for f in range(min(B, 8))]
    print(f"batch {B}: {dt * 1e3:.2f} ms per batch, {B / dt:.0f} frames/s, lines {n}")
    print("profile (per frame, shader cycles):", det.debug_profile())


if __name__ == "__main__":
    main()
