"""Build and run tools/lsd_stream_sim.cpp (CPU model of a round-free
speculative LSD seed loop) over frames of the lines workload.
usage: python tools/lsd_stream_sim.py [frames] [window] [fit_batch]"""
import ctypes
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
OUT = Path("/tmp/lsd_stream_sim")


def build():
    OUT.mkdir(exist_ok=True)
    so = OUT / "libsim.so"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-shared",
                           "-o", str(so), str(ROOT / "tools" / "lsd_stream_sim.cpp"),
                           str(ROOT / "oracle" / "orb_oracle.cpp"), f"-I{ROOT}/oracle", "-lm"])
    return ctypes.CDLL(str(so))


KEYS = ("same", "ref_cands", "cands", "regions", "iters", "grow_iters", "fits", "fit_batches",
        "commits", "regrows", "conflicts", "fetched", "skipped_at_head", "cycles", "round_cycles",
        "stalls")


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    windows = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "256").split(",")]
    fbs = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "8").split(",")]
    L = build()
    sys.path.insert(0, str(ROOT))
    import bench
    g, _ = bench.render_loop(max(nf, 2), 7, 4, cam_name="TUM3")
    out = np.zeros(16, np.float64)
    o4 = np.zeros(4, np.float64)
    for f, window, fb in [(f, w, b) for f in range(nf) for w in windows for b in fbs]:
        img = np.ascontiguousarray(g[f])
        L.lsd_stream_sim(img.ctypes.data_as(ctypes.c_void_p), img.shape[1], img.shape[0], window, fb,
                         out.ctypes.data_as(ctypes.c_void_p), o4.ctypes.data_as(ctypes.c_void_p))
        d = dict(zip(KEYS, out.tolist()))
        print(f"frame {f} window {window} fit_batch {fb}: " +
              " ".join(f"{k}={v:.0f}" for k, v in d.items()) +
              f"  stream/round = {d['cycles'] / d['round_cycles']:.3f}  grow/fit/commit M = "
              f"{o4[0] / 1e6:.1f}/{o4[1] / 1e6:.1f}/{o4[2] / 1e6:.1f}", flush=True)


if __name__ == "__main__":
    main()
