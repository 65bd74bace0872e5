"""The compiled C++ drop-in classes (orb_slam2_..._amd/dropin: ORBextractor,
LineExtractor, Frame, ORBmatcher, LineMatcher, Optimizer with the reference's
signatures, g++-built, linked to liborbpl.so) against the oracle: two RGB-D
frames through extraction, frame glue, the first frame's map, the second
frame's SearchByProjection (points and lines) and PoseOptimizationWithLines.
The driver binary reads / writes flat files (dropin_driver.cpp's header)."""
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

from _pkg import load_oracle, load_pkg
from _scenes import sequence

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "orb_slam2_modification_with-point-and-line-feature_amd"
DRIVER = PKG / "dropin_driver"


def _frame(buf, off, KP, KL):
    (n,) = struct.unpack_from("<i", buf, off); off += 4
    kps = np.frombuffer(buf, KP, n, off); off += n * KP.itemsize
    desc = np.frombuffer(buf, np.uint8, n * 32, off).reshape(n, 32); off += n * 32
    (nl,) = struct.unpack_from("<i", buf, off); off += 4
    kl = np.frombuffer(buf, KL, nl, off); off += nl * KL.itemsize
    ld = np.frombuffer(buf, np.uint8, nl * 32, off).reshape(nl, 32); off += nl * 32
    coef = np.frombuffer(buf, np.float64, nl * 3, off).reshape(nl, 3); off += nl * 24
    ku = np.frombuffer(buf, KP, n, off); off += n * KP.itemsize
    dep = np.frombuffer(buf, np.float32, n, off); off += n * 4
    return dict(kps=kps, desc=desc, kl=kl, ldesc=ld, coef=coef, kps_un=ku, depth=dep), off


@pytest.mark.gpu
@pytest.mark.parametrize("cam_name,seed", [("TUM1", 5), ("TUM3", 8)])
def test_dropin_classes_match_oracle(tmp_path, cam_name, seed):
    pkg = load_pkg()
    O = load_oracle()
    assert DRIVER.exists(), "build the drop-in first (make -C .../dropin)"
    cfg, traj, frames = sequence(2, seed, cam_name=cam_name)
    (g0, d0), (g1, d1) = frames
    H, W = g0.shape
    orb = (1000, 1.2, 8, 20, 7)
    T0 = np.linalg.inv(traj[0]).astype(np.float32)
    cam = O.camera(cfg)
    camv = [cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"], cfg["k1"], cfg["k2"], cfg["p1"],
            cfg["p2"], cfg["k3"], cam.bf, cam.th_depth]
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(struct.pack("<2i", W, H))
        f.write(np.asarray(camv, np.float32).tobytes())
        f.write(struct.pack("<ifiii", orb[0], orb[1], orb[2], orb[3], orb[4]))
        f.write(T0.tobytes())
        for g, d in frames:
            f.write(np.ascontiguousarray(g, np.uint8).tobytes())
            f.write(np.ascontiguousarray(d, np.float32).tobytes())
    out = tmp_path / "out.bin"
    r = subprocess.run([str(DRIVER), str(inp), str(out)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    buf = out.read_bytes()
    KP, KL = O.KP_DTYPE, O.KEYLINE_DTYPE
    F0, off = _frame(buf, 0, KP, KL)
    F1, off = _frame(buf, off, KP, KL)
    p = O.params(*orb)
    for F, (g, d) in zip((F0, F1), frames):
        okps, odesc, _ = O.extract(p, g)
        assert F["kps"].tobytes() == okps.tobytes()
        assert np.array_equal(F["desc"], odesc)
        okl, old, ocoef, _ = O.line_extract(g)
        assert F["kl"].tobytes() == okl.tobytes()
        assert np.array_equal(F["ldesc"], old) and np.array_equal(F["coef"], ocoef)
        ku, dep, _, _, _ = O.frame_prepare(cam, okps, d)
        assert F["kps_un"].tobytes() == ku.tobytes() and np.array_equal(F["depth"], dep)
    # ORBextractor::mvImagePyramid of frame 0 = the oracle's level contents
    (nlev,) = struct.unpack_from("<i", buf, off); off += 4
    opyr = O.pyramid(p, g0)
    for lv in range(nlev):
        w, h = struct.unpack_from("<2i", buf, off); off += 8
        img = np.frombuffer(buf, np.uint8, w * h, off).reshape(h, w); off += w * h
        assert np.array_equal(img, opyr[lv][19:19 + h, 19:19 + w]), lv
    nm, nlm, ninl = struct.unpack_from("<3i", buf, off); off += 12
    T1 = np.frombuffer(buf, np.float32, 16, off).reshape(4, 4); off += 64
    # the oracle's tracking loop over the same two frames (TrackWithMotionModel,
    # no local map: the driver's sequence)
    lvo = O.LVO(p, cam, 1, use_lines=True)
    lvo.reset(T0.reshape(1, 16))
    lvo.step(0, g0, d0)
    To, so = lvo.step(0, g1, d1)
    assert (nm, nlm, ninl) == (so["nmatches"], so["line_matches"], so["ninliers"])
    assert nm > 50 and nlm >= 15
    assert np.abs(T1 - To).max() < 1e-4
