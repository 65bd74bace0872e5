"""CPU tests of the host-side I/O and trajectory evaluator (orbpl.tum):
settings, associations, SaveTrajectoryTUM format, quaternions, ATE."""
import os

import numpy as np
import pytest

from _pkg import load_pkg

load_pkg()
import orbpl.tum as tum  # noqa: E402

REF = "/root/reference"


def _rot(axis, ang):
    a = np.asarray(axis, np.float64)
    a /= np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


@pytest.mark.parametrize("axis,ang", [((0, 0, 1), 0.3), ((1, 2, 3), 2.0), ((1, 0, 0), np.pi),
                                      ((0, 1, 0), 3.1), ((1, 1, 0), -2.9), ((0, 0, 1), 0.0)])
def test_quaternion_round_trip(axis, ang):
    R = _rot(axis, ang)
    q = tum.quaternion_from_matrix(R)
    assert abs(np.linalg.norm(q) - 1) < 1e-12
    assert np.allclose(tum.matrix_from_quaternion(q), R, atol=1e-12)


def test_save_load_trajectory(tmp_path):
    rng = np.random.default_rng(0)
    n = 20
    Twc = np.tile(np.eye(4), (n, 1, 1))
    for i in range(n):
        Twc[i, :3, :3] = _rot(rng.normal(size=3), rng.uniform(-3, 3))
        Twc[i, :3, 3] = rng.normal(size=3)
    Tcw = np.linalg.inv(Twc).astype(np.float32)
    ts = 1305031910.765238 + 0.033 * np.arange(n)
    lost = np.zeros(n, bool)
    lost[5] = True
    p = tmp_path / "CameraTrajectory.txt"
    tum.save_trajectory_tum(p, ts, Tcw, lost)
    lines = open(p).read().splitlines()
    assert len(lines) == n - 1
    tok = lines[0].split()
    assert len(tok) == 8 and tok[0] == "1305031910.765238"
    assert all(len(x.split(".")[1]) == 9 for x in tok[1:])
    t2, Twc2 = tum.load_trajectory_tum(p)
    keep = ~lost
    assert np.allclose(t2, ts[keep], atol=1e-6)
    assert np.allclose(Twc2[:, :3, 3], Twc[keep, :3, 3], atol=1e-5)
    assert np.allclose(Twc2[:, :3, :3], Twc[keep, :3, :3], atol=1e-5)
    tum.save_keyframe_trajectory_tum(tmp_path / "kf.txt", ts, Tcw)
    assert all(len(x.split(".")[1]) == 7 for x in open(tmp_path / "kf.txt").readline().split()[1:])


def test_load_settings_opencv_yaml(tmp_path):
    p = tmp_path / "cam.yaml"
    p.write_text("%YAML:1.0\n\n# comment\nCamera.fx: 517.3\nCamera.fy: 516.5\nCamera.cx: 318.6\n"
                 "Camera.cy: 255.3\nCamera.k1: 0.26\nCamera.width: 640\nCamera.height: 480\n"
                 "Camera.bf: 40.0\nThDepth: 40.0\nDepthMapFactor: 5000.0\n"
                 "ORBextractor.nFeatures: 1000\nORBextractor.scaleFactor: 1.2\n"
                 "ORBextractor.nLevels: 8\nORBextractor.iniThFAST: 20\n"
                 "ORBextractor.minThFAST: 7\nViewer.PointSize:2\n")
    raw, cam, orb, dmf = tum.load_settings(p)
    assert cam["fx"] == 517.3 and cam["k1"] == 0.26 and cam["k2"] == 0.0
    assert orb == (1000, 1.2, 8, 20, 7)
    assert raw["Viewer.PointSize"] == 2
    assert dmf == np.float32(1) / np.float32(5000)
    d = tum.depth_to_metres(np.array([[5000, 0, 12345]], np.uint16), dmf)
    assert d.dtype == np.float32 and d[0, 1] == 0 and abs(d[0, 0] - 1) < 1e-6


def test_associations(tmp_path):
    p = tmp_path / "assoc.txt"
    p.write_text("1.0 rgb/1.png 1.01 depth/1.png 1.005 0 0 0 0 0 0 1\n\n"
                 "2.0 rgb/2.png 2.01 depth/2.png 2.005 1 0 0 0 0 0 1\n")
    a = tum.load_associations(p)
    assert a["rgb"] == ["rgb/1.png", "rgb/2.png"] and a["depth"][1] == "depth/2.png"
    assert a["gt"].shape == (2, 8) and a["gt"][1, 1] == 1.0
    assert tum.associate([1.0, 2.0, 3.0], [2.01, 0.995, 5.0]) == [(0, 1), (1, 0)]


def test_ate_alignment():
    rng = np.random.default_rng(1)
    gt = rng.normal(size=(100, 3))
    R = _rot((1, 2, 0.5), 0.7)
    est = (gt - [1, 2, 3]) @ R.T
    assert tum.ate(est, gt)["rmse"] < 1e-12
    assert abs(tum.ate(gt + [0.1, 0, 0], gt, aligned=False)["rmse"] - 0.1) < 1e-12
    Tcw = np.tile(np.eye(4), (2, 1, 1))
    Tcw[1, :3, 3] = [1, 0, 0]
    assert np.allclose(tum.camera_centres(Tcw), [[0, 0, 0], [-1, 0, 0]])


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_ate_of_the_reference_result():
    """the reference's own fr1_room trajectory against the
    ground-truth columns of its association file (read in place)."""
    t, Twc = tum.load_trajectory_tum(f"{REF}/results/CameraTrajectory.txt")
    a = tum.load_associations(f"{REF}/Examples/RGB-D/associate_with_groundtruth.txt")
    assert np.array_equal(t, a["t_rgb"])
    r = tum.ate(Twc[:, :3, 3], tum.poses_from_rows(a["gt"])[:, :3, 3])
    assert r["n"] == 1352
    assert round(r["rmse"], 4) == 0.0540 and round(r["mean"], 4) == 0.0454
    assert round(r["median"], 4) == 0.0367 and round(r["max"], 4) == 0.1782


TUM1_TEXT = ("%YAML:1.0\n\n# Camera calibration and distortion parameters (OpenCV)\n"
             "Camera.fx: 517.306408\nCamera.fy: 516.469215\nCamera.cx: 318.643040\n"
             "Camera.cy: 255.313989\n\nCamera.k1: 0.262383\nCamera.k2: -0.953104\n"
             "Camera.p1: -0.005358\nCamera.p2: 0.002628\nCamera.k3: 1.163314\n\n"
             "Camera.width: 640\nCamera.height: 480\n\n# Camera frames per second \n"
             "Camera.fps: 30.0\n\nCamera.bf: 40.0\nCamera.RGB: 1\nThDepth: 40.0\n"
             "DepthMapFactor: 5000.0\n\nORBextractor.nFeatures: 1000\n"
             "ORBextractor.scaleFactor: 1.2\nORBextractor.nLevels: 8\n"
             "ORBextractor.iniThFAST: 20\nORBextractor.minThFAST: 7\n"
             "Viewer.KeyFrameSize: 0.05\nViewer.PointSize:2\n")


def test_native_settings_loader(tmp_path, orbpl):
    """orbpl_settings_load (the C++ reader of Tracking.cc:53-147) on the
    reference's TUM1.yaml content (Examples/RGB-D/TUM1.yaml): every field as
    Tracking::Tracking reads it, equal to the Python reader's camera; a
    settings file without fps / ThDepth / DepthMapFactor takes the
    reference's fallbacks (fps 30, depth factor 1)."""
    p = tmp_path / "TUM1.yaml"
    p.write_text(TUM1_TEXT)
    orb, cam, extra = orbpl.load_settings(p, "rgbd")
    _, pc, porb, pdmf = tum.load_settings(p)
    ref = orbpl.make_camera(pc)
    for f, _ in orbpl.Camera._fields_:
        assert getattr(cam, f) == getattr(ref, f), f
    assert (orb.nfeatures, orb.nlevels, orb.ini_th_fast, orb.min_th_fast) == (1000, 8, 20, 7)
    assert orb.scale_factor == np.float32(1.2)
    assert extra["fps"] == 30.0 and extra["max_frames"] == 30 and extra["rgb"] == 1
    assert np.float32(extra["depth_map_factor"]) == pdmf
    assert extra["depth_map_factor_setting"] == 5000.0
    # stereo: no depth factor; monocular: no depth threshold
    _, cs, es = orbpl.load_settings(p, "stereo")
    assert es["depth_map_factor"] == 1.0 and cs.th_depth == ref.th_depth
    _, cm, _ = orbpl.load_settings(p, "monocular")
    assert cm.th_depth == 0.0
    q = tmp_path / "bare.yaml"
    q.write_text("%YAML:1.0\nCamera.fx: 700\nCamera.bf: 350.0\nORBextractor.nFeatures: 2000.4\n")
    orb2, cam2, e2 = orbpl.load_settings(q, "rgbd")
    assert e2["fps"] == 30.0 and e2["max_frames"] == 30 and e2["depth_map_factor"] == 1.0
    assert orb2.nfeatures == 2000 and cam2.th_depth == 0.0 and cam2.k1 == 0.0
    import pytest
    with pytest.raises(orbpl.OrbplError):
        orbpl.load_settings(tmp_path / "missing.yaml")
