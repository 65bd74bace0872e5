"""CPU tests of the Frame::ComputeStereoMatches oracle (Frame.cc:886-1063)
on a rendered rectified stereo pair (tests/_scenes.stereo_pair)."""
import numpy as np

from _scenes import stereo_pair


def _run(oracle, seed):
    cfg, left, right = stereo_pair(seed)
    p = oracle.params(2000, 1.2, 8, 20, 7)
    kl, dl, _ = oracle.extract(p, left)
    kr, dr, _ = oracle.extract(p, right)
    ur, d = oracle.stereo_matches(oracle.camera(cfg), p, left, right, kl, dl, kr, dr)
    return cfg, kl, ur, d


def test_stereo_depths_follow_the_scene(oracle):
    from _pkg import load_pkg
    load_pkg()
    import orbpl.synth as synth
    cfg, kl, ur, d = _run(oracle, 0)
    m = d > 0
    assert m.sum() > 0.3 * len(kl)
    # unmatched keypoints carry -1 in both outputs
    assert np.all(ur[~m] == -1) and np.all(d[~m] == -1)
    # depth = mbf / disparity (Frame.cc:1039-1040)
    disp = kl["x"][m] - ur[m]
    assert np.allclose(d[m], np.float32(cfg["bf"]) / disp, rtol=1e-6)
    _, truth = synth.render(cfg, synth.trajectory(1, seed=0)[0], synth.default_room(0), seed=0)
    t = truth[kl["y"][m].astype(int), kl["x"][m].astype(int)]
    ok = t > 0
    rel = np.abs(d[m][ok] - t[ok]) / t[ok]
    assert np.median(rel) < 0.01 and np.mean(rel < 0.05) > 0.9


def test_stereo_no_right_keypoints(oracle):
    cfg, left, right = stereo_pair(0)
    p = oracle.params(2000, 1.2, 8, 20, 7)
    kl, dl, _ = oracle.extract(p, left)
    ur, d = oracle.stereo_matches(oracle.camera(cfg), p, left, right, kl, dl, kl[:0], dl[:0])
    assert np.all(ur == -1) and np.all(d == -1)


def test_stereo_vo_follows_the_trajectory(oracle):
    """The oracle's stereo TrackWithMotionModel loop (Frame(imLeft, imRight),
    th = 7) tracks the rendered KITTI-camera sequence to a few mm."""
    from _scenes import stereo_sequence
    cfg, traj, pairs = stereo_sequence(3, 51)
    lvo = oracle.LVO(oracle.params(2000), oracle.camera(cfg), 1, use_lines=False)
    lvo.reset(np.linalg.inv(traj[0]).astype(np.float32).reshape(1, 16))
    for f, (l, r) in enumerate(pairs):
        T, st = lvo.step_stereo(0, l, r)
        assert st["ok"] == 1 and st["nlines"] == 0
        if f:
            assert st["nmatches"] >= 100 and st["ninliers"] >= 0.8 * st["nmatches"]
        assert np.abs(T - np.linalg.inv(traj[f])).max() < 5e-3
