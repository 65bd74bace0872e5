"""The oracle's map model (map_oracle.cpp; Tracking::Track with KeyFrame /
MapPoint / MapLine, pinned P23-P25) on CPU: the invariants the reference's
Tracking / KeyFrame / MapPoint code guarantees, checked on synthetic RGB-D
sequences (the device map path is compared with this oracle in
test_gpu_map.py)."""
import numpy as np
import pytest

from _scenes import sequence


def _frames(F, seed, lines, turn=None):
    seqs = [sequence(F, seed, cam_name="TUM3" if lines else "TUM1")]
    fr = [seqs[0][2][f] for f in range(F)]
    if turn is not None:
        for f in range(turn, F):
            g, d = fr[f]
            fr[f] = (np.ascontiguousarray(g[::-1, ::-1]), np.ascontiguousarray(d[::-1, ::-1]))
    return seqs[0][0], seqs[0][1], fr


@pytest.mark.parametrize("lines", [False, True])
def test_map_initialisation_and_keyframes(oracle, lines):
    """StereoInitialization: one keyframe, a map point per keypoint with
    positive depth (each observed once, nObs 1 or 2 by uRight), a map line per
    line with both end-point depths; later keyframes get connected (parent =
    the best covisible keyframe, covisibility weights >= 15 or the best)."""
    cfg, traj, fr = _frames(8, 110, lines)
    m = oracle.MapVO(oracle.params(), oracle.camera(cfg), 1, use_lines=lines)
    m.reset(np.linalg.inv(traj[0]).astype(np.float32).reshape(1, 16))
    T, c0 = m.step(0, *fr[0])
    assert c0["keyframe"] == 2 and c0["keyframes"] == 1 and c0["state"] == 1
    p = oracle.params()
    kps, desc, _ = oracle.extract(p, fr[0][0])
    _, dep, ur, _, _ = oracle.frame_prepare(oracle.camera(cfg), kps, fr[0][1])
    assert c0["map_points"] == int((dep > 0).sum())
    nobs, _, _ = m.points(0)
    assert len(nobs) == c0["map_points"]
    assert set(np.unique(nobs)) <= {1, 2}
    if not lines:
        assert c0["map_lines"] == 0
    np.testing.assert_allclose(T, np.linalg.inv(traj[0]), atol=1e-6)   # the reset pose
    recs = [c0] + [m.step(0, *fr[f])[1] for f in range(1, 8)]
    assert all(r["ok"] == 1 and r["state"] == 1 for r in recs)
    # without a vocabulary every frame runs the motion model
    assert all(r["trk"] == 0 for r in recs)
    assert all(r["local_points"] > 0 for r in recs[1:])
    # counts only grow (no culling: P23)
    for a, b in zip(recs, recs[1:]):
        assert b["keyframes"] >= a["keyframes"] and b["map_points"] >= a["map_points"]
        assert (b["keyframe"] == 1) == (b["keyframes"] == a["keyframes"] + 1)
    par, ords = m.keyframes(0)
    assert len(par) == recs[-1]["keyframes"] and par[0] == -1
    for k in range(1, len(par)):
        assert 0 <= par[k] < k and len(ords[k]) >= 1 and ords[k][0] == par[k]
    nobs, _, _ = m.points(0)
    assert (nobs >= 1).all()


def test_map_temporal_points(oracle):
    """UpdateLastFrame: frames that are not keyframes get temporal VO points
    (at least 100 closest with depth not already map points)."""
    cfg, traj, fr = _frames(5, 120, False)
    m = oracle.MapVO(oracle.params(), oracle.camera(cfg), 1, use_lines=False)
    m.reset(np.linalg.inv(traj[0]).astype(np.float32).reshape(1, 16))
    recs = [m.step(0, *fr[f])[1] for f in range(5)]
    # frame 1's last frame is the initial keyframe: no temporal points
    assert recs[1]["temporal_points"] == 0
    assert any(r["temporal_points"] > 0 for r in recs[2:] if r["keyframe"] == 0)


def test_map_lost_resets_small_map(oracle):
    """Images turned by 180 degrees: tracking fails, the stream goes LOST and,
    its map holding <= 5 keyframes, resets (Tracking.cc:558-568); the reset
    step keeps its frame counts; the next frame initialises again."""
    cfg, traj, fr = _frames(7, 130, True, turn=4)
    m = oracle.MapVO(oracle.params(), oracle.camera(cfg), 1, use_lines=True)
    m.reset(np.linalg.inv(traj[0]).astype(np.float32).reshape(1, 16))
    recs = [m.step(0, *fr[f])[1] for f in range(7)]
    assert [r["state"] for r in recs[:4]] == [1, 1, 1, 1]
    r = recs[4]
    assert r["ok"] == 0 and r["state"] == 0 and r["keyframes"] == 0 and r["map_points"] == 0
    assert r["nkeypoints"] > 500 and r["nlines"] > 0      # the step's own counts survive the reset
    assert recs[5]["keyframe"] == 2 and recs[5]["state"] == 1
