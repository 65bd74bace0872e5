"""CPU tests of the SearchLocalPoints oracle (oracle/track_oracle.cpp):
Frame::IsInFrustum + PredictScale and the local-map SearchByProjection."""
import numpy as np

from _scenes import local_map_problem


def _log_scale(oracle):
    return float(np.float32(oracle.lsdm(1, float(np.float32(1.2)))))


def test_in_frustum_fields(oracle):
    cfg, cam, sc, mps, cur, cur_nobs, T3 = local_map_problem(1)
    tr = oracle.frame_is_in_frustum(cam, _log_scale(oracle), 8, T3, mps, 0.5)
    v = tr["in_view"] > 0
    assert v.sum() > 0.5 * len(v)
    # projections inside the image, levels in range, viewing cosine above the limit
    assert np.all((tr["proj_x"][v] >= 0) & (tr["proj_x"][v] <= cfg["width"]))
    assert np.all((tr["level"][v] >= 0) & (tr["level"][v] < 8)) and np.all(tr["level"][~v] == -1)
    assert np.all(tr["view_cos"][v] >= 0.5)
    # a point behind the camera is never in view
    far = dict(mps)
    far["xyz"] = -mps["xyz"][:5] * 100
    assert oracle.frame_is_in_frustum(cam, _log_scale(oracle), 8, T3, far, 0.5)["in_view"].sum() == 0


def test_local_map_matches_are_geometric(oracle):
    cfg, cam, sc, mps, cur, cur_nobs, T3 = local_map_problem(2)
    tr = oracle.frame_is_in_frustum(cam, _log_scale(oracle), 8, T3, mps, 0.5)
    m, n = oracle.search_by_projection_local(cam, sc, cur, tr, mps["desc"], mps["nobs"], cur_nobs,
                                             3.0, 0.8)
    assert n > 100 and (m >= 0).sum() <= n
    # claimed keypoints (Observations() > 0) are never reassigned
    assert np.all(m[cur_nobs > 0] == -1)
    j = np.nonzero(m >= 0)[0]
    dx = cur["kps_un"]["x"][j] - tr["proj_x"][m[j]]
    dy = cur["kps_un"]["y"][j] - tr["proj_y"][m[j]]
    assert np.median(np.hypot(dx, dy)) < 3.0


def test_search_by_bow_oracle_properties(oracle):
    from _scenes import bow_problem
    b = bow_problem(1)
    m, n = oracle.search_by_bow(**b)
    j = np.nonzero(m >= 0)[0]
    assert n == len(j) > 50
    # matched pairs share a node, have a valid keyframe map point and pass TH_LOW
    assert np.all(b["kf_node"][m[j]] == b["f_node"][j])
    assert np.all(b["kf_valid"][m[j]] == 1)
    d = np.unpackbits(b["kf_desc"][m[j]] ^ b["f_desc"][j], axis=1).sum(1)
    assert d.max() <= 50
    # a keyframe feature is used at most once per node walk
    assert len(np.unique(m[j])) == len(j)


def test_predict_scale_hand_computed(oracle):
    """MapPoint::PredictScale's ratio is mfMaxDistance / dist (MapPoint.cc:421),
    not GetMaxDistanceInvariance() / dist: a point seen from its creation
    distance at octave k predicts octave k (0 exactly for octave 0)."""
    from _scenes import predict_scale_problem
    cfg, T, mps, lev, ratio = predict_scale_problem()
    tr = oracle.frame_is_in_frustum(oracle.camera(cfg), _log_scale(oracle), 8, T, mps, 0.5)
    assert tr["in_view"].all()
    assert np.array_equal(tr["level"], lev)
    # a point at its creation distance and octave: level == octave
    same = np.isclose(ratio, mps["max_dist"] / mps["xyz"][:, 2]) & (
        np.abs(np.log(ratio) / np.log(1.2) - np.round(np.log(ratio) / np.log(1.2))) < 1e-5)
    k = np.round(np.log(ratio[same]) / np.log(1.2)).astype(int)
    assert tr["level"][same][k == 0].tolist() == [0] * int((k == 0).sum()) and (k == 0).sum() >= 2
    assert np.all(np.abs(tr["level"][same] - k) <= 1)


def test_in_frustum_reject_branches(oracle):
    """The oracle's IsInFrustum rejects every point of each branch subset of
    frustum_reject_problem (behind, outside, far, near, view cosine) and keeps
    most of the others (the GPU parity test relies on this problem)."""
    from _scenes import frustum_reject_problem
    cfg, cam, sc, mps, cur, cur_nobs, T, masks = frustum_reject_problem(1)
    iv = oracle.frame_is_in_frustum(cam, _log_scale(oracle), 8, T, mps, 0.5)["in_view"].astype(bool)
    rest = ~np.any(np.stack(list(masks.values())), 0)
    for b, mk in masks.items():
        assert mk.sum() > 0 and not iv[mk].any(), b
    assert iv[rest].mean() > 0.9
