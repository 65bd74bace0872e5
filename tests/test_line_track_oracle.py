"""CPU tests of the line-tracking oracle (oracle/line_track_oracle.cpp):
Frame::UndistortKeyLines + line depths, LineMatcher::SearchByProjection(Frame,
Frame) and the point+line TrackWithMotionModel loop (LVO)."""
import numpy as np

from _scenes import sequence


def test_line_frame_prepare_identity_without_distortion(oracle):
    cfg, _, frames = sequence(1, 3, cam_name="TUM3")
    gray, depth = frames[0]
    kl, _, _, _ = oracle.line_extract(gray)
    ku, ds, de, _, _ = oracle.line_frame_prepare(oracle.camera(cfg), kl, depth)
    assert len(kl) > 20
    # k1 == 0: UndistortKeyLines returns the key lines untouched (Frame.cc:771)
    assert ku.tobytes() == kl.tobytes()
    # imDepth.at<float>(v, u) at the end points, -1 where no depth (P14)
    W, H = cfg["width"], cfg["height"]
    for j in range(len(kl)):
        for x, y, d in ((kl["startPointX"][j], kl["startPointY"][j], ds[j]),
                        (kl["endPointX"][j], kl["endPointY"][j], de[j])):
            idx = int(y) * W + int(x)
            z = depth.reshape(-1)[idx] if 0 <= idx < W * H else 0.0
            assert d == (z if z > 0 else -1.0)


def test_line_frame_prepare_undistorts_end_points(oracle):
    cfg, _, frames = sequence(1, 4, cam_name="TUM1")
    gray, depth = frames[0]
    kl, _, _, _ = oracle.line_extract(gray)
    ku, _, _, _, _ = oracle.line_frame_prepare(oracle.camera(cfg), kl, depth)
    moved = np.abs(ku["startPointX"] - kl["startPointX"]) + np.abs(ku["endPointY"] - kl["endPointY"])
    assert moved.max() > 0.5
    # the refreshed fields follow the undistorted end points
    assert np.array_equal(ku["sPointInOctaveX"], ku["startPointX"])
    assert np.array_equal(ku["ePointInOctaveY"], ku["endPointY"])
    assert np.allclose(ku["lineLength"],
                       np.hypot(ku["endPointX"] - ku["startPointX"],
                                ku["endPointY"] - ku["startPointY"]), rtol=1e-5)


def test_line_search_by_projection_finds_itself(oracle):
    """The last frame's lines as map lines, projected with the same pose,
    match the frame's own lines (each current line's last passing projection
    wins, so a line may take a collinear neighbour; most keep their own)."""
    cfg, traj, frames = sequence(1, 5, cam_name="TUM3")
    gray, depth = frames[0]
    cam = oracle.camera(cfg)
    kl, desc, _, _ = oracle.line_extract(gray)
    ku, ds, de, _, _ = oracle.line_frame_prepare(cam, kl, depth)
    Tcw = np.linalg.inv(traj[0]).astype(np.float32)
    Twc = np.linalg.inv(Tcw.astype(np.float64))
    has = ((ds > 0) & (de > 0)).astype(np.uint8)
    xyz = np.zeros((len(ku), 6), np.float32)
    for j in range(len(ku)):
        for e, (u, v, z) in enumerate(((ku["startPointX"][j], ku["startPointY"][j], ds[j]),
                                       (ku["endPointX"][j], ku["endPointY"][j], de[j]))):
            Pc = np.array([(u - cfg["cx"]) * z / cfg["fx"], (v - cfg["cy"]) * z / cfg["fy"], z, 1.0])
            xyz[j, 3 * e:3 * e + 3] = (Twc @ Pc)[:3]
    match, nm = oracle.line_search_by_projection_last(cam, Tcw, ku, desc, ku, has,
                                                      np.zeros(len(ku), np.uint8), xyz, desc)
    assert nm >= has.sum()
    matched = match >= 0
    assert matched.sum() >= 0.9 * has.sum()
    assert (match[matched] == np.arange(len(ku))[matched]).mean() > 0.7
    # lines without map lines are never matched by index
    assert not np.isin(np.nonzero(has == 0)[0], match[matched]).any()


def test_lvo_without_lines_equals_points_vo(oracle):
    F = 4
    cfg, traj, frames = sequence(F, 6)
    T0 = np.linalg.inv(traj[0]).astype(np.float32).reshape(1, 16)
    vo = oracle.VO(oracle.params(), oracle.camera(cfg), 1)
    lvo = oracle.LVO(oracle.params(), oracle.camera(cfg), 1, use_lines=False)
    vo.reset(T0)
    lvo.reset(T0)
    for f in range(F):
        Ta, sa = vo.step(0, *frames[f])
        Tb, sb = lvo.step(0, *frames[f])
        assert np.array_equal(Ta, Tb)
        for k in ("nkeypoints", "nmatches", "ninliers", "nmatches_map"):
            assert sa[k] == sb[k], (f, k)
        assert sb["nlines"] == 0 and sb["line_matches"] == 0


def test_lvo_with_lines_tracks(oracle):
    F = 4
    cfg, traj, frames = sequence(F, 7)
    T0 = np.linalg.inv(traj[0]).astype(np.float32).reshape(1, 16)
    lvo = oracle.LVO(oracle.params(), oracle.camera(cfg), 1, use_lines=True)
    lvo.reset(T0)
    for f in range(F):
        T, s = lvo.step(0, *frames[f])
        assert 0 < s["nlines"] <= 80
        if f:
            assert s["line_matches"] >= 15, s
            assert s["ok"] == 1
            assert s["line_nmatches_map"] <= s["line_matches"]
            # the reference's line edge (P7) pulls the pose off by centimetres
            # at most on this scene; the tracker must stay near truth
            Tgt = np.linalg.inv(traj[f])
            assert np.abs(T[:3, 3] - Tgt[:3, 3]).max() < 0.2


def test_list_overload_equals_last_frame_overload(oracle):
    """The local-map / ref-KF body with valid = has_ml && !outlier and no
    claims gives the last-frame overload's result (the projected KeyLine's
    base fields are all rewritten by UpdateKeyLineData)."""
    from _scenes import line_map_problem
    cfg, cam, xyz, desc, ku, ld, cur_nobs, T2 = line_map_problem(4)
    n = len(xyz)
    rng = np.random.default_rng(0)
    has = (rng.random(n) < 0.9).astype(np.uint8)
    out = (rng.random(n) < 0.1).astype(np.uint8)
    base = np.zeros(n, ku.dtype)
    m1, n1 = oracle.line_search_by_projection_last(cam, T2, ku, ld, base, has, out, xyz, desc)
    m2, n2, w = oracle.line_search_by_projection_list(cam, T2, ku, ld, None, has & (1 - out), xyz,
                                                      desc)
    assert n1 == n2 and np.array_equal(m1, m2) and n1 > 10


def test_line_in_frustum(oracle):
    T = np.eye(4, dtype=np.float32)
    X = np.array([[0, 0, 1, 0, 0, 2], [0, 0, -1, 0, 0, 2], [0, 0, -1, 0, 0, -2]], np.float32)
    assert oracle.line_is_in_frustum(T, X).tolist() == [1, 1, 0]


def test_harness_pairs_overloads(oracle):
    """The reference's harness overloads (LineMatcher.cpp:272-487 last frame,
    :954-1170 local map; oracle_line_search_pairs) against the tracking
    overloads: with no Observations() anywhere they assign the same map lines
    and count the same matches; match_indices lists every passing pair in
    (current j, projected i) order, so its last pair per j is the assignment;
    new_kls are the projected lines in map-line order."""
    from _scenes import line_map_problem
    cfg, cam, xyz, desc, ku, ld, cur_nobs, T2 = line_map_problem(4)
    n = len(xyz)
    rng = np.random.default_rng(1)
    has = (rng.random(n) < 0.9).astype(np.uint8)
    out = (rng.random(n) < 0.1).astype(np.uint8)
    base = np.zeros(n, ku.dtype)
    valid = has & (1 - out)
    m1, n1 = oracle.line_search_by_projection_last(cam, T2, ku, ld, base, has, out, xyz, desc)
    m, nm, w, pk, ps, pr = oracle.line_search_pairs(cam, T2, 0, ku, ld, None, valid, base, xyz,
                                                    desc, None)
    assert nm == n1 > 10 and np.array_equal(m, m1) and len(pr) == nm
    assert np.all(np.diff(ps) > 0) and np.all(valid[ps] == 1)
    assert np.all(np.diff(pr[:, 1]) >= 0)                    # j-major
    for j in np.unique(pr[:, 1]):
        assert ps[pr[pr[:, 1] == j][-1, 0]] == m[j]           # the last pair wins
    # local map: the list overload (away from the retry boundary)
    m2, n2, w2 = oracle.line_search_by_projection_list(cam, T2, ku, ld, cur_nobs, valid, xyz, desc)
    mb, nb, wb, pkb, psb, prb = oracle.line_search_pairs(cam, T2, 1, ku, ld, cur_nobs, valid, None,
                                                         xyz, desc, None)
    assert (nb, wb) == (n2, w2) and np.array_equal(mb, m2) and len(prb) == nb
    assert np.array_equal(psb, ps)
    for f in ("startPointX", "startPointY", "endPointX", "endPointY", "lineLength", "angle"):
        assert np.array_equal(pkb[f], pk[f]), f


def test_harness_last_frame_skips_observed_per_pair(oracle):
    """LineMatcher.cpp:272-487 tests Observations() > 0 inside the pair loop:
    once a current line holds an observed map line, its later pairs are
    skipped, so each current line keeps its FIRST passing map line and at
    most one pair (the tracking overload keeps the last and counts all)."""
    from _scenes import line_map_problem
    cfg, cam, xyz, desc, ku, ld, cur_nobs, T2 = line_map_problem(4)
    n = len(xyz)
    valid = np.ones(n, np.uint8)
    base = np.zeros(n, ku.dtype)
    r0 = oracle.line_search_pairs(cam, T2, 0, ku, ld, None, valid, base, xyz, desc, None)
    r1 = oracle.line_search_pairs(cam, T2, 0, ku, ld, None, valid, base, xyz, desc,
                                  np.ones(n, np.int32))
    m0, n0, _, _, ps, pr0 = r0
    m1, n1, _, _, _, pr1 = r1
    assert n1 < n0 and len(pr1) == n1
    assert len(np.unique(pr1[:, 1])) == len(pr1)              # one pair per current line
    for j, i in ((j, pr0[pr0[:, 1] == j][0, 0]) for j in np.unique(pr0[:, 1])):
        assert m1[j] == ps[i]                                 # the first passing map line


def test_bf_knn_ratio_hand_computed(oracle):
    """LineMatcher.cpp:492-525 (BFMatcher knnMatch k = 2, ratio 0.75) on
    descriptors with hand-set Hamming distances to train lines t0 (no bits),
    t1 (bits 100-139), t2 (bits 200-255):
      q0 bits 0-1:      2 / 42 / 58  -> t0 (ratio 0.05)
      q1 bits 100-121:  22 / 18 / 78 -> t1 18 vs t0 22 (0.82): none
      q2 bits 100-119 + 200-219: 40 / 40 / 56 -> tie at the best: ratio 1, none
      q3 bits 100-139:  40 / 0 / 96  -> t1 (zero best)
      q4 bit 0:         1 / 41 / 57  -> t0 again (overwrites q0, both count)."""
    def d(bits):
        v = np.zeros(32, np.uint8)
        for b in bits:
            v[b // 8] |= 1 << (b % 8)
        return v
    t = np.stack([d([]), d(range(100, 140)), d(range(200, 256))])
    q = np.stack([d(range(2)), d(range(100, 122)),
                  d(list(range(100, 120)) + list(range(200, 220))), d(range(100, 140)),
                  d(range(1))])
    dist = np.array([[int(np.unpackbits(a ^ b).sum()) for b in t] for a in q])
    assert dist.tolist() == [[2, 42, 58], [22, 18, 78], [40, 40, 56], [40, 0, 96], [1, 41, 57]]
    out, n = oracle.line_match_bf_knn(q, t)
    assert n == 3
    assert list(out) == [4, 3, -1]
