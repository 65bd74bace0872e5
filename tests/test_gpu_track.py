"""GPU parity of the tracking half against the CPU oracle:
Frame glue (bit-exact), ORBmatcher::SearchByProjection(Frame, Frame)
(bit-exact match sets), PoseOptimization (pose within 1e-4, identical
outlier labels), and the batched tracker vs the oracle VO loop."""
import numpy as np
import pytest

from _scenes import match_problem, sequence, frame_data, unproject

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4   # north_star: pose within 1e-4 RMSE (max-abs used here: stricter)


def _u32(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("cam_name", ["TUM1", "TUM3"])
def test_frame_prepare_bit_exact(cam_name, orbpl, oracle):
    cfg, traj, frames = sequence(2, 3, cam_name)
    cam_o = oracle.camera(cfg)
    cam_g = orbpl.make_camera(cfg)
    kps, desc, _ = oracle.extract(oracle.params(), frames[0][0])
    ku, d, ur, gc, b = orbpl.frame_prepare(cam_g, kps, frames[0][1])
    oku, od, our, ogc, ob = oracle.frame_prepare(cam_o, kps, frames[0][1])
    for f in ("x", "y"):
        assert np.array_equal(_u32(ku[f]), _u32(oku[f])), f
    assert np.array_equal(_u32(d), _u32(od))
    assert np.array_equal(_u32(ur), _u32(our))
    assert np.array_equal(gc, ogc)
    assert np.array_equal(_u32(b), _u32(ob))
    # monocular: no depth
    ku2, d2, ur2, gc2, _ = orbpl.frame_prepare(cam_g, kps, None)
    assert np.all(d2 == -1) and np.all(ur2 == -1)


@pytest.mark.parametrize("case", [
    dict(seed=0), dict(seed=1, th=7.0), dict(seed=2, mono=True), dict(seed=0, check_ori=False),
    dict(seed=1, nobs_zero_frac=0.3), dict(seed=2, outlier_frac=0.2), dict(seed=0, th=30.0),
    dict(seed=1, pert=(0.05, 0.03)),
])
def test_search_by_projection_last_bit_exact(case, orbpl, oracle):
    case = dict(case)
    th = case.pop("th", 15.0)
    mono = case.pop("mono", False)
    ori = case.pop("check_ori", True)
    cfg, cam_o, sc, cur, last, _ = match_problem(**case)
    cam_g = orbpl.make_camera(cfg)
    m_g, n_g = orbpl.ORBmatcher(0.9, ori).SearchByProjectionLastFrame(cam_g, sc, cur, last, th, mono)
    m_o, n_o = oracle.search_by_projection_last(cam_o, sc, cur, last, th, mono, ori)
    assert n_g == n_o
    assert np.array_equal(m_g, m_o), f"{int((m_g != m_o).sum())} assignments differ"
    assert n_o > 50


def _pose_problem(seed, stereo=True, lines=0, outliers=0.0, pert=(0.02, 0.02)):
    from _pkg import load_oracle
    O = load_oracle()
    cfg, cam_o, sc, cur, last, (f0, f1, T0, T1) = match_problem(seed)
    m, n = O.search_by_projection_last(cam_o, sc, cur, last, 15.0)
    has = (m >= 0).astype(np.uint8)
    xyz = np.zeros((len(m), 3), np.float32)
    xyz[has == 1] = last["mp_xyz"][m[has == 1]]
    rng = np.random.default_rng(seed)
    bad = (rng.random(len(m)) < outliers) & (has == 1)
    xyz[bad] += rng.normal(size=(bad.sum(), 3)).astype(np.float32) * 0.3
    ur = cur["uright"] if stereo else np.full(len(m), -1, np.float32)
    lw, lh, nf, scl, isc = O.level_sizes(O.params(), 640, 480)
    prob = dict(kps_un=cur["kps_un"], uright=ur, has_mp=has, mp_xyz=xyz,
                inv_sigma2=(1.0 / (scl * scl)).astype(np.float32))
    if lines:
        # synthetic 3D segments in front of the camera, observed at the true pose
        Twc = np.linalg.inv(T1.astype(np.float64))
        P = rng.uniform([-1.5, -1, 1.5], [1.5, 1, 4], size=(lines, 2, 3))
        Pw = P @ Twc[:3, :3].T + Twc[:3, 3]
        uv = P[..., :2] / P[..., 2:] * [cfg["fx"], cfg["fy"]] + [cfg["cx"], cfg["cy"]]
        uv += rng.normal(size=uv.shape) * 0.5
        prob.update(kl_obs=uv.reshape(lines, 4).astype(np.float32),
                    kl_octave=np.zeros(lines, np.int32),
                    has_ml=(rng.random(lines) < 0.9).astype(np.uint8),
                    ml_xyz=Pw.reshape(lines, 6).astype(np.float32))
    T_init = cur["Tcw"] if pert is None else __import__("_scenes").perturb(T1, *pert, seed=seed + 3)
    return cfg, cam_o, prob, T_init, T1


@pytest.mark.parametrize("case", [
    dict(seed=0), dict(seed=1, stereo=False), dict(seed=2, outliers=0.15),
    dict(seed=0, lines=40), dict(seed=1, lines=60, outliers=0.1), dict(seed=2, pert=(0.08, 0.05)),
    dict(seed=0, lines=40, fixed=True), dict(seed=1, lines=60, outliers=0.1, fixed=True),
])
def test_pose_optimization_parity(case, orbpl, oracle):
    case = dict(case)
    fixed = case.pop("fixed", False)
    cfg, cam_o, prob, T_init, T_true = _pose_problem(**case)
    cam_g = orbpl.make_camera(cfg)
    n = len(prob["kps_un"])
    nl = len(prob.get("kl_obs", ()))
    out0 = np.zeros(n, np.uint8)
    lout0 = np.zeros(nl, np.uint8)
    Tg, og, log_, ng = orbpl.pose_optimization(cam_g, prob, T_init, out0, lout0, fixed)
    To, oo, loo, no = oracle.pose_optimization(cam_o, prob, T_init, out0, lout0, fixed)
    assert np.abs(Tg - To).max() < POSE_TOL, np.abs(Tg - To).max()
    assert ng == no
    assert np.array_equal(og, oo)
    assert np.array_equal(log_, loo)
    if not case.get("lines") or fixed:
        # converged near the truth (the as-written line Jacobian, P7, pulls off it)
        assert np.abs(To[:3, 3] - T_true[:3, 3]).max() < 0.01


def test_pose_too_few_correspondences(orbpl, oracle):
    cfg, cam_o, prob, T_init, _ = _pose_problem(0)
    prob["has_mp"] = np.zeros_like(prob["has_mp"])
    prob["has_mp"][:2] = 1
    n = len(prob["kps_un"])
    Tg, og, _, ng = orbpl.pose_optimization(orbpl.make_camera(cfg), prob, T_init, np.zeros(n, np.uint8))
    assert ng == 0 and np.array_equal(Tg, T_init)


def test_tracker_matches_oracle_vo(orbpl, oracle):
    S, F = 3, 5
    cams = []
    seqs = [sequence(F, 10 + s) for s in range(S)]
    cfg = seqs[0][0]
    orb = oracle.params()
    vo = oracle.VO(orb, oracle.camera(cfg), S)
    tr = orbpl.Tracker(orbpl.OrbParams(1000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S)
    T0 = np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs])
    vo.reset(T0.reshape(S, 16))
    tr.reset(T0.reshape(S, 16))
    gray = orbpl.DeviceBuffer(S * 640 * 480)
    depth = orbpl.DeviceBuffer(S * 640 * 480 * 4)
    for f in range(F):
        gray.upload(np.stack([sq[2][f][0] for sq in seqs]))
        depth.upload(np.stack([sq[2][f][1] for sq in seqs]))
        tr.step_device(gray.ptr, depth.ptr)
        tr.synchronize()
        st = tr.state()
        for s in range(S):
            To, so = vo.step(s, seqs[s][2][f][0], seqs[s][2][f][1])
            assert st["nkeypoints"][s] == so["nkeypoints"]
            assert st["nmatches"][s] == so["nmatches"], (f, s)
            assert st["ninliers"][s] == so["ninliers"], (f, s)
            assert st["nmatches_map"][s] == so["nmatches_map"], (f, s)
            assert np.abs(st["Tcw"][s] - To).max() < POSE_TOL, (f, s)
    ms = tr.stage_ms()
    assert np.all(ms >= 0)


@pytest.mark.parametrize("split", [False, True])
def test_tracker_pipelined_matches_oracle_vo(orbpl, oracle, split, monkeypatch):
    """Two-stream pipelined tracker, steps issued back to back (no host sync
    between steps): the final state equals the oracle VO after F frames.
    split: the ORB extraction batch in two offset halves on two streams
    (ORBPL_ORB_SPLIT=1; frames 0-1 and 2 here)."""
    monkeypatch.setenv("ORBPL_ORB_SPLIT", "1" if split else "0")
    S, F = 3, 6
    seqs = [sequence(F, 20 + s) for s in range(S)]
    cfg = seqs[0][0]
    vo = oracle.VO(oracle.params(), oracle.camera(cfg), S)
    tr = orbpl.Tracker(orbpl.OrbParams(1000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S)
    tr.set_pipelined(True)
    T0 = np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs])
    vo.reset(T0.reshape(S, 16))
    tr.reset(T0.reshape(S, 16))
    tr.set_history(F)
    gray = orbpl.DeviceBuffer.from_array(
        np.stack([np.stack([sq[2][f][0] for sq in seqs]) for f in range(F)]))
    depth = orbpl.DeviceBuffer.from_array(
        np.stack([np.stack([sq[2][f][1] for sq in seqs]) for f in range(F)]))
    fb = S * 640 * 480
    for f in range(F):
        tr.step_device(gray.ptr + f * fb, depth.ptr + f * fb * 4)
    tr.synchronize()
    st = tr.state()
    for s in range(S):
        Th, Ch = tr.history(s)      # device-side per-step history (bench parity source)
        assert len(Th) == F
        for f in range(F):
            To, so = vo.step(s, seqs[s][2][f][0], seqs[s][2][f][1])
            assert np.abs(Th[f] - To).max() < POSE_TOL, (s, f)
            assert Ch[f][0] == so["nkeypoints"] and Ch[f][1] == so["nmatches"], (s, f)
            assert Ch[f][2] == so["ninliers"] and Ch[f][3] == so["nmatches_map"], (s, f)
        assert st["nkeypoints"][s] == so["nkeypoints"]
        assert st["nmatches"][s] == so["nmatches"], s
        assert st["ninliers"][s] == so["ninliers"], s
        assert st["nmatches_map"][s] == so["nmatches_map"], s
        assert np.abs(st["Tcw"][s] - To).max() < POSE_TOL, s


@pytest.mark.parametrize("pipelined,fixed,split", [(False, False, False), (True, False, False),
                                                  (False, True, False), (True, False, True)])
def test_tracker_with_lines_matches_oracle_lvo(orbpl, oracle, pipelined, fixed, split, monkeypatch):
    """Point+line tracker (ORBPL_TRACK_LINES) against the oracle LVO loop:
    identical point and line counts every frame, pose within POSE_TOL, and
    the last frame's undistorted KeyLines / LBD rows bit-exact. split: the LSD
    batch and the ORB extraction batch in two offset halves on two streams
    each (ORBPL_LSD_SPLIT=1, ORBPL_ORB_SPLIT=1; frames 0-1 and 2 here)."""
    monkeypatch.setenv("ORBPL_LSD_SPLIT", "1" if split else "0")
    monkeypatch.setenv("ORBPL_ORB_SPLIT", "1" if split else "0")
    S, F = 3, 5
    seqs = [sequence(F, 30 + s) for s in range(S)]
    cfg = seqs[0][0]
    lvo = oracle.LVO(oracle.params(), oracle.camera(cfg), S, use_lines=True,
                     flags=oracle.TRACK_FIXED_LINE_JAC if fixed else 0)
    tr = orbpl.Tracker(orbpl.OrbParams(1000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S, lines=True,
                       fixed_line_jac=fixed)
    tr.set_pipelined(pipelined)
    T0 = np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs])
    lvo.reset(T0.reshape(S, 16))
    tr.reset(T0.reshape(S, 16))
    gray = orbpl.DeviceBuffer(S * 640 * 480)
    depth = orbpl.DeviceBuffer(S * 640 * 480 * 4)
    for f in range(F):
        gray.upload(np.stack([sq[2][f][0] for sq in seqs]))
        depth.upload(np.stack([sq[2][f][1] for sq in seqs]))
        tr.step_device(gray.ptr, depth.ptr)
        st, ls = tr.state(), tr.status()
        for s in range(S):
            To, so = lvo.step(s, seqs[s][2][f][0], seqs[s][2][f][1])
            got = dict(nkeypoints=st["nkeypoints"][s], nmatches=st["nmatches"][s],
                       ninliers=st["ninliers"][s], nmatches_map=st["nmatches_map"][s],
                       ok=ls["ok"][s], nlines=ls["nlines"][s], line_matches=ls["line_matches"][s],
                       line_nmatches_map=ls["line_nmatches_map"][s])
            assert {k: int(v) for k, v in got.items()} == so, (f, s)
            assert np.abs(st["Tcw"][s] - To).max() < POSE_TOL, (f, s)
    cam_o = oracle.camera(cfg)
    for s in range(S):
        g, d = seqs[s][2][F - 1]
        kl, desc, _, _ = oracle.line_extract(g)
        ku, _, _, _, _ = oracle.line_frame_prepare(cam_o, kl, d)
        kl_g, desc_g, lm_g, lo_g = tr.lines(s)
        assert kl_g.tobytes() == ku.tobytes()
        assert np.array_equal(desc_g, desc)
        assert np.all(lo_g == 0)
        # kept matches = inliers; the map count subtracts the outliers (quirk)
        assert (lm_g >= 0).sum() >= ls["line_nmatches_map"][s]
    lt = tr.line_timings()
    assert lt.shape[1] == 3 and np.all(lt >= 0)


@pytest.mark.parametrize("pipelined,lines", [(False, False), (True, False), (False, True),
                                             (True, True)])
def test_stereo_tracker_matches_oracle(orbpl, oracle, pipelined, lines):
    """Stereo tracker (ORBPL_TRACK_STEREO, KITTI 00 camera, 2000 features):
    ORB on both images, batched ComputeStereoMatches, th = 7 matching and the
    pose, against the oracle's stereo VO loop: identical counts every frame,
    pose within POSE_TOL. With lines (configs[3], the defined P17 mode):
    LineExtractor on both images, stereo line depths, line matching and line
    edges; the last frame's KeyLines bit-exact."""
    from _scenes import stereo_sequence
    S, F = 2, 4
    seqs = [stereo_sequence(F, 50 + s) for s in range(S)]
    cfg = seqs[0][0]
    W, H = cfg["width"], cfg["height"]
    lvo = oracle.LVO(oracle.params(2000), oracle.camera(cfg), S, use_lines=lines)
    tr = orbpl.Tracker(orbpl.OrbParams(2000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S, stereo=True,
                       lines=lines)
    tr.set_pipelined(pipelined)
    T0 = np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs])
    lvo.reset(T0.reshape(S, 16))
    tr.reset(T0.reshape(S, 16))
    left = orbpl.DeviceBuffer(S * W * H)
    right = orbpl.DeviceBuffer(S * W * H)
    for f in range(F):
        left.upload(np.stack([sq[2][f][0] for sq in seqs]))
        right.upload(np.stack([sq[2][f][1] for sq in seqs]))
        tr.step_stereo_device(left.ptr, right.ptr)
        tr.synchronize()
        st, ls = tr.state(), tr.status()
        for s in range(S):
            To, so = lvo.step_stereo(s, *seqs[s][2][f])
            got = dict(nkeypoints=st["nkeypoints"][s], nmatches=st["nmatches"][s],
                       ninliers=st["ninliers"][s], nmatches_map=st["nmatches_map"][s],
                       ok=ls["ok"][s], nlines=ls["nlines"][s], line_matches=ls["line_matches"][s],
                       line_nmatches_map=ls["line_nmatches_map"][s])
            assert {k: int(v) for k, v in got.items()} == so, (f, s)
            assert np.abs(st["Tcw"][s] - To).max() < POSE_TOL, (f, s)
        if f > 0:
            assert st["nmatches"].min() >= 100
            if lines:
                assert ls["line_matches"].min() >= 15
    stt = tr.stereo_timings()
    assert stt.shape[1] == 4 and np.all(stt >= 0)
    if lines:
        assert np.all(stt[:, 2:] > 0)
        cam_o = oracle.camera(cfg)
        for s in range(S):
            g, r = seqs[s][2][F - 1]
            kl, desc, _, _ = oracle.line_extract(g)
            ku, _, _, _, _ = oracle.line_frame_prepare(cam_o, kl, None)
            kl_g, desc_g, _, _ = tr.lines(s)
            assert kl_g.tobytes() == ku.tobytes()
            assert np.array_equal(desc_g, desc)
    with pytest.raises(RuntimeError):
        tr.step_device(left.ptr, right.ptr)


def test_tracker_rig_720p_matches_oracle(orbpl, oracle):
    """configs[4] geometry: two cameras of the synthetic 1280x720 8-camera rig
    (RGB-D, ORB 2000) tracked for 3 frames, identical counts, pose within
    POSE_TOL of the oracle VO loop."""
    load_pkg = __import__("_pkg").load_pkg
    load_pkg()
    import orbpl.synth as synth
    cfg = dict(synth.RIG720)
    traj = synth.loop_trajectory(12, seed=3)
    room = synth.default_room(3)
    cams = (0, 3)
    S, F = len(cams), 3
    frames = [[synth.render(cfg, traj[t] @ synth.rig_offset(c), room, seed=30 + 8 * t + c)
               for c in cams] for t in range(F)]
    vo = oracle.VO(oracle.params(2000), oracle.camera(cfg), S)
    tr = orbpl.Tracker(orbpl.OrbParams(2000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S)
    T0 = np.stack([np.linalg.inv(traj[0] @ synth.rig_offset(c)).astype(np.float32) for c in cams])
    vo.reset(T0.reshape(S, 16))
    tr.reset(T0.reshape(S, 16))
    W, H = cfg["width"], cfg["height"]
    gray = orbpl.DeviceBuffer(S * W * H)
    depth = orbpl.DeviceBuffer(S * W * H * 4)
    for t in range(F):
        gray.upload(np.stack([g for g, _ in frames[t]]))
        depth.upload(np.stack([d for _, d in frames[t]]))
        tr.step_device(gray.ptr, depth.ptr)
        tr.synchronize()
        st = tr.state()
        for s in range(S):
            To, so = vo.step(s, *frames[t][s])
            assert st["nkeypoints"][s] == so["nkeypoints"]
            assert st["nmatches"][s] == so["nmatches"], (t, s)
            assert st["ninliers"][s] == so["ninliers"], (t, s)
            assert np.abs(st["Tcw"][s] - To).max() < POSE_TOL, (t, s)


def test_stereo_overflow_reported_once(orbpl, monkeypatch):
    """A row-band capacity overflow in ComputeStereoMatches (forced with a tiny
    ORBPL_STEREO_ENTRY_CAP) is reported as ORBPL_ERR_OVERFLOW by one
    synchronize, then cleared: the next synchronize succeeds, and reset
    clears it too."""
    from _scenes import stereo_sequence
    cfg, traj, pairs = stereo_sequence(1, 50)
    W, H = cfg["width"], cfg["height"]
    monkeypatch.setenv("ORBPL_STEREO_ENTRY_CAP", "16")
    tr = orbpl.Tracker(orbpl.OrbParams(2000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), 1, stereo=True)
    monkeypatch.delenv("ORBPL_STEREO_ENTRY_CAP")
    left = orbpl.DeviceBuffer.from_array(pairs[0][0])
    right = orbpl.DeviceBuffer.from_array(pairs[0][1])
    tr.step_stereo_device(left.ptr, right.ptr)
    with pytest.raises(orbpl.OrbplError, match="-5"):
        tr.synchronize()
    tr.synchronize()            # reported once
    tr.step_stereo_device(left.ptr, right.ptr)
    with pytest.raises(orbpl.OrbplError, match="-5"):
        tr.synchronize()
    tr.step_stereo_device(left.ptr, right.ptr)
    tr.reset()                  # reset clears the flag as well
    tr.synchronize()
    tr.close()


@pytest.mark.parametrize("cam_name", ["TUM1", "TUM3"])
def test_line_frame_prepare_bit_exact(orbpl, oracle, cam_name):
    cfg, _, fr = sequence(1, 41, cam_name=cam_name)
    g, d = fr[0]
    kl, _, _, _ = oracle.line_extract(g)
    got = orbpl.line_frame_prepare(orbpl.make_camera(cfg), kl, d)
    exp = oracle.line_frame_prepare(oracle.camera(cfg), kl, d)
    assert got[0].tobytes() == exp[0].tobytes()
    for a, b in zip(got[1:], exp[1:]):
        assert np.array_equal(a, b)
    got = orbpl.line_frame_prepare(orbpl.make_camera(cfg), kl, None)
    assert np.all(got[1] == -1) and np.all(got[4] == -1)


def _map_lines(cfg, ku, ds, de, Tcw):
    """Map lines of a frame as the tracker builds them (start depth for both
    end points, Frame.cc:1192), world coordinates in float."""
    has = ((ds > 0) & (de > 0)).astype(np.uint8)
    Twc = np.linalg.inv(Tcw.astype(np.float64))
    xyz = np.zeros((len(ku), 6), np.float32)
    for j in range(len(ku)):
        z = float(ds[j])
        for e, (u, v) in enumerate(((ku["startPointX"][j], ku["startPointY"][j]),
                                    (ku["endPointX"][j], ku["endPointY"][j]))):
            P = np.array([(u - cfg["cx"]) * z / cfg["fx"], (v - cfg["cy"]) * z / cfg["fy"], z, 1.0])
            xyz[j, 3 * e:3 * e + 3] = (Twc @ P)[:3]
    return has, xyz


@pytest.mark.parametrize("case", ["next_frame", "perturbed", "outliers"])
def test_line_search_by_projection_last_bit_exact(orbpl, oracle, case):
    cfg, traj, fr = sequence(2, 42, cam_name="TUM1")
    cam_o, cam_g = oracle.camera(cfg), orbpl.make_camera(cfg)
    frames = []
    for g, d in fr:
        kl, desc, _, _ = oracle.line_extract(g)
        ku, ds, de, _, _ = oracle.line_frame_prepare(cam_o, kl, d)
        frames.append((ku, desc, ds, de))
    T0 = np.linalg.inv(traj[0]).astype(np.float32)
    T1 = np.linalg.inv(traj[1]).astype(np.float32)
    if case == "perturbed":
        T1 = T1.copy()
        T1[:3, 3] += np.float32([0.01, -0.005, 0.01])
    has, xyz = _map_lines(cfg, frames[0][0], frames[0][2], frames[0][3], T0)
    out = np.zeros(len(has), np.uint8)
    if case == "outliers":
        out[::3] = 1
    args = (T1, frames[1][0], frames[1][1], frames[0][0], has, out, xyz, frames[0][1])
    m_g, n_g = orbpl.LineMatcher.SearchByProjectionLastFrame(cam_g, *args)
    m_o, n_o = oracle.line_search_by_projection_last(cam_o, *args)
    assert n_g == n_o and n_o > 10
    assert np.array_equal(m_g, m_o)


def _unproject_p6(cfg, ku, dep, T):
    """Frame::UnprojectStereo as the tracker computes it (float pixel terms,
    double-accumulated Rwc x + Ow, P6)."""
    invfx = np.float32(1.0) / np.float32(cfg["fx"])
    invfy = np.float32(1.0) / np.float32(cfg["fy"])
    cx, cy = np.float32(cfg["cx"]), np.float32(cfg["cy"])
    z = dep.astype(np.float32)
    x3 = np.stack([(ku["x"] - cx) * z * invfx, (ku["y"] - cy) * z * invfy, z], 1).astype(np.float32)
    Td = T.astype(np.float64)
    Ow = [np.float32(-(Td[0, r] * Td[0, 3] + Td[1, r] * Td[1, 3] + Td[2, r] * Td[2, 3]))
          for r in range(3)]
    out = np.zeros_like(x3)
    for r in range(3):
        s = Td[0, r] * x3[:, 0].astype(np.float64) + Td[1, r] * x3[:, 1].astype(np.float64)
        s = s + Td[2, r] * x3[:, 2].astype(np.float64)
        out[:, r] = (s + np.float64(Ow[r])).astype(np.float32)
    return out


@pytest.mark.parametrize("seed", [5, 6, 7, 8])
def test_search_by_projection_tie_order(orbpl, oracle, seed):
    """Equal-distance candidates displaced by a better later one keep their
    grid-scan order (regression: TUM3 seed 5, last point 911 -> 996)."""
    cfg, traj, fr = sequence(2, seed, cam_name="TUM3")
    cam_o = oracle.camera(cfg)
    f0 = frame_data(oracle, cam_o, cfg, *fr[0])
    f1 = frame_data(oracle, cam_o, cfg, *fr[1])
    T0 = np.linalg.inv(traj[0]).astype(np.float32)
    has = (f0["depth"] > 0).astype(np.uint8)
    xyz = _unproject_p6(cfg, f0["kps_un"], np.where(f0["depth"] > 0, f0["depth"], 0), T0)
    last = dict(Tcw=T0, kps_un=f0["kps_un"], has_mp=has, outlier=np.zeros(len(has), np.uint8),
                mp_xyz=xyz, mp_desc=f0["desc"], mp_nobs=np.ones(len(has), np.int32))
    cur = dict(Tcw=T0, kps_un=f1["kps_un"], desc=f1["desc"], uright=f1["uright"])
    sc = oracle.level_sizes(oracle.params(), 640, 480)[3]
    for ori in (True, False):
        m_o, n_o = oracle.search_by_projection_last(cam_o, sc, cur, last, 15.0, False, ori)
        m_g, n_g = orbpl.ORBmatcher(0.9, ori).SearchByProjectionLastFrame(
            orbpl.make_camera(cfg), sc, cur, last, 15.0, False)
        assert n_g == n_o and np.array_equal(m_g, m_o), (ori, np.nonzero(m_g != m_o)[0][:5])


def _log_scale(oracle):
    return float(np.float32(oracle.lsdm(1, float(np.float32(1.2)))))


@pytest.mark.parametrize("seed", [1, 2])
def test_in_frustum_bit_exact(orbpl, oracle, seed):
    """k_in_frustum against the oracle on a local map in which >= 10 % of the
    map points fail each IsInFrustum test (Frame.cc:345-401, MapPoint.cc:
    387-431; _scenes.frustum_reject_problem): behind the camera, outside the
    image, beyond 1.2 mfMaxDistance, inside 0.8 mfMinDistance, view cosine
    < 0.5. in_view / level / projections / view cos bit-exact, every
    branch's points rejected, the rest mostly in view."""
    from _scenes import frustum_reject_problem
    cfg, cam_o, sc, mps, cur, cur_nobs, T3, masks = frustum_reject_problem(seed)
    g = orbpl.frame_is_in_frustum(orbpl.make_camera(cfg), 1.2, 8, T3, mps, 0.5)
    o = oracle.frame_is_in_frustum(cam_o, _log_scale(oracle), 8, T3, mps, 0.5)
    for k in o:
        assert np.array_equal(g[k], o[k]), k
    n = len(mps["xyz"])
    assert (~o["in_view"].astype(bool)).sum() >= 0.1 * n
    for b, mk in masks.items():
        assert mk.sum() > 0 and not o["in_view"][mk].any(), b
    assert 0.2 * n < o["in_view"].sum() < n


def test_predict_scale_hand_computed_gpu(orbpl, oracle):
    """k_in_frustum's mnTrackScaleLevel against hand-computed PredictScale
    values (ratio = mfMaxDistance / dist, MapPoint.cc:421)."""
    from _scenes import predict_scale_problem
    cfg, T, mps, lev, ratio = predict_scale_problem()
    g = orbpl.frame_is_in_frustum(orbpl.make_camera(cfg), 1.2, 8, T, mps, 0.5)
    assert g["in_view"].all()
    assert np.array_equal(g["level"], lev)


@pytest.mark.parametrize("th,nnratio,claims", [(3.0, 0.8, True), (1.0, 0.6, False), (5.0, 0.8, True)])
def test_search_by_projection_local_bit_exact(orbpl, oracle, th, nnratio, claims):
    from _scenes import local_map_problem
    cfg, cam_o, sc, mps, cur, cur_nobs, T3 = local_map_problem(3)
    track = oracle.frame_is_in_frustum(cam_o, _log_scale(oracle), 8, T3, mps, 0.5)
    cn = cur_nobs if claims else None
    m_o, n_o = oracle.search_by_projection_local(cam_o, sc, cur, track, mps["desc"], mps["nobs"],
                                                 cn, th, nnratio)
    m_g, n_g = orbpl.ORBmatcher(nnratio).SearchByProjectionLocalMap(
        orbpl.make_camera(cfg), sc, cur, track, mps["desc"], mps["nobs"], cn, th)
    assert n_g == n_o and n_o > 100
    assert np.array_equal(m_g, m_o), np.nonzero(m_g != m_o)[0][:5]


@pytest.mark.parametrize("nt", ["1024", "512", "256", "128"])
def test_matcher_workgroup_widths_bit_exact(orbpl, oracle, nt, monkeypatch):
    """k_match_last (ORBPL_MATCH_NT) and k_match_local (ORBPL_LOCAL_NT; 128
    is not built for it) at every workgroup width they are built for: the
    same matches as the oracle (the launches pick 256 / 512-or-256 by batch)."""
    monkeypatch.setenv("ORBPL_MATCH_NT", nt)
    if nt != "128":
        monkeypatch.setenv("ORBPL_LOCAL_NT", nt)
    cfg, traj, fr = sequence(2, 5, cam_name="TUM3")
    cam_o = oracle.camera(cfg)
    f0 = frame_data(oracle, cam_o, cfg, *fr[0])
    f1 = frame_data(oracle, cam_o, cfg, *fr[1])
    T0 = np.linalg.inv(traj[0]).astype(np.float32)
    has = (f0["depth"] > 0).astype(np.uint8)
    xyz = _unproject_p6(cfg, f0["kps_un"], np.where(f0["depth"] > 0, f0["depth"], 0), T0)
    last = dict(Tcw=T0, kps_un=f0["kps_un"], has_mp=has, outlier=np.zeros(len(has), np.uint8),
                mp_xyz=xyz, mp_desc=f0["desc"], mp_nobs=np.ones(len(has), np.int32))
    cur = dict(Tcw=T0, kps_un=f1["kps_un"], desc=f1["desc"], uright=f1["uright"])
    sc = oracle.level_sizes(oracle.params(), 640, 480)[3]
    m_o, n_o = oracle.search_by_projection_last(cam_o, sc, cur, last, 15.0, False, True)
    m_g, n_g = orbpl.ORBmatcher(0.9, True).SearchByProjectionLastFrame(
        orbpl.make_camera(cfg), sc, cur, last, 15.0, False)
    assert n_g == n_o and n_o > 100 and np.array_equal(m_g, m_o)
    if nt == "128":
        return
    from _scenes import local_map_problem
    cfg, cam_o, sc, mps, cur, cur_nobs, T3 = local_map_problem(3)
    track = oracle.frame_is_in_frustum(cam_o, _log_scale(oracle), 8, T3, mps, 0.5)
    m_o, n_o = oracle.search_by_projection_local(cam_o, sc, cur, track, mps["desc"], mps["nobs"],
                                                 cur_nobs, 3.0, 0.8)
    m_g, n_g = orbpl.ORBmatcher(0.8).SearchByProjectionLocalMap(
        orbpl.make_camera(cfg), sc, cur, track, mps["desc"], mps["nobs"], cur_nobs, 3.0)
    assert n_g == n_o and n_o > 100 and np.array_equal(m_g, m_o)


def test_search_by_projection_local_many_points_bit_exact(orbpl, oracle):
    """More map points than one in-view window of k_match_local holds (4 x the
    keypoint capacity): the map tiled three times with a few descriptor bits
    flipped per copy, so copies compete for the same keypoints."""
    from _scenes import local_map_problem
    cfg, cam_o, sc, mps, cur, cur_nobs, T3 = local_map_problem(4)
    rng = np.random.default_rng(7)
    tiles = []
    for k in range(3):
        d = mps["desc"].copy()
        if k:
            flip = rng.integers(0, 256, (len(d), 2))
            for c in range(2):
                d[np.arange(len(d)), flip[:, c] // 8] ^= (1 << (flip[:, c] % 8)).astype(np.uint8)
        tiles.append(d)
    big = {key: np.concatenate([v] * 3) for key, v in mps.items()}
    big["desc"] = np.concatenate(tiles)
    assert len(big["xyz"]) > 4 * 1024
    track = oracle.frame_is_in_frustum(cam_o, _log_scale(oracle), 8, T3, big, 0.5)
    m_o, n_o = oracle.search_by_projection_local(cam_o, sc, cur, track, big["desc"], big["nobs"],
                                                 cur_nobs, 3.0, 0.8)
    m_g, n_g = orbpl.ORBmatcher(0.8).SearchByProjectionLocalMap(
        orbpl.make_camera(cfg), sc, cur, track, big["desc"], big["nobs"], cur_nobs, 3.0)
    assert n_g == n_o and n_o > 100
    assert np.array_equal(m_g, m_o), np.nonzero(m_g != m_o)[0][:5]


@pytest.mark.parametrize("case", ["local_map", "ref_kf", "retry"])
def test_line_search_by_projection_list_bit_exact(orbpl, oracle, case):
    from _scenes import line_map_problem
    cfg, cam_o, xyz, desc, ku, ld, cur_nobs, T2 = line_map_problem(5)
    cam_g = orbpl.make_camera(cfg)
    if case == "retry":   # a pose far off: few matches, the relaxed pass runs
        T0 = T2
        for off in (0.3, 0.6, 1.0, 2.0, 4.0):
            T2 = T0.copy()
            T2[:3, 3] += np.float32([off, 0.0, 0.5 * off])
            v = oracle.line_is_in_frustum(T2, xyz)
            if oracle.line_search_by_projection_list(cam_o, T2, ku, ld, cur_nobs, v, xyz, desc)[2]:
                break
    valid = oracle.line_is_in_frustum(T2, xyz)
    assert np.array_equal(orbpl.line_is_in_frustum(T2, xyz), valid)
    if case == "ref_kf":
        valid = np.ones(len(xyz), np.uint8)
        valid[::7] = 0
    cn = None if case == "ref_kf" else cur_nobs
    m_o, n_o, w_o = oracle.line_search_by_projection_list(cam_o, T2, ku, ld, cn, valid, xyz, desc)
    m_g, n_g, w_g = orbpl.LineMatcher.SearchByProjectionLocalMap(cam_g, T2, ku, ld, cn, valid, xyz,
                                                                 desc)
    assert (n_g, w_g) == (n_o, w_o)
    assert np.array_equal(m_g, m_o)
    if case == "retry":
        assert w_o
    else:
        assert n_o > 20 and not w_o


@pytest.mark.parametrize("bits,nnratio,ori", [(12, 0.7, True), (8, 0.75, True), (16, 0.7, False),
                                              (6, 0.9, True)])
def test_search_by_bow_bit_exact(orbpl, oracle, bits, nnratio, ori):
    from _scenes import bow_problem
    b = bow_problem(2, bits)
    m_o, n_o = oracle.search_by_bow(**b, nnratio=nnratio, check_ori=ori)
    m_g, n_g = orbpl.ORBmatcher(nnratio, ori).SearchByBoW(**b)
    assert n_g == n_o and n_o > 20
    assert np.array_equal(m_g, m_o)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_stereo_matches_bit_exact(orbpl, oracle, seed):
    """Frame::ComputeStereoMatches on the GPU pyramids of both extractors vs
    the oracle on its own pyramids: uRight and depth bit-exact."""
    from _scenes import stereo_pair
    cfg, left, right = stereo_pair(seed)
    W, H = cfg["width"], cfg["height"]
    exl = orbpl.ORBextractor(2000, 1.2, 8, 20, 7, width=W, height=H)
    exr = orbpl.ORBextractor(2000, 1.2, 8, 20, 7, width=W, height=H)
    kl, dl = exl(left)
    kr, dr = exr(right)
    ur_g, d_g = orbpl.stereo_matches(orbpl.make_camera(cfg), exl, exr, kl, dl, kr, dr)
    p = oracle.params(2000, 1.2, 8, 20, 7)
    ur_o, d_o = oracle.stereo_matches(oracle.camera(cfg), p, left, right, kl, dl, kr, dr)
    assert (d_o > 0).sum() > 0.3 * len(kl)
    assert np.array_equal(_u32(ur_g), _u32(ur_o)), np.nonzero(_u32(ur_g) != _u32(ur_o))[0][:5]
    assert np.array_equal(_u32(d_g), _u32(d_o))
    # no right keypoints: nothing matches
    ur0, d0 = orbpl.stereo_matches(orbpl.make_camera(cfg), exl, exr, kl, dl, kr[:0], dr[:0])
    assert np.all(ur0 == -1) and np.all(d0 == -1)


@pytest.mark.parametrize("lines,stereo,pipelined,fixed", [
    (False, False, False, False), (True, False, False, False), (True, False, True, True),
    (True, True, False, True)])
def test_tracker_local_map_matches_oracle(orbpl, oracle, lines, stereo, pipelined, fixed):
    """TrackWithMotionModel + TrackLocalMap (ORBPL_TRACK_LOCAL_MAP, defined
    local map P18: the last 4 frames' map points / lines) against the oracle
    LVO loop with the same flags: every frame's 8 tracking counts and the 4
    TrackLocalMap counts identical, pose within POSE_TOL, through 6 frames
    (the ring fills and wraps)."""
    from _scenes import stereo_sequence
    S, F = 2, 6
    if stereo:
        seqs = [stereo_sequence(F, 70 + s) for s in range(S)]
        orb = (2000, 1.2, 8, 20, 7)
    else:
        seqs = [sequence(F, 80 + s, cam_name="TUM3" if lines else "TUM1") for s in range(S)]
        orb = (1000, 1.2, 8, 20, 7)
    cfg = seqs[0][0]
    W, H = cfg["width"], cfg["height"]
    flags = oracle.TRACK_LOCAL_MAP | (oracle.TRACK_FIXED_LINE_JAC if fixed else 0)
    lvo = oracle.LVO(oracle.params(*orb), oracle.camera(cfg), S, use_lines=lines, flags=flags)
    tr = orbpl.Tracker(orbpl.OrbParams(*orb), orbpl.make_camera(cfg), S, lines=lines, stereo=stereo,
                       local_map=True, fixed_line_jac=fixed)
    tr.set_pipelined(pipelined)
    T0 = np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs])
    lvo.reset(T0.reshape(S, 16))
    tr.reset(T0.reshape(S, 16))
    tr.set_history(F)
    # one device slot per frame: pipelined steps return before extraction has
    # read its input, so a reused upload buffer would race the next upload
    fa, fb = S * W * H, S * W * H * (1 if stereo else 4)
    a = orbpl.DeviceBuffer(F * fa)
    b = orbpl.DeviceBuffer(F * fb)
    keys = ("nkeypoints", "nmatches", "ninliers", "nmatches_map", "ok", "nlines", "line_matches",
            "line_nmatches_map")
    lkeys = ("local_matches", "local_inliers", "local_line_matches", "local_line_inliers")
    ref = [[None] * F for _ in range(S)]
    for f in range(F):
        a.upload(np.stack([sq[2][f][0] for sq in seqs]), offset=f * fa)
        b.upload(np.stack([sq[2][f][1] for sq in seqs]), offset=f * fb)
        if stereo:
            tr.step_stereo_device(a.ptr + f * fa, b.ptr + f * fb)
        else:
            tr.step_device(a.ptr + f * fa, b.ptr + f * fb)
        if not pipelined:
            tr.synchronize()
        for s in range(S):
            g, d = seqs[s][2][f]
            To, so = lvo.step_stereo(s, g, d) if stereo else lvo.step(s, g, d)
            ref[s][f] = (To, [so[k] for k in keys] + [lvo.local_stats(s)[k] for k in lkeys])
    tr.synchronize()
    for s in range(S):
        Th, Ch = tr.history(s)
        assert len(Th) == F
        for f in range(F):
            To, co = ref[s][f]
            assert [int(x) for x in Ch[f]] == co, (s, f, list(Ch[f]), co)
            assert np.abs(Th[f] - To).max() < POSE_TOL, (s, f)
        assert ref[s][F - 1][1][8] > 0       # local map matches were found
        assert ref[s][F - 1][1][4] == 1      # and tracking succeeded


@pytest.mark.parametrize("lines", [False, True])
def test_tracker_step_host_u16_depth(orbpl, oracle, lines):
    """orbpl_tracker_step_host: frames from pinned host memory, 16-bit TUM
    depth converted on the device as imDepth.convertTo(CV_32F, 1/5000)
    (pinned P21), pipelined: the same counts and poses as the oracle loop on
    the converted depth."""
    S, F = 2, 4
    seqs = [sequence(F, 60 + s, cam_name="TUM3" if lines else "TUM1") for s in range(S)]
    cfg = seqs[0][0]
    scale = np.float32(1.0) / np.float32(5000.0)
    lvo = oracle.LVO(oracle.params(), oracle.camera(cfg), S, use_lines=lines)
    tr = orbpl.Tracker(orbpl.OrbParams(1000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S, lines=lines)
    tr.set_pipelined(True)
    T0 = np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs])
    lvo.reset(T0.reshape(S, 16))
    tr.reset(T0.reshape(S, 16))
    tr.set_history(F)
    hg, hd, d32 = [], [], []
    for f in range(F):
        g = orbpl.HostBuffer((S, 480, 640), np.uint8)
        d = orbpl.HostBuffer((S, 480, 640), np.uint16)
        g.array[:] = np.stack([sq[2][f][0] for sq in seqs])
        d.array[:] = np.clip(np.round(np.stack([sq[2][f][1] for sq in seqs]) * 5000.0), 0, 65535)
        hg.append(g)
        hd.append(d)
        d32.append(d.array.astype(np.float32) * scale)
        tr.step_host(g.ptr, d.ptr, 5000.0)
    tr.synchronize()
    for s in range(S):
        Th, Ch = tr.history(s)
        for f in range(F):
            To, so = lvo.step(s, seqs[s][2][f][0], np.ascontiguousarray(d32[f][s]))
            keys = ("nkeypoints", "nmatches", "ninliers", "nmatches_map", "ok", "nlines",
                    "line_matches", "line_nmatches_map")
            assert [int(x) for x in Ch[f][:8]] == [so[k] for k in keys], (s, f)
            assert np.abs(Th[f] - To).max() < POSE_TOL, (s, f)
    for b in hg + hd:
        b.free()


@pytest.mark.parametrize("lines,local_map,pipelined", [(False, False, False), (False, True, True),
                                                       (True, True, False), (True, False, True)])
def test_tracker_refkf_matches_oracle(orbpl, oracle, lines, local_map, pipelined):
    """ORBPL_TRACK_REFKF (P22): the first tracked frame and every motion-model
    failure go through TrackReferenceKeyFrame (SearchByBoW on the frames'
    device-computed FeatureVectors + the reference-keyframe line search +
    pose); every frame's counts and the TRK choice identical to the oracle
    loop, pose within POSE_TOL. Stream 1's frame 3 is its image turned by
    180 degrees: the motion model fails there (and after it), so
    TrackReferenceKeyFrame runs on a failure too."""
    from _vocab import vocabulary
    path, _ = vocabulary(k=10, L=5, seed=3, n_frames=8)
    voc = orbpl.ORBVocabulary(path)
    ovoc = oracle.Vocabulary(path)
    S, F = 2, 5
    seqs = [sequence(F, 90 + s, cam_name="TUM3" if lines else "TUM1") for s in range(S)]
    frames = [[sq[2][f] for f in range(F)] for sq in seqs]
    g3, d3 = frames[1][3]
    frames[1][3] = (np.ascontiguousarray(g3[::-1, ::-1]), np.ascontiguousarray(d3[::-1, ::-1]))
    cfg = seqs[0][0]
    flags = oracle.TRACK_REFKF | (oracle.TRACK_LOCAL_MAP if local_map else 0)
    lvo = oracle.LVO(oracle.params(), oracle.camera(cfg), S, use_lines=lines, flags=flags)
    lvo.set_vocabulary(ovoc)
    tr = orbpl.Tracker(orbpl.OrbParams(1000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S, lines=lines,
                       local_map=local_map, refkf=True)
    tr.set_vocabulary(voc, 4)
    tr.set_pipelined(pipelined)
    T0 = np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs])
    lvo.reset(T0.reshape(S, 16))
    tr.reset(T0.reshape(S, 16))
    tr.set_history(F)
    fa, fb = S * 640 * 480, S * 640 * 480 * 4
    a = orbpl.DeviceBuffer(F * fa)
    b = orbpl.DeviceBuffer(F * fb)
    keys = ("nkeypoints", "nmatches", "ninliers", "nmatches_map", "ok", "nlines", "line_matches",
            "line_nmatches_map")
    lkeys = ("local_matches", "local_inliers", "local_line_matches", "local_line_inliers")
    trk_seen = 0
    for f in range(F):
        a.upload(np.stack([frames[s][f][0] for s in range(S)]), offset=f * fa)
        b.upload(np.stack([frames[s][f][1] for s in range(S)]), offset=f * fb)
        tr.step_device(a.ptr + f * fa, b.ptr + f * fb)
        gtrk = tr.trk()
        for s in range(S):
            To, so = lvo.step(s, *frames[s][f])
            assert int(gtrk[s]) == lvo.trk(s), (s, f)
            trk_seen += lvo.trk(s)
            if s == 1 and f >= 3:
                assert lvo.trk(s) == 1, f      # the motion model failed
            Th, Ch = tr.history(s)
            ref = [so[k] for k in keys] + [lvo.local_stats(s)[k] for k in lkeys]
            assert [int(x) for x in Ch[f]] == ref, (s, f, list(Ch[f]), ref)
            assert np.abs(Th[f] - To).max() < POSE_TOL, (s, f)
    assert trk_seen >= S + 2    # every stream's first tracked frame, and the failures


@pytest.mark.parametrize("mode,case", [(0, "plain"), (0, "observed"), (0, "retry"), (1, "plain"),
                                       (1, "retry")])
def test_line_search_pairs_bit_exact(orbpl, oracle, mode, case):
    """orbl_search_by_projection_pairs (the reference's harness overloads,
    LineMatcher.cpp:272-487 / 954-1170) against oracle_line_search_pairs:
    match, count, wiped, the projected KeyLines (new_kls) and every pair
    (match_indices) byte for byte; 'observed' gives map lines Observations()
    so the last-frame variant's per-pair skip runs, 'retry' a pose far off."""
    from _scenes import line_map_problem
    cfg, cam_o, xyz, desc, ku, ld, cur_nobs, T2 = line_map_problem(5)
    cam_g = orbpl.make_camera(cfg)
    n = len(xyz)
    rng = np.random.default_rng(3)
    valid = (rng.random(n) < 0.9).astype(np.uint8)
    base = np.zeros(n, ku.dtype) if mode == 0 else None
    if mode == 0:
        base = np.resize(ku, n).copy()
    ml_nobs = (np.arange(n) % 3 == 0).astype(np.int32) if case == "observed" else None
    if case == "retry":
        T2 = T2.copy()
        T2[:3, 3] += np.float32([0.4, 0.0, 0.2])
    cn = cur_nobs if mode == 1 else None
    o = oracle.line_search_pairs(cam_o, T2, mode, ku, ld, cn, valid, base, xyz, desc, ml_nobs)
    g = orbpl.LineMatcher.SearchByProjectionPairs(cam_g, T2, mode, ku, ld, cn, valid, base, xyz,
                                                  desc, ml_nobs)
    assert g[1:3] == o[1:3]
    assert np.array_equal(g[0], o[0])
    assert g[3].tobytes() == o[3].tobytes() and np.array_equal(g[4], o[4])
    assert np.array_equal(g[5], o[5])
    assert len(o[3]) > 10
    if case == "retry":
        assert o[2] and o[1] > 5


def test_line_bf_knn_bit_exact(orbpl, oracle):
    """orbl_match_bf_knn (LineMatcher.cpp:492-525) against the oracle on two
    frames' LBD rows, both directions."""
    from _scenes import line_map_problem
    cfg, cam_o, xyz, desc, ku, ld, cur_nobs, T2 = line_map_problem(5)
    for q, t in ((desc[:80], ld), (ld, desc[:80])):
        og, ng = orbpl.LineMatcher.MatchBFKnn(q, t)
        oo, no = oracle.line_match_bf_knn(q, t)
        assert ng == no and np.array_equal(og, oo)
        assert no > 0
