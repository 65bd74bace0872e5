"""ORBPL_TRACK_MAP: Tracking::Track with the reference's map model on the
device (map_kernels.hip) against the oracle's restatement (map_oracle.cpp,
pinned P23-P25): every step's 24 counts identical (matches, inliers, the
TrackLocalMap counts, keyframe decisions, map sizes, temporal points / lines,
the TrackReferenceKeyFrame choice, the reference keyframe, the state and the
local map sizes), poses within POSE_TOL."""
import numpy as np
import pytest

from _scenes import sequence

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4   # north_star: pose within 1e-4 RMSE (max-abs used here: stricter)


def _vocab_arrays(L, seed=3):
    """A seeded k = 10 vocabulary of depth L as arrays (no text round trip:
    L = 6 has 1.1M nodes, ORB-SLAM2's ORBvoc shape)."""
    import orbpl.synth as synth
    from _vocab import training_descriptors
    tree = synth.vocabulary_tree(training_descriptors(8), k=10, L=L, seed=seed)
    return dict(parent=tree["parent"], leaf=tree["leaf"], desc=tree["desc"], weight=tree["weight"],
                k=10, L=L, scoring=0, weighting=0)


def _run(orbpl, oracle, lines, refkf, S, F, seed, turn=None, pipelined=False, clears=None,
         vocab_levels=5, stereo=False, fps=None, thdepth=None, nseq=None):
    """clears: {frame: [streams]} whose velocity is cleared before that
    frame's step (orbpl_tracker_clear_velocity / MapVO.clear_velocity).
    stereo: KITTI 00 rectified pairs (2000 features) through
    orbpl_tracker_step_stereo / MapVO.step_stereo."""
    clears = clears or {}
    nseq = nseq or S    # stream s renders sequence seed + (s mod nseq)
    if stereo:
        from _scenes import stereo_sequence
        seqs = [stereo_sequence(F, seed + s % nseq) for s in range(S)]
    else:
        seqs = [sequence(F, seed + s % nseq, cam_name="TUM3" if lines else "TUM1") for s in range(S)]
    frames = [[sq[2][f] for f in range(F)] for sq in seqs]
    if turn is not None:
        s, f0 = turn
        for f in range(f0, F):
            g, d = frames[s][f]
            frames[s][f] = (np.ascontiguousarray(g[::-1, ::-1]), np.ascontiguousarray(d[::-1, ::-1]))
    cfg = dict(seqs[0][0])
    if thdepth is not None:
        cfg["thdepth"] = thdepth   # ThDepth: the close / far split of NeedNewKeyFrame
    flags = (oracle.TRACK_REFKF if refkf else 0) | (oracle.TRACK_STEREO if stereo else 0)
    nf = 2000 if stereo else 1000
    W, H = cfg.get("width", 640), cfg.get("height", 480)
    mvo = oracle.MapVO(oracle.params(nf), oracle.camera(cfg), S, use_lines=lines, flags=flags)
    tr = orbpl.Tracker(orbpl.OrbParams(nf, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S, lines=lines,
                       refkf=refkf, map=True, stereo=stereo)
    if fps is not None:
        mvo.set_fps(fps)
        tr.set_fps(fps)
    if refkf and vocab_levels != 5:
        arr = _vocab_arrays(vocab_levels)
        voc = orbpl.ORBVocabulary(arrays=arr)
        mvo.set_vocabulary(oracle.Vocabulary(arrays=arr))
        tr.set_vocabulary(voc, 4)
    elif refkf:
        from _vocab import vocabulary
        path, _ = vocabulary(k=10, L=5, seed=3, n_frames=8)
        voc = orbpl.ORBVocabulary(path)
        mvo.set_vocabulary(oracle.Vocabulary(path))
        tr.set_vocabulary(voc, 4)
    tr.set_pipelined(pipelined)
    T0 = np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs])
    mvo.reset(T0.reshape(S, 16))
    tr.reset(T0.reshape(S, 16))
    tr.set_history(F)
    fa = S * W * H
    fb = fa if stereo else fa * 4   # right image (u8) or depth (f32)
    a = orbpl.DeviceBuffer(F * fa)
    b = orbpl.DeviceBuffer(F * fb)
    for f in range(F):
        a.upload(np.stack([frames[s][f][0] for s in range(S)]), offset=f * fa)
        b.upload(np.stack([frames[s][f][1] for s in range(S)]), offset=f * fb)
        if f in clears:
            tr.clear_velocity(np.isin(np.arange(S), clears[f]))
        if stereo:
            tr.step_stereo_device(a.ptr + f * fa, b.ptr + f * fb)
        else:
            tr.step_device(a.ptr + f * fa, b.ptr + f * fb)
    tr.synchronize()
    ref = [[None] * F for _ in range(S)]
    ostep = mvo.step_stereo if stereo else mvo.step
    for s in range(S):
        for f in range(F):
            if s in clears.get(f, ()):
                mvo.clear_velocity(s)
            ref[s][f] = ostep(s, *frames[s][f])
    keys = orbpl.Tracker.MAP_COUNTS
    assert tuple(keys) == tuple(oracle.MAP_COUNTS)
    out = []
    for s in range(S):
        Th, _ = tr.history(s)
        Ch = tr.map_history(s)
        assert len(Th) == F and len(Ch) == F
        for f in range(F):
            To, co = ref[s][f]
            want = [co[k] for k in keys]
            got = [int(x) for x in Ch[f]]
            assert got == want, (s, f, [(k, g, w) for k, g, w in zip(keys, got, want) if g != w])
            assert np.abs(Th[f] - To).max() < POSE_TOL, (s, f, np.abs(Th[f] - To).max())
        out.append([r[1] for r in ref[s]])
        _same_map(tr, mvo, s, lines)
    assert (tr.map_errors() == 0).all()
    return out


def _same_map(tr, mvo, s, lines):
    """The stream's map after the sequence equals the oracle's element by
    element: keyframe parents and covisibility orders, and per map point /
    line (same pool ids: both create them in the reference's order) nObs,
    the distinctive descriptor, the position, the normal and the distance
    bounds - bit for bit."""
    par, ords = tr.map_keyframes(s)
    opar, oords = mvo.keyframes(s)
    assert np.array_equal(par, opar), (s, par, opar)
    assert len(ords) == len(oords) and all(np.array_equal(a, b) for a, b in zip(ords, oords)), s
    P = tr.map_points(s)
    onobs, odesc, oxyz = mvo.points(s)
    onrm, od2 = mvo.points_geom(s)
    assert len(P["nobs"]) == len(onobs), s
    assert np.array_equal(P["nobs"], onobs), s
    assert np.array_equal(P["desc"], odesc), s
    assert np.array_equal(P["xyz"].view(np.uint32), oxyz.view(np.uint32)), s
    assert np.array_equal(P["normal"].view(np.uint32), onrm.view(np.uint32)), s
    assert np.array_equal(P["dist"].view(np.uint32), od2.view(np.uint32)), s
    if lines:
        Lm = tr.map_lines(s)
        lnobs, ldesc, lpos = mvo.lines(s)
        assert np.array_equal(Lm["nobs"], lnobs) and np.array_equal(Lm["desc"], ldesc), s
        assert np.array_equal(Lm["pos"].view(np.uint32), lpos.view(np.uint32)), s


@pytest.mark.parametrize("lines,refkf,pipelined,seed", [(True, True, False, 110),
                                                        (False, True, True, 140),
                                                        (True, False, True, 110)])
def test_map_tracker_matches_oracle(orbpl, oracle, lines, refkf, pipelined, seed):
    """Initialisation, motion model / reference keyframe, covisibility local
    map, keyframe insertion: 8 frames of 2 streams, every count identical."""
    res = _run(orbpl, oracle, lines, refkf, S=2, F=8, seed=seed, pipelined=pipelined)
    for r in res:
        assert r[0]["keyframe"] == 2 and r[0]["state"] == 1      # StereoInitialization
        assert all(c["ok"] == 1 for c in r[1:])
        assert r[-1]["local_points"] > 0                          # the covisibility local map
    assert any(c["keyframe"] == 1 for r in res for c in r[1:])    # CreateNewKeyFrame ran
    if refkf:
        assert all(r[1]["trk"] == 1 for r in res)                 # no velocity yet


def test_map_tracker_lost_and_reset(orbpl, oracle):
    """A stream whose images turn by 180 degrees mid-sequence: the trackers
    fail, go LOST and reset (<= 5 keyframes), then initialise again -- the same
    states, counts and poses as the oracle."""
    res = _run(orbpl, oracle, True, True, S=2, F=8, seed=130, turn=(1, 4))
    st = [c["state"] for c in res[1]]
    assert 2 in st or 0 in st[4:], st


def test_map_tracker_long_sequence(orbpl, oracle):
    """16 frames of 3 streams (points + lines, TrackReferenceKeyFrame,
    pipelined): several keyframes per stream, covisibility orders and spanning
    tree, the maps equal element by element."""
    res = _run(orbpl, oracle, True, True, S=3, F=16, seed=150, pipelined=True)
    for r in res:
        assert all(c["ok"] == 1 for c in r)
    assert max(r[-1]["keyframes"] for r in res) >= 4


def test_map_capacity_flag(orbpl, oracle, monkeypatch):
    """A keyframe table of 2 slots: NeedNewKeyFrame wants a third keyframe,
    the tracker declines it and reports capacity flag 1 (the map no longer
    matches the reference's)."""
    monkeypatch.setenv("ORBPL_MAP_KF", "2")
    S, F = 2, 8
    seqs = [sequence(F, 130 + s, cam_name="TUM3") for s in range(S)]   # stream 0: 4 keyframes
    cfg = seqs[0][0]
    tr = orbpl.Tracker(orbpl.OrbParams(1000, 1.2, 8, 20, 7), orbpl.make_camera(cfg), S, lines=True,
                       map=True)
    tr.reset(np.stack([np.linalg.inv(sq[1][0]).astype(np.float32) for sq in seqs]).reshape(S, 16))
    fa, fb = S * 640 * 480, S * 640 * 480 * 4
    a = orbpl.DeviceBuffer(fa)
    b = orbpl.DeviceBuffer(fb)
    for f in range(F):
        a.upload(np.stack([seqs[s][2][f][0] for s in range(S)]))
        b.upload(np.stack([seqs[s][2][f][1] for s in range(S)]))
        tr.step_device(a.ptr, b.ptr)
        tr.synchronize()
    err = tr.map_errors()
    assert (err & 1).any(), err
    assert all(tr.map_keyframes(s)[0].shape[0] <= 2 for s in range(S))


@pytest.mark.parametrize("lines,vocab_levels,pipelined", [(False, 5, True), (True, 6, False),
                                                          (False, 6, True)])
def test_map_tracker_reference_keyframe_under_load(orbpl, oracle, lines, vocab_levels, pipelined):
    """TrackReferenceKeyFrame for many streams at once: velocities cleared
    for half the streams at frame 3 and for all at frame 5 (as after a
    relocalisation), so those frames run SearchByBoW + the reference-keyframe
    pose; with a 6-level vocabulary (ORBvoc's depth: FeatureVector nodes at
    level 2) and a 5-level one. Every count, pose and the maps equal the
    oracle's."""
    S = 4
    res = _run(orbpl, oracle, lines, True, S=S, F=7, seed=170, pipelined=pipelined,
               clears={3: [1, 3], 5: list(range(S))}, vocab_levels=vocab_levels)
    for s, r in enumerate(res):
        assert r[5]["trk"] == 1
        assert r[3]["trk"] == (1 if s in (1, 3) else r[3]["trk"])
        assert r[5]["ok"] == 1 and r[5]["nmatches"] >= 15, r[5]


@pytest.mark.parametrize("lines,refkf,pipelined", [(True, True, False), (False, True, True),
                                                   (True, False, True)])
def test_map_tracker_stereo_matches_oracle(orbpl, oracle, lines, refkf, pipelined):
    """The map model on KITTI 00 stereo pairs (configs[3]): ComputeStereoMatches
    depths, P17 line depths, the STEREO branches of Track() (radius 7 / 1,
    outliers leave the frame after TrackLocalMap), Camera.fps 10: every count
    and pose of 8 frames of 2 streams and the maps equal the oracle's (the
    slow synthetic KITTI motion inserts no keyframe in 8 frames: keyframe
    insertion is covered on RGB-D above and by the bench's stereo leg)."""
    res = _run(orbpl, oracle, lines, refkf, S=2, F=8, seed=60, pipelined=pipelined, stereo=True,
               fps=10)
    for r in res:
        assert r[0]["keyframe"] == 2 and r[0]["state"] == 1      # StereoInitialization
        assert all(c["ok"] == 1 for c in r[1:])
        assert r[-1]["local_points"] > 0 and r[-1]["temporal_points"] > 0   # UpdateLastFrame


@pytest.mark.parametrize("lines,pipelined", [(False, True), (True, False)])
def test_map_tracker_stereo_keyframe_after_outliers(orbpl, oracle, lines, pipelined):
    """A stereo keyframe inserted on a frame whose TrackLocalMap found
    outliers: CreateNewKeyFrame's close-point pass (Tracking.cc:1583-1660)
    runs before Track() drops the outliers' map points (Tracking.cc:547-555),
    and the next frames track against what it created. ThDepth 5 (2.7 m)
    makes most of the room's points far, so frame 4 of stream 0 needs a
    keyframe (nTrackedClose < 100 and nNonTrackedClose > 70,
    Tracking.cc:1465-1480); the oracle inserts it there
    (tests/_scenes.stereo_sequence, seed 60). Every count, pose and both maps
    equal the oracle's."""
    res = _run(orbpl, oracle, lines, True, S=2, F=6, seed=60, pipelined=pipelined, stereo=True,
               fps=10, thdepth=5.0)
    r = res[0]
    kf = [f for f in range(1, 6) if r[f]["keyframe"] == 1]
    assert kf, [c["keyframe"] for c in r]
    assert any(r[f]["ninliers"] < r[f]["nmatches"] for f in range(1, kf[0] + 1)), r
    assert r[kf[0]]["map_points"] > r[0]["map_points"]
    assert all(c["ok"] == 1 for c in r[1:])


@pytest.mark.parametrize("groups", ["1/2/3", "1/3/5"])
def test_map_tracker_level_pipeline_64_streams(orbpl, oracle, monkeypatch, groups):
    """The ORB level pipeline (per-group pyramid / FAST / octree launches on a
    second stream, orbpl_runtime.cpp; on for batches of >= 64 frames) forced
    on (ORBPL_LEVEL_PIPE=1, whatever the box's queue count) in a 64-stream
    tracker: every stream's counts, poses and map equal the oracle's."""
    monkeypatch.setenv("ORBPL_LEVEL_PIPE", "1")
    monkeypatch.setenv("ORBPL_LEVEL_GROUPS", groups)
    res = _run(orbpl, oracle, False, False, S=64, F=3, seed=190, pipelined=True, nseq=8)
    assert all(c["ok"] == 1 for r in res for c in r[1:])
