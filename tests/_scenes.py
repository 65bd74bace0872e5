"""Seeded test problems for the tracking half (frame glue, matcher, pose),
built with the CPU oracle's extraction so GPU and oracle see identical
inputs."""
import functools

import numpy as np

from _pkg import load_oracle, load_pkg


@functools.lru_cache(maxsize=8)
def sequence(n=3, seed=0, cam_name="TUM1", width=640, height=480):
    load_pkg()
    import orbpl.synth as synth
    cfg = dict(getattr(synth, cam_name))
    if (width, height) != (cfg["width"], cfg["height"]):
        cfg.update(width=width, height=height)
    room = synth.default_room(seed)
    traj = synth.trajectory(n, seed=seed)
    frames = [synth.render(cfg, T, room, seed=seed * 100 + i) for i, T in enumerate(traj)]
    return cfg, traj, frames


def frame_data(O, cam, cfg, gray, depth, orb=(1000, 1.2, 8, 20, 7)):
    p = O.params(*orb)
    kps, desc, _ = O.extract(p, gray)
    ku, d, ur, gc, b = O.frame_prepare(cam, kps, depth)
    return dict(kps=kps, desc=desc, kps_un=ku, depth=d, uright=ur, gcell=gc, bounds=b)


def unproject(cam_cfg, ku, depth, Tcw):
    """Frame::UnprojectStereo in numpy (float64 is fine for test inputs)."""
    z = depth.astype(np.float64)
    x = (ku["x"] - cam_cfg["cx"]) * z / cam_cfg["fx"]
    y = (ku["y"] - cam_cfg["cy"]) * z / cam_cfg["fy"]
    Pc = np.stack([x, y, z], 1)
    Twc = np.linalg.inv(Tcw.astype(np.float64))
    return (Pc @ Twc[:3, :3].T + Twc[:3, 3]).astype(np.float32)


def perturb(T, dt=0.01, dr=0.01, seed=0):
    rng = np.random.default_rng(seed)
    w = rng.normal(size=3) * dr
    th = np.linalg.norm(w)
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]) / max(th, 1e-12)
    R = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    P = np.eye(4)
    P[:3, :3] = R
    P[:3, 3] = rng.normal(size=3) * dt
    return (P @ T).astype(np.float32)


def match_problem(seed=0, nobs_zero_frac=0.0, outlier_frac=0.0, pert=(0.01, 0.01)):
    """(cam, scale, cur, last) for SearchByProjection(cur, last) from frames
    0 -> 1 of a seeded sequence; the last frame's map points come from its
    depth at the true pose, the current pose is the truth perturbed."""
    O = load_oracle()
    cfg, traj, frames = sequence(3, seed)
    cam = O.camera(cfg)
    f0 = frame_data(O, cam, cfg, *frames[0])
    f1 = frame_data(O, cam, cfg, *frames[1])
    T0 = np.linalg.inv(traj[0]).astype(np.float32)
    T1 = np.linalg.inv(traj[1]).astype(np.float32)
    rng = np.random.default_rng(seed + 7)
    n0 = len(f0["kps"])
    has = (f0["depth"] > 0).astype(np.uint8)
    xyz = unproject(cfg, f0["kps_un"], np.where(f0["depth"] > 0, f0["depth"], 1.0), T0)
    nobs = np.where(rng.random(n0) < nobs_zero_frac, 0, 1).astype(np.int32)
    outl = (rng.random(n0) < outlier_frac).astype(np.uint8)
    last = dict(Tcw=T0, kps_un=f0["kps_un"], has_mp=has, outlier=outl, mp_xyz=xyz,
                mp_desc=f0["desc"], mp_nobs=nobs)
    cur = dict(Tcw=perturb(T1, *pert, seed=seed), kps_un=f1["kps_un"], desc=f1["desc"],
               uright=f1["uright"])
    lw, lh, nf, sc, isc = O.level_sizes(O.params(), 640, 480)
    return cfg, cam, sc, cur, last, (f0, f1, T0, T1)


def local_map_problem(seed=0, cam_name="TUM1", nobs_zero_frac=0.1, cur_claim_frac=0.2):
    """A local map for SearchLocalPoints: map points from frames 0 and 1 of a
    seeded sequence (world position from depth at the true pose, normal and
    scale-invariance distances as MapPoint::UpdateNormalAndDepth sets them,
    keypoint descriptor, Observations()), the current frame = frame 3 at its
    true pose, and some current keypoints already holding a map point."""
    O = load_oracle()
    cfg, traj, frames = sequence(4, seed, cam_name=cam_name)
    cam = O.camera(cfg)
    lw, lh, nf, sc, isc = O.level_sizes(O.params(), cfg["width"], cfg["height"])
    rng = np.random.default_rng(seed + 11)
    xyz, nrm, dmin, dmax, desc, nobs = [], [], [], [], [], []
    for k in (0, 1):
        fd = frame_data(O, cam, cfg, *frames[k])
        Tk = np.linalg.inv(traj[k]).astype(np.float32)
        ok = fd["depth"] > 0
        P = unproject(cfg, fd["kps_un"][ok], fd["depth"][ok], Tk)
        Ow = traj[k][:3, 3].astype(np.float64)
        v = P.astype(np.float64) - Ow
        d = np.linalg.norm(v, axis=1)
        mx = (d * sc[fd["kps_un"]["octave"][ok]]).astype(np.float32)
        xyz.append(P)
        nrm.append((v / d[:, None]).astype(np.float32))
        dmax.append(mx)
        dmin.append((mx / sc[-1]).astype(np.float32))
        desc.append(fd["desc"][ok])
        nobs.append(np.where(rng.random(ok.sum()) < nobs_zero_frac, 0,
                             rng.integers(1, 4, ok.sum())).astype(np.int32))
    mps = dict(xyz=np.concatenate(xyz), normal=np.concatenate(nrm), min_dist=np.concatenate(dmin),
               max_dist=np.concatenate(dmax), desc=np.concatenate(desc), nobs=np.concatenate(nobs))
    f3 = frame_data(O, cam, cfg, *frames[3])
    cur = dict(kps_un=f3["kps_un"], desc=f3["desc"], uright=f3["uright"])
    cur_nobs = np.where(rng.random(len(f3["kps_un"])) < cur_claim_frac, 1, 0).astype(np.int32)
    T3 = np.linalg.inv(traj[3]).astype(np.float32)
    return cfg, cam, sc, mps, cur, cur_nobs, T3


def frustum_reject_problem(seed=0, frac=0.05):
    """local_map_problem's map points with disjoint subsets (each `frac` of
    them) moved so that each Frame::IsInFrustum rejection (Frame.cc:345-401)
    fires: behind the camera (Pc.z < 0), outside the image bounds, distance
    above 1.2 mfMaxDistance, distance below 0.8 mfMinDistance, view cosine
    below 0.5 (normal turned against the viewing ray). Returns
    local_map_problem's tuple plus {branch: mask}."""
    cfg, cam, sc, mps, cur, cur_nobs, T = local_map_problem(seed)
    mps = {k: v.copy() for k, v in mps.items()}
    n = len(mps["xyz"])
    rng = np.random.default_rng(seed + 101)
    order = rng.permutation(n)
    m = int(frac * n)
    names = ("behind", "outside", "far", "near", "view_cos")
    sel = {b: order[i * m:(i + 1) * m] for i, b in enumerate(names)}
    T64 = T.astype(np.float64)
    R, t = T64[:3, :3], T64[:3, 3]
    Ow = -R.T @ t
    P = mps["xyz"].astype(np.float64)
    Pc = P @ R.T + t
    # behind the camera: mirror the camera-frame point through the image plane
    i = sel["behind"]
    Pb = Pc[i] * np.array([1.0, 1.0, -1.0])
    mps["xyz"][i] = ((Pb - t) @ R).astype(np.float32)
    # outside the image: shift along x by more than the image width at its depth
    i = sel["outside"]
    Po = Pc[i] + np.stack([np.abs(Pc[i, 2]) * (1.5 * cfg["width"] / cfg["fx"]),
                           np.zeros(len(i)), np.zeros(len(i))], 1)
    mps["xyz"][i] = ((Po - t) @ R).astype(np.float32)
    dist = np.linalg.norm(P - Ow, axis=1)
    # distance out of [0.8 min, 1.2 max]
    i = sel["far"]
    mps["max_dist"][i] = (dist[i] / 1.5).astype(np.float32)
    mps["min_dist"][i] = (mps["max_dist"][i] / sc[-1]).astype(np.float32)
    i = sel["near"]
    mps["min_dist"][i] = (dist[i] / 0.6).astype(np.float32)
    mps["max_dist"][i] = (mps["min_dist"][i] * sc[-1]).astype(np.float32)
    # view cosine -1: the normal points along the ray from the camera
    i = sel["view_cos"]
    mps["normal"][i] = (-(P[i] - Ow) / dist[i, None]).astype(np.float32)
    masks = {}
    for b, i in sel.items():
        mk = np.zeros(n, bool)
        mk[i] = True
        masks[b] = mk
    return cfg, cam, sc, mps, cur, cur_nobs, T, masks


def line_map_problem(seed=0, cam_name="TUM1", claim_frac=0.15):
    """Map lines from frames 0 and 1 (end points unprojected with their own
    depths at the true poses, LBD rows), the current frame 2's undistorted key
    lines and LBD rows at its true pose, and some current lines already
    holding a map line with Observations() > 0."""
    O = load_oracle()
    cfg, traj, frames = sequence(3, seed, cam_name=cam_name)
    cam = O.camera(cfg)
    xyz, desc = [], []
    for k in (0, 1):
        g, d = frames[k]
        kl, ld, _, _ = O.line_extract(g)
        ku, ds, de, _, _ = O.line_frame_prepare(cam, kl, d)
        ok = (ds > 0) & (de > 0)
        Twc = traj[k].astype(np.float64)
        for j in np.nonzero(ok)[0]:
            row = []
            for (u, v, z) in ((ku["startPointX"][j], ku["startPointY"][j], ds[j]),
                              (ku["endPointX"][j], ku["endPointY"][j], de[j])):
                P = np.array([(u - cfg["cx"]) * z / cfg["fx"], (v - cfg["cy"]) * z / cfg["fy"], z, 1.0])
                row.extend((Twc @ P)[:3])
            xyz.append(row)
            desc.append(ld[j])
    g, d = frames[2]
    kl, ld, _, _ = O.line_extract(g)
    ku, _, _, _, _ = O.line_frame_prepare(cam, kl, d)
    rng = np.random.default_rng(seed + 3)
    cur_nobs = np.where(rng.random(len(ku)) < claim_frac, 1, 0).astype(np.int32)
    T2 = np.linalg.inv(traj[2]).astype(np.float32)
    return (cfg, cam, np.array(xyz, np.float32), np.array(desc, np.uint8), ku, ld, cur_nobs, T2)


def bow_problem(seed=0, bits=12):
    """Keyframe = frame 0, frame = frame 1 of a seeded sequence, with a
    stand-in vocabulary: a feature's node is the top `bits` bits of its
    descriptor (similar descriptors share nodes, as DBoW2 words do; the
    reference's ORBvoc.txt is not available). ~5 % of the features get no
    node, ~10 % of the keyframe map points are invalid."""
    O = load_oracle()
    cfg, traj, frames = sequence(2, seed)
    p = O.params()
    k0, d0, _ = O.extract(p, frames[0][0])
    k1, d1, _ = O.extract(p, frames[1][0])
    rng = np.random.default_rng(seed + 5)

    def nodes(d):
        v = (d[:, 0].astype(np.int64) << 8 | d[:, 1].astype(np.int64)) >> (16 - bits)
        return np.where(rng.random(len(d)) < 0.05, -1, v).astype(np.int32)

    return dict(kf_node=nodes(d0), kf_valid=(rng.random(len(d0)) > 0.1).astype(np.uint8),
                kf_desc=d0, kf_angle=k0["angle"], f_node=nodes(d1), f_desc=d1, f_angle=k1["angle"])


@functools.lru_cache(maxsize=4)
def stereo_pair(seed=0, cam_name="KITTI00"):
    """A rectified stereo pair: the right camera sits mb = bf / fx metres
    along the left camera's x axis (Frame.cc:62-63), same room and noise."""
    load_pkg()
    import orbpl.synth as synth
    cfg = dict(getattr(synth, cam_name))
    room = synth.default_room(seed)
    Twc = synth.trajectory(1, seed=seed)[0]
    shift = np.eye(4)
    shift[0, 3] = cfg["bf"] / cfg["fx"]
    left, _ = synth.render(cfg, Twc, room, seed=seed)
    right, _ = synth.render(cfg, Twc @ shift, room, seed=seed)
    return cfg, left, right


@functools.lru_cache(maxsize=8)
def stereo_sequence(n=3, seed=0, cam_name="KITTI00"):
    """n rectified stereo pairs along a seeded trajectory (right camera at
    +mb along the left camera's x axis): cfg, Twc list, [(left, right)]."""
    load_pkg()
    import orbpl.synth as synth
    cfg = dict(getattr(synth, cam_name))
    room = synth.default_room(seed)
    traj = synth.trajectory(n, seed=seed)
    shift = np.eye(4)
    shift[0, 3] = cfg["bf"] / cfg["fx"]
    pairs = []
    for i, T in enumerate(traj):
        left, _ = synth.render(cfg, T, room, seed=seed * 100 + i)
        right, _ = synth.render(cfg, T @ shift, room, seed=seed * 100 + i)
        pairs.append((left, right))
    return cfg, traj, pairs


def predict_scale_problem():
    """Map points straight ahead of an identity camera whose expected
    mnTrackScaleLevel is known by hand: a point created at distance d0 from an
    observation at octave k has mfMaxDistance = d0 * scale[k] and mfMinDistance
    = mfMaxDistance / scale[7] (MapPoint::UpdateNormalAndDepth, MapPoint.cc:
    376-382). Seen again from d0, MapPoint::PredictScale (MapPoint.cc:416-431)
    gives ceil(log(scale[k]) / log(1.2)), which is k up to the float rounding of
    the log ratio; octave 0 must give exactly 0 (ratio 1). Returns (cfg,
    Tcw, mps, expected level, ratio) with the expected levels computed here in
    numpy from the reference's formula, independently of the oracle."""
    load_pkg()
    import orbpl.synth as synth
    cfg = dict(synth.TUM1)
    sc = np.ones(8, np.float32)
    for i in range(1, 8):
        sc[i] = np.float32(sc[i - 1] * np.float32(1.2))
    xyz, nrm, dmin, dmax, exp_level, ratio = [], [], [], [], [], []
    for k in range(8):
        for d0, dview in ((2.0, 2.0), (1.5, 1.5), (2.0, 2.0 * 1.1), (3.0, 3.0 / 1.1)):
            # straight ahead: u = cx, v = cy, dist = z exactly
            P = np.array([0, 0, dview], np.float32)
            mx = np.float32(np.float32(d0) * sc[k])
            mn = np.float32(mx / sc[7])
            dist = np.float32(dview)
            if not (dist >= np.float32(0.8) * mn and dist <= np.float32(1.2) * mx):
                continue
            r = np.float32(mx / dist)
            lv = int(np.ceil(np.float32(np.log(np.float64(r))) / np.float32(np.log(np.float64(np.float32(1.2))))))
            xyz.append(P)
            nrm.append(np.array([0, 0, 1], np.float32))
            dmin.append(mn)
            dmax.append(mx)
            exp_level.append(min(max(lv, 0), 7))
            ratio.append(r)
    mps = dict(xyz=np.array(xyz, np.float32), normal=np.array(nrm, np.float32),
               min_dist=np.array(dmin, np.float32), max_dist=np.array(dmax, np.float32))
    return cfg, np.eye(4, dtype=np.float32), mps, np.array(exp_level, np.int32), np.array(ratio)
