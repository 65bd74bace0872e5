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
