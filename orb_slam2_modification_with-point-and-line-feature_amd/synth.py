"""Seeded synthetic RGB-D scenes for tests and the benchmark.

There are no datasets on either box, so every frame is rendered here: a room of
textured planes (value-noise texture at 4-64 px scales plus anti-aliased line
segments, contrast 40-120 DN) seen by a pinhole camera moving on a smooth SE(3)
trajectory. Depth comes exactly from the render (metres, float32) with ~5 %
zero holes; Gaussian pixel noise sigma = 2 DN. Textures live in plane
coordinates, so the same world point keeps its appearance across frames and
FAST/ORB/LSD fire on consistent structure.

Pure numpy; deterministic for a given seed.
"""
from __future__ import annotations

import numpy as np

# TUM1.yaml intrinsics (Examples/RGB-D/TUM1.yaml:8-22)
TUM1 = dict(fx=517.306408, fy=516.469215, cx=318.643040, cy=255.313989,
            k1=0.262383, k2=-0.953104, p1=-0.005358, p2=0.002628, k3=1.163314,
            width=640, height=480, bf=40.0, thdepth=40.0, depth_factor=5000.0)
# TUM3.yaml (no distortion)
TUM3 = dict(fx=535.4, fy=539.2, cx=320.1, cy=247.6, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0,
            width=640, height=480, bf=40.0, thdepth=40.0, depth_factor=5000.0)
# Upstream ORB-SLAM2 KITTI 00-02 values
KITTI00 = dict(fx=718.856, fy=718.856, cx=607.1928, cy=185.2157, k1=0.0, k2=0.0, p1=0.0,
               p2=0.0, k3=0.0, width=1241, height=376, bf=386.1448, thdepth=35.0,
               depth_factor=1.0)

# BASELINE configs[4]: synthetic 1280x720 camera of an 8-camera rig (no
# distortion, 90 deg horizontal field of view, RGB-D depth)
RIG720 = dict(fx=640.0, fy=640.0, cx=639.5, cy=359.5, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0,
              width=1280, height=720, bf=40.0, thdepth=40.0, depth_factor=5000.0)
RIG_CAMERAS = 8


def rig_offset(k, n=RIG_CAMERAS):
    """Camera-to-rig pose of rig camera k: yaw k * 360/n degrees (45 deg spacing
    for 8 cameras) about the rig's y axis, shared optical centre."""
    return se3(rot_xyz(0.0, 2 * np.pi * k / n, 0.0), np.zeros(3))


def _hash2(ix, iy, seed):
    """uint32 hash of integer lattice coordinates -> float in [0, 1)."""
    h = (ix.astype(np.int64) * 374761393 + iy.astype(np.int64) * 668265263 +
         np.int64(seed) * 2246822519) & 0xFFFFFFFF
    h = h.astype(np.uint64)
    h = (h ^ (h >> np.uint64(13))) * np.uint64(1274126177) & np.uint64(0xFFFFFFFF)
    h = h ^ (h >> np.uint64(16))
    return (h & np.uint64(0xFFFFFF)).astype(np.float64) / float(1 << 24)


def _value_noise(u, v, freq, seed):
    x = u * freq
    y = v * freq
    ix = np.floor(x)
    iy = np.floor(y)
    fx = x - ix
    fy = y - iy
    fx = fx * fx * (3 - 2 * fx)
    fy = fy * fy * (3 - 2 * fy)
    ix = ix.astype(np.int64)
    iy = iy.astype(np.int64)
    a = _hash2(ix, iy, seed)
    b = _hash2(ix + 1, iy, seed)
    c = _hash2(ix, iy + 1, seed)
    d = _hash2(ix + 1, iy + 1, seed)
    return (a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy


def _segments_layer(u, v, cell, seed, width):
    """Anti-aliased random segments: each `cell`-sized texture cell holds one
    segment with random endpoints, contrast and polarity."""
    cx = np.floor(u / cell).astype(np.int64)
    cy = np.floor(v / cell).astype(np.int64)
    out = np.zeros_like(u)
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            gx = cx + dx
            gy = cy + dy
            x0 = (gx + _hash2(gx, gy, seed + 11)) * cell
            y0 = (gy + _hash2(gx, gy, seed + 12)) * cell
            ang = _hash2(gx, gy, seed + 13) * np.pi
            ln = (0.4 + 0.8 * _hash2(gx, gy, seed + 14)) * cell
            con = (40 + 80 * _hash2(gx, gy, seed + 15)) * np.where(
                _hash2(gx, gy, seed + 16) < 0.5, -1.0, 1.0)
            ex = np.cos(ang)
            ey = np.sin(ang)
            px = u - x0
            py = v - y0
            t = np.clip(px * ex + py * ey, 0.0, ln)
            dist = np.hypot(px - t * ex, py - t * ey)
            cov = np.clip(1.0 - (dist - width * 0.5) / (width * 0.5 + 1e-12), 0.0, 1.0)
            out += con * cov
    return out


def texture(u, v, seed):
    """Intensity (float DN, unclipped) of plane texture coordinates (metres)."""
    t = 128.0
    for k, (freq, amp) in enumerate(((4.0, 60.0), (12.0, 40.0), (30.0, 30.0), (70.0, 18.0))):
        t = t + amp * (_value_noise(u, v, freq, seed * 31 + k) - 0.5)
    t = t + _segments_layer(u, v, 0.35, seed * 7 + 1, 0.008)
    t = t + _segments_layer(u + 0.17, v + 0.05, 0.6, seed * 7 + 2, 0.012)
    return t


def default_room(seed=0):
    """Planes as (point, normal, u_axis, v_axis, texture_seed)."""
    rng = np.random.default_rng(seed)
    planes = []
    size = 4.0
    specs = [((0, 0, size), (0, 0, -1), (1, 0, 0), (0, 1, 0)),     # front wall z=+4
             ((0, 0, -size), (0, 0, 1), (-1, 0, 0), (0, 1, 0)),    # back wall
             ((size, 0, 0), (-1, 0, 0), (0, 0, -1), (0, 1, 0)),    # right wall
             ((-size, 0, 0), (1, 0, 0), (0, 0, 1), (0, 1, 0)),     # left wall
             ((0, 1.2, 0), (0, -1, 0), (1, 0, 0), (0, 0, 1)),      # floor (y down)
             ((0, -2.0, 0), (0, 1, 0), (1, 0, 0), (0, 0, -1))]     # ceiling
    for p, n, ua, va in specs:
        planes.append((np.array(p, float), np.array(n, float), np.array(ua, float),
                       np.array(va, float), int(rng.integers(1, 1 << 20))))
    # a few boxes' front faces for depth discontinuities
    for k in range(3):
        z = 2.0 + 1.2 * k
        x = rng.uniform(-1.5, 1.5)
        planes.append((np.array([x, 0, z]), np.array([0, 0, -1.0]), np.array([1.0, 0, 0]),
                       np.array([0, 1.0, 0]), int(rng.integers(1, 1 << 20)), (x - 0.5, x + 0.5,
                                                                                -0.8, 0.9)))
    return planes


def render(cam, Twc, planes, seed=0, noise_sigma=2.0, hole_frac=0.05):
    """Render gray u8 (H, W) and depth float32 metres (H, W) for pose Twc (4x4,
    camera-to-world). Rays are cast through the *distorted* pixel grid if the
    camera has distortion, so keypoints need undistortion like a real TUM
    frame."""
    W, H = cam["width"], cam["height"]
    fx, fy, cx, cy = cam["fx"], cam["fy"], cam["cx"], cam["cy"]
    us, vs = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
    xn = (us - cx) / fx
    yn = (vs - cy) / fy
    k1, k2, p1, p2, k3 = cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"]
    if k1 != 0.0:
        # invert the distortion model by fixed-point iteration (pixel -> ray)
        x, y = xn.copy(), yn.copy()
        for _ in range(8):
            r2 = x * x + y * y
            rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
            dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
            dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
            x = (xn - dx) / rad
            y = (yn - dy) / rad
        xn, yn = x, y
    R = Twc[:3, :3]
    t = Twc[:3, 3]
    dirs_c = np.stack([xn, yn, np.ones_like(xn)], -1)          # z = 1 in camera
    dirs_w = dirs_c @ R.T
    best = np.full((H, W), np.inf)
    owner = np.full((H, W), -1, np.int32)
    for k, pl in enumerate(planes):
        p0, n = pl[0], pl[1]
        denom = dirs_w @ n
        with np.errstate(divide="ignore", invalid="ignore"):
            lam = ((p0 - t) @ n) / denom
        hit = (lam > 0.05) & np.isfinite(lam)
        if len(pl) > 5:
            P = t + dirs_w * lam[..., None]
            x0, x1, y0, y1 = pl[5]
            hit &= (P[..., 0] >= x0) & (P[..., 0] <= x1) & (P[..., 1] >= y0) & (P[..., 1] <= y1)
        closer = hit & (lam < best)
        best = np.where(closer, lam, best)
        owner = np.where(closer, k, owner)
    img = np.full((H, W), 128.0)
    for k, pl in enumerate(planes):
        sel = owner == k
        if not sel.any():
            continue
        p0, ua, va, tseed = pl[0], pl[2], pl[3], pl[4]
        P = t + dirs_w[sel] * best[sel][:, None]
        img[sel] = texture((P - p0) @ ua, (P - p0) @ va, tseed)
    depth = np.where(np.isfinite(best), best, 0.0)   # lam is z in camera (dir z = 1)
    rng = np.random.default_rng(seed)
    img = img + rng.normal(0.0, noise_sigma, img.shape)
    gray = np.clip(np.rint(img), 0, 255).astype(np.uint8)
    if hole_frac > 0:
        holes = rng.random(depth.shape) < hole_frac
        depth = np.where(holes, 0.0, depth)
    return gray, depth.astype(np.float32)


def se3(R, t):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


def rot_xyz(rx, ry, rz):
    cx, sx, cy, sy, cz, sz = np.cos(rx), np.sin(rx), np.cos(ry), np.sin(ry), np.cos(rz), np.sin(rz)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def trajectory(n, seed=0, step_t=0.01, step_r_deg=0.5, yaw0=0.0):
    """Smooth camera-to-world poses: <= step_t metres and <= step_r_deg per
    frame, starting near the room centre looking along +z."""
    rng = np.random.default_rng(seed)
    ph = rng.uniform(0, 2 * np.pi, 6)
    fr = rng.uniform(0.3, 1.0, 6)
    poses = []
    for i in range(n):
        s = i / 30.0
        tx = 0.4 * np.sin(fr[0] * s + ph[0]) * step_t / 0.01
        ty = 0.15 * np.sin(fr[1] * s + ph[1]) * step_t / 0.01
        tz = 0.4 * np.sin(fr[2] * s + ph[2]) * step_t / 0.01 - 0.5
        k = np.deg2rad(step_r_deg) * 30.0
        rx = 0.2 * k * np.sin(fr[3] * s + ph[3])
        ry = yaw0 + 0.6 * k * np.sin(fr[4] * s + ph[4])
        rz = 0.15 * k * np.sin(fr[5] * s + ph[5])
        poses.append(se3(rot_xyz(rx, ry, rz), np.array([tx, ty, tz])))
    return poses


def textured_image(width=640, height=480, seed=0, noise_sigma=2.0):
    """One gray frame of the default room from a seeded pose (extraction tests)."""
    rng = np.random.default_rng(seed)
    cam = dict(TUM3)
    cam.update(width=width, height=height, cx=width / 2.0 - 0.5, cy=height / 2.0 - 0.5,
               fx=0.83 * width, fy=0.83 * width)
    R = rot_xyz(rng.uniform(-0.2, 0.2), rng.uniform(-np.pi, np.pi), rng.uniform(-0.1, 0.1))
    t = np.array([rng.uniform(-1, 1), rng.uniform(-0.3, 0.3), rng.uniform(-1, 1)])
    gray, _ = render(cam, se3(R, t), default_room(seed), seed=seed, noise_sigma=noise_sigma)
    return gray


def loop_trajectory(n, seed=0, step_t=0.012, rot_amp_deg=4.0):
    """Closed smooth loop of n camera-to-world poses (frame n == frame 0), so a
    stream can cycle through it indefinitely with continuous motion: a circle
    whose per-frame chord is ~step_t metres plus periodic rotation of
    +-rot_amp_deg degrees (<= ~1 deg per frame for n >= 32)."""
    rng = np.random.default_rng(seed)
    r = step_t * n / (2 * np.pi)
    ph = rng.uniform(0, 2 * np.pi, 4)
    a = np.deg2rad(rot_amp_deg)
    yaw0 = rng.uniform(-np.pi, np.pi)
    poses = []
    for i in range(n):
        th = 2 * np.pi * i / n
        t = np.array([r * np.cos(th + ph[0]), 0.1 * r * np.sin(2 * th + ph[1]),
                      r * np.sin(th + ph[0]) - 0.3])
        R = rot_xyz(0.5 * a * np.sin(th + ph[2]), yaw0 + a * np.sin(th + ph[3]),
                    0.3 * a * np.cos(th + ph[2]))
        poses.append(se3(R, t))
    return poses


# ---------------------------------------------------------------------------
# Synthetic ORB vocabulary (the reference's ORBvoc.txt is not in its
# checkout): a complete k-ary tree of depth L built DBoW2-style by
# hierarchical k-medians on binary descriptors (seeded centres, member
# majority bits), TF-IDF word weights idf = log((N + 1) / (N_i + 1)) over the
# training documents (smoothed so that, as with ORBvoc's large training set,
# nearly every word carries a weight; a word in every document is stopped,
# weight 0), written in DBoW2's
# text format (TemplatedVocabulary::saveToTextFile, TemplatedVocabulary.h:1427).
# Node ids are breadth-first, so a node's children are contiguous.
# ---------------------------------------------------------------------------
def _hamming_rows(X, Cc):
    """X [m,4] u64, Cc [k,4] u64 -> [m,k] Hamming distances."""
    return np.bitwise_count(X[:, None, :] ^ Cc[None, :, :]).sum(-1)


def _majority(X):
    """Bitwise majority of rows X [m,4] u64 (FORB::meanValue: bit set when
    its count >= ceil(m / 2))."""
    bits = np.unpackbits(X.view(np.uint8).reshape(len(X), 32), axis=1)
    need = (len(X) + 1) // 2
    return np.packbits((bits.sum(0) >= need).astype(np.uint8)).view(np.uint64).reshape(4)


def vocabulary_tree(train, k=10, L=5, seed=0, iters=3):
    """train: list of [n_i, 32] u8 descriptor arrays (one per document).
    Returns dict(parent, desc [N,32] u8, leaf, weight, first_child, k, L)."""
    rng = np.random.default_rng(seed)
    docs = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in train]
    X = np.concatenate(docs).view(np.uint64).reshape(-1, 4)
    nn = (k ** (L + 1) - 1) // (k - 1)
    desc = np.zeros((nn, 4), np.uint64)
    parent = np.full(nn, -1, np.int64)
    members = {0: np.arange(len(X))}
    nxt = 1
    first_child = np.full(nn, -1, np.int64)
    for node in range(nn):
        level = 0 if node == 0 else int(np.floor(np.log(node * (k - 1) + 1) / np.log(k) + 1e-9))
        if level >= L:
            break
        idx = members.pop(node, np.zeros(0, np.int64))
        m = len(idx)
        if m >= k:
            Cc = X[idx[rng.choice(m, k, replace=False)]].copy()
            for _ in range(iters):
                a = _hamming_rows(X[idx], Cc).argmin(1)
                for c in range(k):
                    sel = idx[a == c]
                    if len(sel):
                        Cc[c] = _majority(X[sel])
            a = _hamming_rows(X[idx], Cc).argmin(1)
        else:
            Cc = rng.integers(0, 2 ** 63, size=(k, 4), dtype=np.uint64)
            if m:
                Cc[:m] = X[idx]
            a = _hamming_rows(X[idx], Cc).argmin(1) if m else np.zeros(0, np.int64)
        first_child[node] = nxt
        for c in range(k):
            desc[nxt + c] = Cc[c]
            parent[nxt + c] = node
            members[nxt + c] = idx[a == c]
        nxt += k
    leaf = first_child < 0
    tree = dict(parent=parent, desc=desc.view(np.uint8).reshape(nn, 32), leaf=leaf,
                first_child=first_child, k=k, L=L, weight=np.zeros(nn))
    # idf over the documents
    N = len(docs)
    Ni = np.zeros(nn, np.int64)
    for d in docs:
        Ni[np.unique(vocabulary_words(tree, d))] += 1
    tree["weight"] = idf_weights(tree, Ni, N)
    return tree


def idf_weights(tree, Ni, N):
    """Leaf weights log((N + 1) / (N_i + 1)) (0 for inner nodes)."""
    w = np.zeros(len(tree["parent"]))
    leaf = tree["leaf"]
    w[leaf] = np.log((N + 1.0) / (np.asarray(Ni, np.float64)[leaf] + 1.0))
    return w


def vocabulary_words(tree, desc):
    """Leaf node of every descriptor (strict <: first minimal child)."""
    D = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32).view(np.uint64).reshape(-1, 4)
    V = tree["desc"].view(np.uint64).reshape(-1, 4)
    k = tree["k"]
    node = np.zeros(len(D), np.int64)
    while True:
        fc = tree["first_child"][node]
        if np.all(fc < 0):
            return node
        ch = fc[:, None] + np.arange(k)[None, :]
        d = np.bitwise_count(D[:, None, :] ^ V[ch]).sum(-1)
        node = np.where(fc >= 0, ch[np.arange(len(D)), d.argmin(1)], node)


def vocabulary_text(tree, scoring=0, weighting=0):
    """DBoW2 text format: "k L  scoring weighting", then one line per node
    1..N-1: parent, isLeaf, 32 descriptor bytes, weight (C++ stream default
    formatting), each line ended by '\\n' like saveToTextFile's endl."""
    out = [f"{tree['k']} {tree['L']}  {scoring} {weighting}\n"]
    for i in range(1, len(tree["parent"])):
        d = " ".join(str(int(b)) for b in tree["desc"][i])
        out.append(f"{int(tree['parent'][i])} {1 if tree['leaf'][i] else 0} {d}  "
                   f"{tree['weight'][i]:g}\n")
    return "".join(out)
