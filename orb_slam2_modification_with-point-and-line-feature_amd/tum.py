"""Host-side I/O of the reference's RGB-D examples and the trajectory
evaluator, in plain numpy:

* ``load_settings``      - the OpenCV FileStorage YAML settings read by
                           ``Tracking::Tracking`` (``Tracking.cc:54-146``,
                           ``Examples/RGB-D/TUM1.yaml``);
* ``load_associations``  - ``LoadImages`` of ``Examples/RGB-D/rgbd_my.cpp:141-166``
                           (plus the ground-truth columns of
                           ``associate_with_groundtruth.txt`` when present);
* ``depth_to_metres``    - ``imDepth.convertTo(CV_32F, mDepthMapFactor)``
                           (``Tracking.cc:142-146``, ``Tracking.cc:233-234``);
* ``save_trajectory_tum`` / ``save_keyframe_trajectory_tum`` / ``load_trajectory_tum``
                         - ``System::SaveTrajectoryTUM`` / ``SaveKeyFrameTrajectoryTUM``
                           text format (``System.cc:337-432``): ``t tx ty tz qx qy qz qw``
                           with ``Converter::toQuaternion`` (Eigen's
                           rotation-matrix-to-quaternion, ``Converter.cc:137-149``);
* ``ate``                - absolute trajectory error after the closed-form
                           rigid (SE(3), no scale) alignment of the camera
                           centres (Horn / Umeyama), as TUM's ``evaluate_ate``.

The tracker keeps no keyframes, so a frame's pose is written directly
(the reference composes it with its reference keyframe; for a map that never
changes the two agree).
"""
import numpy as np


def _parse_scalar(v):
    v = v.strip()
    if len(v) >= 2 and v[0] == v[-1] and v[0] in "\"'":
        return v[1:-1]
    try:
        return int(v)
    except ValueError:
        pass
    try:
        return float(v)
    except ValueError:
        return v


def load_settings(path):
    """Flat ``key: value`` settings of an OpenCV FileStorage YAML file
    (``%YAML:1.0`` header, ``#`` comments, ``Viewer.PointSize:2`` without a
    space all accepted) -> (raw dict, camera dict for ``make_camera``, ORB
    parameter tuple, depth map factor)."""
    raw = {}
    with open(path) as f:
        for line in f:
            s = line.split("#", 1)[0].strip()
            if not s or s.startswith("%") or s == "---" or ":" not in s:
                continue
            k, v = s.split(":", 1)
            raw[k.strip()] = _parse_scalar(v)
    g = lambda k, d=0.0: raw.get(k, d)
    cam = dict(fx=float(g("Camera.fx")), fy=float(g("Camera.fy")), cx=float(g("Camera.cx")),
               cy=float(g("Camera.cy")), k1=float(g("Camera.k1")), k2=float(g("Camera.k2")),
               p1=float(g("Camera.p1")), p2=float(g("Camera.p2")), k3=float(g("Camera.k3")),
               width=int(g("Camera.width", 640)), height=int(g("Camera.height", 480)),
               bf=float(g("Camera.bf")), thdepth=float(g("ThDepth", 35.0)),
               depth_factor=float(g("DepthMapFactor", 1.0)))
    orb = (int(g("ORBextractor.nFeatures", 1000)), float(g("ORBextractor.scaleFactor", 1.2)),
           int(g("ORBextractor.nLevels", 8)), int(g("ORBextractor.iniThFAST", 20)),
           int(g("ORBextractor.minThFAST", 7)))
    # mDepthMapFactor (Tracking.cc:142-146): 1 if |factor| < 1e-5 else 1 / factor, in float
    f = np.float32(cam["depth_factor"])
    dmf = np.float32(1.0) if abs(float(f)) < 1e-5 else np.float32(1.0) / f
    return raw, cam, orb, dmf


def load_associations(path):
    """``LoadImages`` (rgbd_my.cpp:141-166): per non-empty line the RGB
    timestamp and file, the depth timestamp and file. Extra columns are the
    ground truth ``t tx ty tz qx qy qz qw`` of
    ``associate_with_groundtruth.txt`` and are returned when present."""
    t_rgb, rgb, t_d, dep, gt = [], [], [], [], []
    with open(path) as f:
        for line in f:
            tok = line.split()
            if not tok:
                continue
            t_rgb.append(float(tok[0]))
            rgb.append(tok[1])
            t_d.append(float(tok[2]))
            dep.append(tok[3])
            if len(tok) >= 12:
                gt.append([float(x) for x in tok[4:12]])
    out = dict(t_rgb=np.array(t_rgb), rgb=rgb, t_depth=np.array(t_d), depth=dep)
    if gt and len(gt) == len(rgb):
        out["gt"] = np.array(gt)        # (N, 8): t tx ty tz qx qy qz qw
    return out


def depth_to_metres(depth_u16, depth_map_factor):
    """``imDepth.convertTo(imDepth, CV_32F, mDepthMapFactor)``: u16 * float
    scale, one float rounding."""
    return (np.asarray(depth_u16).astype(np.float32) * np.float32(depth_map_factor)).astype(
        np.float32)


def quaternion_from_matrix(R):
    """Eigen's ``Quaternion(Matrix3)`` (the published algorithm of
    ``quaternionbase_assign_impl``), double precision -> (x, y, z, w)."""
    m = np.asarray(R, np.float64)
    t = m[0, 0] + m[1, 1] + m[2, 2]
    q = np.zeros(4)                      # x y z w
    if t > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (m[2, 1] - m[1, 2]) * t
        q[1] = (m[0, 2] - m[2, 0]) * t
        q[2] = (m[1, 0] - m[0, 1]) * t
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j = (i + 1) % 3
        k = (j + 1) % 3
        t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k, j] - m[j, k]) * t
        q[j] = (m[j, i] + m[i, j]) * t
        q[k] = (m[k, i] + m[i, k]) * t
    return q


def matrix_from_quaternion(q):
    x, y, z, w = (float(v) for v in q)
    n = np.sqrt(x * x + y * y + z * z + w * w)
    x, y, z, w = x / n, y / n, z / n, w / n
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _twc_rwc(Tcw):
    """Rwc = Rcw^T (exact) and twc = -Rwc * tcw as a float cv::Mat product
    (products summed in double, one rounding)."""
    T = np.asarray(Tcw, np.float32).reshape(4, 4)
    Rwc = T[:3, :3].T.copy()
    twc = -(Rwc.astype(np.float64) @ T[:3, 3].astype(np.float64)).astype(np.float32)
    return Rwc, twc


def _format_line(t, twc, q, prec):
    vals = [np.float32(v) for v in list(twc) + list(q)]
    return f"{t:.6f} " + " ".join(f"{float(v):.{prec}f}" for v in vals)


def save_trajectory_tum(path, timestamps, Tcw, lost=None):
    """``System::SaveTrajectoryTUM`` (System.cc:337-396) for per-frame poses
    Tcw (N, 4, 4): frames flagged lost are skipped, timestamp with 6
    decimals, position and quaternion (x y z w, float) with 9."""
    with open(path, "w") as f:
        for i, (t, T) in enumerate(zip(timestamps, Tcw)):
            if lost is not None and lost[i]:
                continue
            Rwc, twc = _twc_rwc(T)
            q = quaternion_from_matrix(Rwc).astype(np.float32)
            f.write(_format_line(float(t), twc, q, 9) + "\n")


def save_keyframe_trajectory_tum(path, timestamps, Tcw):
    """``System::SaveKeyFrameTrajectoryTUM`` (System.cc:398-432): camera
    centre and quaternion of R^T with 7 decimals."""
    with open(path, "w") as f:
        for t, T in zip(timestamps, Tcw):
            Rwc, twc = _twc_rwc(T)
            q = quaternion_from_matrix(Rwc).astype(np.float32)
            f.write(_format_line(float(t), twc, q, 7) + "\n")


def load_trajectory_tum(path):
    """``t tx ty tz qx qy qz qw`` rows -> (timestamps (N,), Twc (N, 4, 4))."""
    rows = []
    with open(path) as f:
        for line in f:
            tok = line.split()
            if len(tok) >= 8 and not line.lstrip().startswith("#"):
                rows.append([float(x) for x in tok[:8]])
    a = np.array(rows).reshape(-1, 8)
    return a[:, 0], poses_from_rows(a)


def poses_from_rows(a):
    """(N, 8) ``t tx ty tz qx qy qz qw`` -> (N, 4, 4) Twc."""
    T = np.tile(np.eye(4), (len(a), 1, 1))
    for i, r in enumerate(a):
        T[i, :3, :3] = matrix_from_quaternion(r[4:8])
        T[i, :3, 3] = r[1:4]
    return T


def associate(t_a, t_b, max_difference=0.02):
    """Greedy timestamp association of TUM's ``associate.py``: pairs (i, j)
    by increasing |t_a[i] - t_b[j]| below max_difference, each used once."""
    t_a, t_b = np.asarray(t_a, np.float64), np.asarray(t_b, np.float64)
    cand = [(abs(a - b), i, j) for i, a in enumerate(t_a) for j, b in enumerate(t_b)
            if abs(a - b) < max_difference]
    cand.sort()
    ua, ub, out = set(), set(), []
    for _, i, j in cand:
        if i not in ua and j not in ub:
            ua.add(i)
            ub.add(j)
            out.append((i, j))
    out.sort()
    return out


def align(est, gt):
    """Closed-form rigid alignment (rotation + translation, no scale) of the
    point sets est -> gt (N, 3): returns (R, t) minimising
    sum |R est_i + t - gt_i|^2 (Umeyama without scale)."""
    est = np.asarray(est, np.float64)
    gt = np.asarray(gt, np.float64)
    me, mg = est.mean(0), gt.mean(0)
    H = (est - me).T @ (gt - mg)
    U, _, Vt = np.linalg.svd(H)
    S = np.eye(3)
    if np.linalg.det(Vt.T @ U.T) < 0:
        S[2, 2] = -1
    R = Vt.T @ S @ U.T
    return R, mg - R @ me


def ate(est_xyz, gt_xyz, aligned=True):
    """Absolute trajectory error of camera centres (N, 3) in metres:
    dict(rmse, mean, median, max, n) after the rigid alignment (or raw)."""
    est = np.asarray(est_xyz, np.float64)
    gt = np.asarray(gt_xyz, np.float64)
    if aligned:
        R, t = align(est, gt)
        est = est @ R.T + t
    e = np.linalg.norm(est - gt, axis=1)
    return dict(rmse=float(np.sqrt(np.mean(e * e))), mean=float(e.mean()),
                median=float(np.median(e)), max=float(e.max()), n=int(len(e)))


def camera_centres(Tcw):
    """Camera centres -R^T t of Tcw poses (N, 4, 4) in double."""
    T = np.asarray(Tcw, np.float64).reshape(-1, 4, 4)
    return -np.einsum("nji,nj->ni", T[:, :3, :3], T[:, :3, 3])
