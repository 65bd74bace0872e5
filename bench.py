#!/usr/bin/env python3
"""Benchmark: frames/sec of the per-frame hot path (extract + match + pose).

BASELINE.json metric "frames/sec (extract+match+pose) at 640x480", quoted on
configs[1] = "TUM fr1_desk RGB-D, ORB point features only, 1 MI355X":
TUM1.yaml camera + distortion, ORB 1000 features / 1.2 / 8 levels / FAST 20,7.

A step = one Tracking::TrackWithMotionModel pass (ORB extraction, Frame glue,
SearchByProjection(th=15, retry 30), PoseOptimization, outlier discard) over a
batch of `--streams` independent synthetic 640x480 RGB-D streams, all inputs
resident in HBM before the timed region. The configs[2] workload (TUM3, ORB +
LSD/LBD LineExtractor, LineMatcher::SearchByProjection, line edges in the
pose) is timed the same way and reported under "secondary" (or as the
headline with --workload lines), and so is configs[3] (KITTI 00 camera,
1241x376 rectified stereo pairs, ORB 2000 on both images, ComputeStereoMatches,
th = 7 matching, pose) under "stereo" (or --workload kitti). Frames are
rendered from a seeded textured room along closed loop trajectories (no
datasets on the box).

Multi-GPU: one process per GPU (torchrun), streams sharded across ranks with
no data-path collective (weak scaling); the gloo process group only carries the
barrier and the max-over-ranks time.

Prints ONE JSON line (rank 0). See DESIGN.md for the roofline accounting.
"""
import argparse
import json
import os
import sys
import threading
import time
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "tests"))

W, H = 640, 480
ORB = (1000, 1.2, 8, 20, 7)
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8 TB/s spec

# BASELINE.json configs[1..3]: camera (orbpl.synth), ORB parameters, sensor
WORKLOADS = {
    "points": dict(cam="TUM1", orb=ORB, lines=False, stereo=False,
                   desc="TUM fr1_desk-like RGB-D, ORB points only (configs[1])",
                   data="synthetic (seeded textured-room RGB-D loop, TUM1 intrinsics+distortion)"),
    "lines": dict(cam="TUM3", orb=ORB, lines=True, stereo=False,
                  desc="TUM fr3_structure_texture_far-like RGB-D, ORB + LSD/LBD lines (configs[2])",
                  data="synthetic (seeded textured-room RGB-D loop, TUM3 intrinsics, no distortion)"),
    "kitti": dict(cam="KITTI00", orb=(2000, 1.2, 8, 20, 7), lines=False, stereo=True,
                  desc="KITTI 00-like stereo 1241x376, ORB 2000 both images + ComputeStereoMatches "
                       "+ PoseOptimization (configs[3]; the reference's stereo Frame has no lines)",
                  data="synthetic (seeded textured-room rectified stereo loop, KITTI 00 intrinsics, "
                       "bf 386.1448)"),
    "rig": dict(cam="RIG720", orb=(2000, 1.2, 8, 20, 7), lines=False, stereo=False, cams=8,
                desc="synthetic 1280x720 8-camera rig (45 deg yaw spacing), RGB-D, ORB 2000 "
                     "(configs[4]); stream 8r+c = camera c of rig r",
                data="synthetic (seeded textured-room RGB-D loop of an 8-camera rig, 1280x720)"),
}


class Layout:
    """Which rendered loop frame stream s reads at step t. cams == 1: stream s
    reads loop frame (s + t) mod F. Rig (cams == 8): stream s = 8 r + c is
    camera c of rig r and reads rig frame (r + t) mod F of camera c. Rendered
    frames are ordered [frame][camera]; the device buffer replicates them so
    that every step's batch is one contiguous slice starting at t * cams."""

    def __init__(self, traj, cams=1):
        import orbpl.synth as synth
        self.traj, self.F, self.cams = traj, len(traj), cams
        self.off = [synth.rig_offset(c, cams) if cams > 1 else np.eye(4) for c in range(cams)]

    def elem(self, s, t):
        r, c = divmod(s, self.cams)
        return ((r + t) % self.F) * self.cams + c

    def Twc(self, s, t):
        r, c = divmod(s, self.cams)
        return self.traj[(r + t) % self.F] @ self.off[c]

    def replicated(self, S):
        return np.arange((S // self.cams + self.F) * self.cams) % (self.F * self.cams)


def _render(args):
    e, n, seed, cam_name, stereo, cams = args
    from _pkg import load_pkg
    load_pkg()
    import orbpl.synth as synth
    traj = synth.loop_trajectory(n, seed=seed)
    room = synth.default_room(seed)
    cam = getattr(synth, cam_name)
    i, c = divmod(e, cams)
    Twc = traj[i] @ synth.rig_offset(c, cams) if cams > 1 else traj[i]
    g, d = synth.render(cam, Twc, room, seed=seed * 1000 + e)
    if stereo:  # right image of the rectified pair: camera at +mb along x
        shift = np.eye(4)
        shift[0, 3] = cam["bf"] / cam["fx"]
        d, _ = synth.render(cam, Twc @ shift, room, seed=seed * 1000 + e)
    return g, d


def render_loop(n, seed, workers, cam_name="TUM1", stereo=False, cams=1):
    """(gray, depth) of an n-frame loop ([frame][camera] for a rig), or
    (left, right) for stereo."""
    with ProcessPoolExecutor(max_workers=workers) as ex:
        out = list(ex.map(_render, [(e, n, seed, cam_name, stereo, cams) for e in range(n * cams)]))
    return np.stack([o[0] for o in out]), np.stack([o[1] for o in out])


def level_areas(w=W, h=H, orb=ORB):
    from _pkg import load_pkg
    d = load_pkg().describe(*orb, width=w, height=h)
    return [int(a) * int(b) for a, b in zip(d["width"], d["height"])], d


def algorithmic_bytes(n_kp, w=W, h=H, orb=ORB):
    """Per-frame algorithmic HBM bytes of each kernel:
    the bytes the kernel must move at minimum (each input read once, each
    output written once), with n_kp keypoints per frame."""
    areas, d = level_areas(w, h, orb)
    S = sum(areas)
    dims = list(zip((int(a) for a in d["width"]), (int(b) for b in d["height"])))
    pads = [(a + 38) * (b + 38) for a, b in dims]
    return {
        # read the input (level 0) or the previous level, write the padded level
        "pyramid": w * h + sum(areas[:-1]) + sum(pads),
        # read each level's content + 3 px halo, write the blurred content
        "blur": sum((a + 6) * (b + 6) for a, b in dims) + S,
        # read every pyramid level once (candidate output is ~1 % of it)
        "fast": S,
        # candidates in (4 B) and keypoints out (4 B); ~8 candidates per keypoint
        "octree": 8 * n_kp * 4 + n_kp * 4,
        # per keypoint: 31x31 raw patch + 37x37 blurred footprint + 60 B out
        "orient_desc": n_kp * (961 + 1369 + 60),
        # current frame (kp 28 + desc 32 + ur 4 + cell 4 + match out 4) and
        # last frame (kp 28 + flags 2 + xyz 12 + desc 32 + nobs 4)
        "match": n_kp * (72 + 78),
        # per keypoint: kp 28 + ur 4 + match 4 + xyz 12 + outlier 2
        "pose": n_kp * 50,
    }


def pmc_traffic(kernel, streams):
    """HBM bytes per launch of `kernel` from the committed PMC summary of the
    same bench command (tools/prof.sh + tools/pmc_traffic.py; FETCH_SIZE x2
    gfx950 correction + WRITE_SIZE), scaled to this run's stream count. PMC
    counters need their own rocprofv3 passes, so they cannot be read live."""
    for rnd in ("r01",):
        f = ROOT / "profiles" / rnd / "pmc_traffic.json"
        if f.exists():
            d = json.load(open(f))
            e = d.get(kernel)
            meta = d.get("_meta", {})
            if e and e.get("traffic_bytes") and meta.get("streams"):
                return (int(e["traffic_bytes"] * streams / meta["streams"]),
                        f"profiles/{rnd}/pmc_traffic.json ({meta['streams']} streams, scaled)")
    return None, None


def _oracle_vo(O, wl):
    """The oracle's VO loop for a workload; returns (vo, step(vo, a, b))."""
    import orbpl.synth as synth
    cam = O.camera(getattr(synth, wl["cam"]))
    if wl["stereo"]:
        return (O.LVO(O.params(*wl["orb"]), cam, 1, use_lines=False),
                lambda vo, a, b: vo.step_stereo(0, a, b))
    if wl["lines"]:
        return O.LVO(O.params(*wl["orb"]), cam, 1, use_lines=True), lambda vo, a, b: vo.step(0, a, b)
    return O.VO(O.params(*wl["orb"]), cam, 1), lambda vo, a, b: vo.step(0, a, b)


def cpu_baseline(seconds, threads, gray, depth, L, workload="points"):
    """The CPU oracle (C++ restatement, oracle/) running the same per-frame
    step, one stream per thread (throughput mode), for a bounded wall time."""
    from _pkg import load_oracle
    O = load_oracle()
    wl = WORKLOADS[workload]
    counts = [0] * threads
    stop = time.time() + seconds

    def worker(k):
        vo, vstep = _oracle_vo(O, wl)
        i = 0
        while time.time() < stop:   # worker k runs stream k of the layout
            e = L.elem(k, i)
            vstep(vo, gray[e], depth[e])
            i += 1
        counts[k] = i

    t0 = time.time()
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.time() - t0
    return sum(counts) / dt, sum(counts), dt


def accuracy_gpu(pkg, cam, wl, d_gray, d_depth, L, A, local_rank, fb, db):
    """Untimed accuracy leg: A streams tracked over a whole loop of F frames
    (Layout L, each stream starts at its true pose); returns the (A, F, 4, 4)
    Tcw poses after every step."""
    F = L.F
    tr = pkg.Tracker(pkg.OrbParams(*wl["orb"]), cam, A, device=local_rank, lines=wl["lines"],
                     stereo=wl["stereo"])
    tr.reset(np.stack([np.linalg.inv(L.Twc(s, 0)).astype(np.float32) for s in range(A)]).reshape(
        A, 16))
    out = np.zeros((A, F, 4, 4), np.float32)
    for t in range(F):
        o = t * L.cams
        if wl["stereo"]:
            tr.step_stereo_device(d_gray.ptr + o * fb, d_depth.ptr + o * db)
        else:
            tr.step_device(d_gray.ptr + o * fb, d_depth.ptr + o * db)
        tr.synchronize()
        out[:, t] = tr.state()["Tcw"]
    tr.close()
    return out


def accuracy_ref(gray, depth, L, A, workload):
    """The oracle's VO loop (the reference restatement) over the same A x F
    frames, one host thread per stream; returns its (A, F, 4, 4) poses."""
    from _pkg import load_oracle
    O = load_oracle()
    wl = WORKLOADS[workload]
    F = L.F
    out = np.zeros((A, F, 4, 4), np.float32)

    def worker(s):
        vo, vstep = _oracle_vo(O, wl)
        vo.reset(np.linalg.inv(L.Twc(s, 0)).astype(np.float32).reshape(1, 16))
        for t in range(F):
            e = L.elem(s, t)
            out[s, t] = vstep(vo, gray[e], depth[e])[0]

    ths = [threading.Thread(target=worker, args=(s,)) for s in range(A)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return out


def ate_report(T_gpu, T_ref, L):
    """ATE RMSE (m) of the GPU poses vs the reference restatement's poses of
    the same frames (raw: both start at the same pose) and of both vs the
    ground truth (rigidly aligned, as TUM's evaluate_ate)."""
    import orbpl.tum as tum
    A, F = T_gpu.shape[:2]
    gt = np.stack([np.linalg.inv(L.Twc(s, t)) for s in range(A) for t in range(F)])
    cg = tum.camera_centres(T_gpu.reshape(-1, 4, 4))
    cgt = tum.camera_centres(gt)
    rep = {"streams": A, "frames_per_stream": F,
           "ate_rmse_vs_gt_m": round(tum.ate(cg, cgt)["rmse"], 6)}
    if T_ref is not None:
        cr = tum.camera_centres(T_ref.reshape(-1, 4, 4))
        rep["ate_rmse_vs_ref_m"] = float(f"{tum.ate(cg, cr, aligned=False)['rmse']:.3e}")
        rep["max_abs_pose_diff_vs_ref"] = float(f"{np.abs(T_gpu - T_ref).max():.3e}")
        rep["ref_ate_rmse_vs_gt_m"] = round(tum.ate(cr, cgt)["rmse"], 6)
    return rep


def run_workload(pkg, synth, args, workload, S, steps, warmup, rank, world, local_rank, dist):
    """Time `steps` tracker steps of one workload; returns the measurements."""
    wl = WORKLOADS[workload]
    lines, stereo, cam_name = wl["lines"], wl["stereo"], wl["cam"]
    cams = wl.get("cams", 1)
    F = args.loop if cams == 1 else args.rig_loop
    if S % cams:
        raise SystemExit(f"--streams must be a multiple of the rig's {cams} cameras")
    workers = min(16, os.cpu_count() or 4)
    gray, depth = render_loop(F, seed=1 + rank, workers=workers, cam_name=cam_name, stereo=stereo,
                              cams=cams)
    fh, fw = gray.shape[1:]
    traj = synth.loop_trajectory(F, seed=1 + rank)
    L = Layout(traj, cams)
    # every step's batch is one contiguous slice of a replicated buffer (Layout)
    rep = L.replicated(S)
    d_gray = pkg.DeviceBuffer.from_array(gray[rep], device=local_rank)
    d_depth = pkg.DeviceBuffer.from_array(depth[rep], device=local_rank)
    cam = pkg.make_camera(getattr(synth, cam_name))
    tr = pkg.Tracker(pkg.OrbParams(*wl["orb"]), cam, S, device=local_rank, lines=lines,
                     stereo=stereo)
    # pipelining overlaps extraction of step t+1 with tracking of step t; the
    # lines workload is bound by the LSD stream, which the overlap only slows
    pipelined = args.pipelined if args.pipelined >= 0 else (0 if lines else 1)
    tr.set_pipelined(bool(pipelined))
    tr.reset(np.stack([np.linalg.inv(L.Twc(s, 0)).astype(np.float32) for s in range(S)]).reshape(S, 16))
    fb = fw * fh
    db = fb * depth.itemsize   # right image (u8) for stereo, depth (f32) otherwise

    def step(k):
        o = (k % F) * cams
        if stereo:
            tr.step_stereo_device(d_gray.ptr + o * fb, d_depth.ptr + o * db)
        else:
            tr.step_device(d_gray.ptr + o * fb, d_depth.ptr + o * db)

    for k in range(warmup):
        step(k)
    tr.synchronize()
    tr.timings_reset()
    if dist:
        dist.barrier()
    tr.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(warmup + k)
    tr.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = tr.state()
    tim = tr.timings(steps)                            # (steps, 9) ms, in-stream hipEvents
    avg = tim.mean(0)
    stages = dict(zip(tr.STAGES, [round(float(x), 4) for x in avg]))
    tracking = {"mean_keypoints": float(st["nkeypoints"].mean()),
                "mean_matches": float(st["nmatches"].mean()),
                "mean_inliers": float(st["ninliers"].mean()),
                "ok_frac": float(tr.status()["ok"].mean())}
    if lines:
        lt = tr.line_timings(steps).mean(0)
        stages.update(zip(tr.LINE_STAGES, [round(float(x), 4) for x in lt]))
        ls = tr.status()
        tracking.update(mean_lines=float(ls["nlines"].mean()),
                        mean_line_matches=float(ls["line_matches"].mean()))
    if stereo:
        stt = tr.stereo_timings(steps).mean(0)
        stages.update(zip(tr.STEREO_STAGES, [round(float(x), 4) for x in stt]))
    frames = S * steps * world
    value = frames / elapsed

    # roofline of the dominant single-launch kernel; k_pyramid (pyramid +
    # borders + blur, one launch) is timed by the "pyramid" stage
    n_kp = float(st["nkeypoints"].mean())
    ab = algorithmic_bytes(n_kp, fw, fh, wl["orb"])
    ab["pyramid"] = ab["pyramid"] + ab.pop("blur")
    names = {"pyramid": "k_pyramid", "fast": "k_fast_cells", "octree": "k_octree",
             "orient_desc": "k_orient_desc", "match": "k_match_last", "pose": "k_pose"}
    idx = {k: tr.STAGES.index(k) for k in names}
    iso = None
    if pipelined and args.isolated_steps > 0:
        # untimed: more steps with the two HIP streams serialised, so each
        # kernel's in-stream hipEvent time is its own. In the pipelined timed
        # region a kernel's event time also counts the time it waits for CUs
        # the other stream occupies, so the dominant kernel (the one with the
        # most GPU time) is chosen on these isolated times.
        tr.set_pipelined(False)
        tr.timings_reset()
        for k in range(args.isolated_steps):
            step(warmup + steps + k)
        tr.synchronize()
        iso = tr.timings(args.isolated_steps).mean(0)
    sel = iso if iso is not None else avg
    dom = max(names, key=lambda k: sel[idx[k]])
    dom_ms = float(avg[idx[dom]])          # live: timed region, in-stream hipEvents
    bytes_launch = int(ab[dom] * S)
    achieved = bytes_launch / (dom_ms * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic(names[dom], S) if workload == "points" else (None, None)
    roof = {"bound": "hbm", "kernel": names[dom],
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "traffic_source": tsrc,
            "algorithmic_bytes_per_launch": bytes_launch, "avg_launch_ms": round(dom_ms, 4),
            "per_kernel_GBps": {k: round(ab[k] * S / (float(avg[idx[k]]) * 1e-3) / 1e9, 1)
                                for k in names}}
    if iso is not None:
        ims = float(iso[idx[dom]])
        roof["isolated"] = {
            "stage_ms": dict(zip(tr.STAGES, [round(float(x), 4) for x in iso])),
            "avg_launch_ms": round(ims, 4),
            "achieved": round(bytes_launch / (ims * 1e-3) / 1e9, 2),
            "frac": round(bytes_launch / (ims * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "steps": args.isolated_steps}
    tr.close()
    A = min(args.ate_streams, S)
    T_acc = (accuracy_gpu(pkg, cam, wl, d_gray, d_depth, L, A, local_rank, fb, db)
             if A > 0 else None)
    return dict(S=S, value=value, T_acc=T_acc, layout=L, elapsed=elapsed, stages=stages,
                tracking=tracking, roof=roof, gray=gray, depth=depth, workload=wl["desc"],
                data=wl["data"], image=f"{fw}x{fh}", nfeatures=wl["orb"][0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, default=256, help="streams (frames per step) per GPU")
    ap.add_argument("--loop", type=int, default=32, help="frames in the synthetic loop")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=tuple(WORKLOADS), default="points",
                    help="points = configs[1] (headline); lines = configs[2] ORB + LSD/LBD; "
                         "kitti = configs[3] stereo; rig = configs[4] 1280x720 8-camera rig")
    ap.add_argument("--rig-loop", type=int, default=12,
                    help="rig frames in the synthetic loop (x8 camera renders)")
    ap.add_argument("--secondary-steps", type=int, default=3,
                    help="steps of the configs[2] lines workload reported under 'secondary' "
                         "(points runs only; 0 = skip)")
    ap.add_argument("--lines-streams", type=int, default=3072,
                    help="streams of the lines workload: the LSD seed loop is one wave per "
                         "frame, latency-bound, so it needs many frames in flight")
    ap.add_argument("--stereo-steps", type=int, default=3,
                    help="steps of the configs[3] stereo workload reported under 'stereo' "
                         "(points runs only; 0 = skip)")
    ap.add_argument("--stereo-streams", type=int, default=256)
    ap.add_argument("--rig-steps", type=int, default=3,
                    help="steps of the configs[4] 8-camera rig workload reported under 'rig' "
                         "(points runs only; 0 = skip)")
    ap.add_argument("--rig-streams", type=int, default=256, help="rig cameras per GPU (x8)")
    ap.add_argument("--ate-streams", type=int, default=8,
                    help="streams of the untimed accuracy leg (ATE vs ground truth and vs the "
                         "reference restatement over one loop); 0 = skip")
    ap.add_argument("--isolated-steps", type=int, default=5,
                    help="untimed non-pipelined steps after the timed region: per-kernel "
                         "times without the other stream's interference (roofline.isolated)")
    ap.add_argument("--pipelined", type=int, default=-1,
                    help="1 = overlap extraction of step t+1 with tracking of step t; 0 = no; "
                         "-1 = per workload (on, except for the LSD-bound lines workload)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    from _pkg import load_pkg
    pkg = load_pkg()
    import orbpl.synth as synth

    res = run_workload(pkg, synth, args, args.workload, args.streams, args.steps, args.warmup,
                       rank, world, local_rank, dist)
    # other BASELINE configs, same clock discipline, fewer steps (points runs only):
    # configs[2] (ORB + LSD/LBD lines) under "secondary", configs[3] (stereo) under "stereo",
    # configs[4] (1280x720 8-camera rig) under "rig"
    others = {}
    if args.workload == "points" and args.secondary_steps > 0:
        others["secondary"] = ("lines", run_workload(
            pkg, synth, args, "lines", args.lines_streams, args.secondary_steps,
            max(1, args.warmup // 2), rank, world, local_rank, dist), args.secondary_steps)
    if args.workload == "points" and args.stereo_steps > 0:
        others["stereo"] = ("kitti", run_workload(
            pkg, synth, args, "kitti", args.stereo_streams, args.stereo_steps,
            max(1, args.warmup // 2), rank, world, local_rank, dist), args.stereo_steps)
    if args.workload == "points" and args.rig_steps > 0:
        others["rig"] = ("rig", run_workload(
            pkg, synth, args, "rig", args.rig_streams, args.rig_steps,
            max(1, args.warmup // 2), rank, world, local_rank, dist), args.rig_steps)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        thr = args.cpu_threads or min(16, os.cpu_count() or 1)
        fps, nfr, dt = cpu_baseline(args.cpu_seconds, thr, res["gray"], res["depth"],
                                    res["layout"], args.workload)
        if res["T_acc"] is not None:
            res["T_ref"] = accuracy_ref(res["gray"], res["depth"], res["layout"],
                                        len(res["T_acc"]), args.workload)
        for key, (wname, o, _) in others.items():
            if o["T_acc"] is not None:
                o["T_ref"] = accuracy_ref(o["gray"], o["depth"], o["layout"], len(o["T_acc"]), wname)
        cpu = {"value": round(fps, 2), "unit": "frames/s", "cores": thr, "kind": "port",
               "sample": f"{nfr} frames of the same {res['image']} loop in {dt:.1f} s, oracle/ "
                         f"C++ restatement ({args.workload} workload), one stream per thread"}

    if rank == 0:
        S = res["S"]
        out = {
            "metric": "frames/sec (extract+match+pose) at 640x480; ATE RMSE vs ref",
            "value": round(res["value"], 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(res["elapsed"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": res["data"],
            "config": {"workload": res["workload"],
                       "image": res["image"], "nfeatures": res["nfeatures"], "streams_per_gpu": S,
                       "frames_per_step": S * world, "parallelism": f"streams sharded x{world}"},
            "stage_ms": res["stages"],
            "tracking": res["tracking"],
            "roofline": res["roof"],
            "cpu_baseline": cpu,
        }
        if res["T_acc"] is not None:
            out["accuracy"] = ate_report(res["T_acc"], res.get("T_ref"), res["layout"])
        for key, (wname, o, nsteps) in others.items():
            out[key] = {
                "workload": o["workload"], "value": round(o["value"], 2),
                "unit": "frames/s", "image": o["image"], "nfeatures": o["nfeatures"],
                "steps": nsteps, "streams_per_gpu": o["S"],
                "ms_per_step": round(o["elapsed"] / nsteps * 1e3, 3),
                "stage_ms": o["stages"], "tracking": o["tracking"], "roofline": o["roof"],
                "data": o["data"]}
            if o["T_acc"] is not None:
                out[key]["accuracy"] = ate_report(o["T_acc"], o.get("T_ref"), o["layout"])
            if cpu is not None:
                thr = cpu["cores"]
                fps, nfr, dt = cpu_baseline(args.cpu_seconds / 2, thr, o["gray"], o["depth"],
                                            o["layout"], wname)
                out[key]["cpu_baseline"] = {
                    "value": round(fps, 2), "unit": "frames/s", "cores": thr, "kind": "port",
                    "sample": f"{nfr} frames in {dt:.1f} s, oracle/ C++ restatement "
                              f"({wname} workload), one stream per thread"}
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
