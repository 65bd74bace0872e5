#!/usr/bin/env python3
"""Benchmark: frames/sec of the per-frame hot path (extract + match + pose).

BASELINE.json metric "frames/sec (extract+match+pose) at 640x480", quoted on
configs[1] = "TUM fr1_desk RGB-D, ORB point features only, 1 MI355X":
TUM1.yaml camera + distortion, ORB 1000 features / 1.2 / 8 levels / FAST 20,7.

A step = one pass of the reference's per-frame Tracking::Track() (ORB
extraction, Frame glue, KeyFrame::ComputeBoW, TrackWithMotionModel or
TrackReferenceKeyFrame, TrackLocalMap, the keyframe push) over a batch of
`--streams` independent synthetic 640x480 RGB-D streams (default 2048), all
inputs resident in HBM before the timed region. The other BASELINE configs are timed
the same way and reported in the same JSON line: configs[2] (TUM3, ORB +
LSD/LBD LineExtractor, LineMatcher::SearchByProjection, line edges) under
"secondary", configs[3] (KITTI 00 camera, 1241x376 rectified stereo pairs, ORB
2000 on both images, ComputeStereoMatches, LineExtractor on both images with
the defined stereo line depths, th = 7, pose with line edges) under "stereo",
configs[4] (1280x720 8-camera rig) under "rig". Frames are rendered from a
seeded textured room along closed-loop trajectories (no datasets on the box).

Parity: every timed tracker records its streams' poses and counts on the
device (orbpl_tracker_set_history); after the timed region streams 0, S/2 and
S-1 of every rank are replayed by the CPU oracle on the same frames and
compared (counts exact, pose max-abs < 1e-4) under "parity".

Multi-GPU: `--gpus N` (without torchrun's environment) starts N ranks with
torch.distributed.run before anything touches the GPU; under torchrun each
rank reads RANK / LOCAL_RANK / WORLD_SIZE, uses device LOCAL_RANK (mod the
visible devices) and tracks its own streams (weak scaling, no data-path
collective); the gloo group carries the barriers, the max-over-ranks time and
the per-rank parity reports.

Prints ONE JSON line (rank 0). See DESIGN.md §5 for the roofline accounting.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

import numpy as np

# HIP hardware queues per process, read when the HIP runtime starts (nothing
# above touches it): a tracker drives up to eight streams at once (ORB
# extraction and LSD each in two offset halves, the line glue, tracking, host
# copies; the right image's ORB and LSD in stereo), and the bench holds one
# tracker per leg. With the runtime's default of 4 queues, streams share a
# queue and their kernels serialise (at 16 queues vs 4 / 8,
# stereo 3.4k / 3.2k -> 4.9k, lines 13.0k / 11.5k -> 13.1k frames/s).
# (the GPU box exports the default 4 explicitly, so raise rather than default)
if int(os.environ.get("GPU_MAX_HW_QUEUES") or 0) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "tests"))

W, H = 640, 480
ORB = (1000, 1.2, 8, 20, 7)
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8 TB/s spec
POSE_TOL = 1e-4         # north_star: pose within 1e-4

# BASELINE.json configs[1..4]: camera (orbpl.synth), ORB parameters, sensor
WORKLOADS = {
    "points": dict(cam="TUM1", orb=ORB, lines=False, stereo=False,
                   desc="TUM fr1_desk-like RGB-D, ORB points only (configs[1])",
                   data="synthetic (seeded textured-room RGB-D loop, TUM1 intrinsics+distortion)"),
    "lines": dict(cam="TUM3", orb=ORB, lines=True, stereo=False,
                  desc="TUM fr3_structure_texture_far-like RGB-D, ORB + LSD/LBD lines (configs[2])",
                  data="synthetic (seeded textured-room RGB-D loop, TUM3 intrinsics, no distortion)"),
    "kitti": dict(cam="KITTI00", orb=(2000, 1.2, 8, 20, 7), lines=True, stereo=True, fps=10,
                  desc="KITTI 00-like stereo 1241x376, ORB 2000 + LSD/LBD on both images, "
                       "ComputeStereoMatches + stereo line depths (defined mode P17) + "
                       "PoseOptimizationWithLines (configs[3])",
                  data="synthetic (seeded textured-room rectified stereo loop, KITTI 00 intrinsics, "
                       "bf 386.1448)"),
    "kitti_points": dict(cam="KITTI00", orb=(2000, 1.2, 8, 20, 7), lines=False, stereo=True, fps=10,
                         desc="KITTI 00-like stereo 1241x376, ORB 2000 both images + "
                              "ComputeStereoMatches + PoseOptimization (points only)",
                         data="synthetic (seeded textured-room rectified stereo loop, KITTI 00 "
                              "intrinsics, bf 386.1448)"),
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


def lsd_access_volume(counts):
    """Per-frame ACCESS VOLUME of the sequential LSD in the kernels' layout,
    from the oracle's element-access counts (oracle.lsd_traffic, averaged over
    sampled frames of the workload): every access charged as if served from
    memory with no reuse - the traffic of a cacheless machine, a ceiling on
    what a kernel with any reuse should move, not a floor.
      pseudo-order sort: (compares + element writes) x 4 B packed key;
      seed loop: seeds x (4 B key + 8 B pixel word) + neighbour reads x 16 B
        (the paired word: angle, claim stamp, cos, sin) + adds x (8 B stamp +
        16 B list entry) + expansions x 16 B + fit list reads / writes x 16 B;
      NFA validation: rectangle pixels x 4 B angle + evaluations x 96 B
        (the rectangle's 12 doubles)."""
    c = counts
    return {"lsd_sort": 4 * (c["sort_cmp"] + c["sort_moves"]),
            "lsd_seed": (12 * c["seeds"] + 16 * c["grow_nb"] + 24 * c["grow_add"] +
                         16 * c["grow_expand"] + 16 * (c["fit_reads"] + c["fit_writes"])),
            "lsd_validate": 4 * c["nfa_px"] + 96 * c["nfa_evals"]}


def lsd_unique_floor(counts):
    """Per-frame UNIQUE-BYTES floor of the LSD kernels: the distinct addresses
    the sequential algorithm touches (the oracle's touched-address bitmaps,
    oracle/lsd_oracle.cpp LsdTraffic), each fetched or stored once in the
    kernels' layout.
      sort: every pseudo-ordered key read once and written once (2 x 4 B);
      seed loop: the seed list's keys (4 B each), the distinct pixel words
        read (16 B: angle, stamp, cos, sin), the distinct USED stamps written
        (8 B), the distinct weights q read (4 B), the longest region list
        written and read once (2 x 16 B per entry), the rectangles out (96 B);
      NFA validation: the distinct rectangle pixels' angles (4 B), the
        rectangles in (96 B) and their verdict + end points out (17 B)."""
    c = counts
    return {"lsd_sort": 8 * c["sort_n"],
            "lsd_seed": (4 * c["seeds"] + 16 * c["u_seed_px"] + 8 * c["u_used_px"] +
                         4 * c["u_q_px"] + 32 * c["max_reg"] + 96 * c["rects"]),
            "lsd_validate": 4 * c["u_nfa_px"] + (96 + 17) * c["rects"]}


def lsd_counts(frames, k=8):
    """oracle.lsd_traffic averaged over k frames spread over `frames`."""
    from _pkg import load_oracle
    O = load_oracle()
    idx = np.linspace(0, len(frames) - 1, min(k, len(frames))).astype(int)
    cs = [O.lsd_traffic(frames[i]) for i in idx]
    out = {key: float(np.mean([c[key] for c in cs])) for key in cs[0]}
    out["frames_sampled"] = len(idx)
    return out


def algorithmic_bytes(n_kp, w=W, h=H, orb=ORB, n_lines=80):
    """Per-frame algorithmic HBM bytes of each kernel: the
    bytes the kernel must move at minimum (each input read once, each output
    written once, SURVEY §8(d)-style one-pass bytes), with n_kp keypoints per
    frame. LSD works on the 0.8-scaled image (sA pixels, LSD's `scale` of
    LineSegmentDetector). The LSD kernels' unique-bytes floor and access
    volume (lsd_unique_floor, lsd_access_volume) are reported beside these in
    roofline.lsd_floor, never in their place."""
    areas, d = level_areas(w, h, orb)
    S = sum(areas)
    dims = list(zip((int(a) for a in d["width"]), (int(b) for b in d["height"])))
    pads = [(a + 38) * (b + 38) for a, b in dims]
    A0 = w * h
    sA = int(np.ceil(w * 0.8)) * int(np.ceil(h * 0.8))
    return {
        # read the input (level 0) or the previous level, write the padded
        # level; read each level's content + 3 px halo, write the blurred content
        "pyramid": w * h + sum(areas[:-1]) + sum(pads) +
                   sum((a + 6) * (b + 6) for a, b in dims) + S,
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
        # every k_pose launch of the step: TrackWithMotionModel's and
        # TrackLocalMap's over all keypoints (TrackReferenceKeyFrame's runs
        # only where the motion model failed: counted as 0 bytes)
        "pose_all": n_kp * 50 * 2,
        # SearchLocalPoints: the frame (kp 28 + desc 32 + ur 4 + nobs 4 + match
        # out 4) and ~4 local map points per keypoint (desc 32, projection +
        # level + view cos + in-view 25 B)
        "match_local": n_kp * 72 + 4 * n_kp * 57,
        # LSD: read the image, write the scaled u8 image, the angle (f32) and
        # the gradient-norm key (i32) per scaled pixel
        "lsd_prep": A0 + sA * 9,
        # pseudo-ordering: read the keys, write the pixel order (4 B each)
        "lsd_sort": sA * 8,
        # seed loop: read the order, the angles and the USED/region state once,
        # write the state once (4 + 4 + 1 + 1 B per scaled pixel)
        "lsd_seed": sA * 10,
        # NFA validation: each rectangle's pixels' angles, bounded by one read
        "lsd_validate": sA * 4,
        # KeyLines: segments in (16 B x ~1500), 80 KeyLines (68 B) + 80 coef (24 B) out
        "keylines": 1500 * 16 + n_lines * (68 + 24),
        # LBD: read the image, 5x5 blur out + in, Sobel dx/dy i16 out + in,
        # 80 x 32 B descriptors out
        "lbd": A0 + 2 * A0 + 2 * 4 * A0 + n_lines * 32,
        # UndistortKeyLines + line depths: 80 KeyLines in and out, 160 depth reads
        "line_prepare": n_lines * (68 * 2 + 8 + 8),
    }


def frame_bytes(n_kp, w=W, h=H, orb=ORB, lines=False, stereo=False):
    """SURVEY.md §8(d) whole-frame algorithmic bytes: B_orb = 7 S - A_last +
    60 N (read the input, write levels 1-7, read levels 0-6 for the resize,
    FAST read, blur read + write, orientation read, descriptor read, 28 B
    keypoint + 32 B descriptor out); lines add LSD A0 + 6 (0.64 A0) 4 +
    2 (0.64 A0) and LBD A0 + 8 A0. Stereo extracts both images."""
    areas, _ = level_areas(w, h, orb)
    S = sum(areas)
    A0 = w * h
    b = 7 * S - areas[-1] + 60 * n_kp
    if lines:
        b += A0 + 6 * 0.64 * A0 * 4 + 2 * 0.64 * A0 + A0 + 8 * A0
    return int(b * (2 if stereo else 1))


KERNELS = {"pyramid": "k_pyramid", "fast": "k_fast_cells", "octree": "k_octree",
           "orient_desc": "k_orient_desc", "match": "k_match_last", "pose": "k_pose",
           "pose_all": "k_pose", "match_local": "k_match_local",
           "lsd_prep": "k_lsd_prep", "lsd_sort": "k_lsd_sort+k_lsd_sort_wave",
           "lsd_seed": "k_lsd_spec", "lsd_validate": "k_lsd_validate+k_lsd_compact",
           "keylines": "k_keylines", "lbd": "k_blur_sobel+k_lbd",
           "line_prepare": "k_line_prepare"}


def pmc_traffic(kernel, workload, streams):
    """HBM bytes per launch of `kernel` from the committed PMC summary of the
    same workload (tools/prof.sh + tools/pmc_traffic.py: FETCH_SIZE x2 gfx950
    correction + WRITE_SIZE), scaled to this run's frames per launch (the
    kernel's "frames_per_launch" in the summary, else its stream count). PMC counters
    need their own rocprofv3 passes, so they cannot be read live. Stage
    kernels joined with '+' sum their parts."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        f = ROOT / "profiles" / rnd / f"pmc_traffic_{workload}.json"
        if not f.exists() and workload == "points":
            f = ROOT / "profiles" / rnd / "pmc_traffic.json"
        if not f.exists():
            continue
        d = json.load(open(f))
        meta = d.get("_meta", {})
        parts = kernel.split("+")
        es = [d.get(k) for k in parts]
        if all(e and e.get("traffic_bytes") for e in es) and meta.get("streams"):
            per = es[0].get("frames_per_launch", meta["streams"])
            tb = sum(e["traffic_bytes"] for e in es)
            return (int(tb * streams / per),
                    f"{f.relative_to(ROOT)} ({per} frames per launch, scaled)")
    return None, None


def oracle_flags(O, args):
    return ((O.TRACK_LOCAL_MAP if args.local_map else 0) |
            (O.TRACK_FIXED_LINE_JAC if args.fixed_line_jacobian else 0) |
            (O.TRACK_REFKF if args.refkf and args.bow else 0))


# the shared vocabulary's node arrays (build_vocabulary): the oracle loops get
# the same tree (KeyFrame::ComputeBoW, TrackReferenceKeyFrame)
VOCAB = {"arrays": None, "oracle": None}


def oracle_vocabulary(O):
    if VOCAB["arrays"] is None:
        return None
    if VOCAB["oracle"] is None:
        VOCAB["oracle"] = O.Vocabulary(arrays=VOCAB["arrays"])
    return VOCAB["oracle"]


def map_mode(args, wl):
    """Tracking::Track with the reference's map model (ORBPL_TRACK_MAP) for
    every workload (RGB-D and, through orbpl_tracker_step_stereo, stereo)."""
    return bool(args.map)


def leg_summary(out):
    """A compact copy of every leg's headline figures (value, ms per step,
    roofline fraction, parity), the batch-1 latencies and the reference-faithful
    CPU per-frame times, emitted as the JSON line's last key so that a log cut
    to its tail still carries the north-star (points + lines) numbers."""
    def leg(o):
        if not o:
            return None
        roof = o.get("roofline") or {}
        par = o.get("parity") or {}
        return {"value": o.get("value"), "ms_per_step": o.get("ms_per_step"),
                "streams": o.get("streams_per_gpu", (o.get("config") or {}).get("streams_per_gpu")),
                "frac": roof.get("frac"), "kernel": roof.get("kernel"),
                "parity_pass": par.get("pass") if isinstance(par, dict) else None}
    s = {"points": leg(out)}
    for k in ("secondary", "stereo", "rig", "ingress"):
        if k in out:
            s[k] = leg(out[k])
    sw = out.get("sweep") or {}
    s["batch1_ms"] = {k: (v[0].get("latency_ms_per_step") if v else None) for k, v in sw.items()}
    for k in ("trk_load",):
        if k in out:
            s[k] = out[k]
    cpu = out.get("cpu_baseline") or {}
    rf = {"points": (cpu.get("reference_faithful") or {}).get("median_ms_per_frame")}
    if "secondary" in out:
        rf["lines"] = ((out["secondary"].get("cpu_baseline") or {}).get("reference_faithful")
                       or {}).get("median_ms_per_frame")
    s["cpu_reference_faithful_ms"] = rf
    if "secondary" in out and out["secondary"].get("dropin_frame"):
        s["dropin_frame_ms"] = out["secondary"]["dropin_frame"].get("median_ms_per_frame")
    return s


COMPACT_MAX = 6000   # bytes: the driver reads the line from an 8 KB tail


def _roof_compact(r):
    if not r:
        return None
    keep = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "traffic_source",
            "traffic_over_algorithmic", "algorithmic_bytes_per_launch", "avg_launch_ms",
            "frames_per_launch", "launches_per_step")
    c = {k: r.get(k) for k in keep}
    iso = r.get("isolated_dominant")
    if iso:
        c["isolated_dominant"] = {k: iso.get(k) for k in ("kernel", "avg_launch_ms", "frac",
                                                          "traffic", "traffic_source")}
    if r.get("pipeline"):
        c["pipeline_frac"] = r["pipeline"].get("frac")
    return c


def compact_line(out, detail):
    """The one JSON line stdout ends with (<= COMPACT_MAX bytes): the
    contract's keys, the dominant kernel's roofline, the CPU baseline, the
    parity verdict and every leg's headline figures. Everything else (stage
    times, sweeps, LSD floors, per-kernel GB/s, host facts) is in the side
    file named by "detail"."""
    cpu = out.get("cpu_baseline")
    par = out.get("parity") or {}
    c = {k: out.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup",
                                 "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
                                 "dtype", "data", "config")}
    c["roofline"] = _roof_compact(out.get("roofline"))
    c["cpu_baseline"] = None if cpu is None else {
        "value": cpu.get("value"), "unit": cpu.get("unit"), "cores": cpu.get("cores"),
        "kind": cpu.get("kind"), "sample": cpu.get("sample"),
        "host": (cpu.get("host") or {}).get("model"),
        "reference_faithful_ms": (cpu.get("reference_faithful") or {}).get("median_ms_per_frame"),
        "reference_faithful_fps": (cpu.get("reference_faithful") or {}).get("value")}
    legs = [par] + [(out.get(k) or {}).get("parity") or {} for k in
                    ("secondary", "stereo", "rig", "ingress")]

    def passed(p):   # one rank's report, or the gathered {"all_ranks_pass", "by_rank"}
        return p.get("all_ranks_pass", p.get("pass")) if isinstance(p, dict) and p else None
    if isinstance(par, dict) and "by_rank" in par:
        par = dict((par["by_rank"] or [None])[0] or {}, all_ranks_pass=par.get("all_ranks_pass"))
    c["parity"] = {"pass": all(passed(p) is not False for p in legs),
                   "headline_pass": passed(par),
                   "max_abs_pose_diff": par.get("max_abs_pose_diff_vs_ref"),
                   "pose_tol": par.get("pose_tol"), "counts_equal": par.get("counts_equal"),
                   "ate_rmse_vs_gt_m": par.get("ate_rmse_vs_gt_m"),
                   "ref_ate_rmse_vs_gt_m": par.get("ref_ate_rmse_vs_gt_m")}
    s = dict(out.get("summary") or {})
    for k in ("secondary", "stereo", "rig"):
        o = out.get(k)
        if o and s.get(k):
            s[k] = dict(s[k], roofline=_roof_compact(o.get("roofline")),
                        cpu_fps=(o.get("cpu_baseline") or {}).get("value"))
    s.pop("trk_load", None)
    c["summary"] = s
    c["detail"] = detail
    if len(json.dumps(c)) > COMPACT_MAX:       # never print a line the driver cannot take
        for k in ("secondary", "stereo", "rig"):
            if s.get(k):
                s[k].pop("roofline", None)
    return c


def map_capacity(total_steps):
    """Keyframe slots per stream for a tracker that runs `total_steps` steps:
    at most one keyframe per step, so the map never declines one (the
    ORBPL_MAP_KF environment read at tracker creation; 64 at most). Beyond 63
    steps a stream may run out of slots (capacity flag 1, a declined keyframe,
    no longer the reference's map): say so loudly; the run's parity check and
    `map_capacity_flags` then show whether it happened."""
    if total_steps + 1 > 64:
        print(f"bench: WARNING {total_steps} steps exceed the 63 keyframes the map model's "
              f"64-slot table (ORBPL_MAP_KF) guarantees; a stream that inserts more declines "
              f"keyframes (capacity flag 1)", file=sys.stderr, flush=True)
    os.environ["ORBPL_MAP_KF"] = str(max(2, min(64, total_steps + 1)))


def oracle_vo(O, wl, flags=0, use_map=False):
    """The oracle's tracking loop for a workload (oracle/line_track_oracle.cpp
    LVO, or map_oracle.cpp MapVO for the map model, with the tracker's flags
    and vocabulary); returns (vo, step(vo, a, b))."""
    import orbpl.synth as synth
    cam = O.camera(getattr(synth, wl["cam"]))
    if use_map:
        vo = O.MapVO(O.params(*wl["orb"]), cam, 1, use_lines=wl["lines"],
                     flags=flags | (O.TRACK_STEREO if wl["stereo"] else 0))
        vo.set_fps(wl.get("fps", 30))
    else:
        vo = O.LVO(O.params(*wl["orb"]), cam, 1, use_lines=wl["lines"], flags=flags)
    voc = oracle_vocabulary(O)
    if voc is not None:
        vo.set_vocabulary(voc)
    if wl["stereo"]:
        return vo, lambda vo, a, b: vo.step_stereo(0, a, b)
    return vo, lambda vo, a, b: vo.step(0, a, b)


OUT8 = ("nkeypoints", "nmatches", "ninliers", "nmatches_map", "ok", "nlines", "line_matches",
        "line_nmatches_map", "local_matches", "local_inliers", "local_line_matches",
        "local_line_inliers")


def parity_check(T_gpu, C_gpu, streams, gray, depth, L, workload, flags=0, use_map=False):
    """Replay `streams` of the timed tracker on the CPU oracle over the same
    frames (one host thread per stream) and compare every step: the 12 counts
    (24 with the map model: + keyframe decisions, map sizes, temporal points /
    lines, reference keyframe, state, local map sizes) exactly, the pose to
    POSE_TOL. T_gpu[k]: (n, 4, 4), C_gpu[k]: (n, 12 | 24)."""
    from _pkg import load_oracle
    import orbpl.tum as tum
    O = load_oracle()
    wl = WORKLOADS[workload]
    keys = O.MAP_COUNTS if use_map else OUT8
    n = min(len(T) for T in T_gpu)
    T_ref = np.zeros((len(streams), n, 4, 4), np.float32)
    C_ref = np.zeros((len(streams), n, len(keys)), np.int32)

    errors = []

    def worker(k, s):
        try:
            vo, vstep = oracle_vo(O, wl, flags, use_map)
            vo.reset(np.linalg.inv(L.Twc(s, 0)).astype(np.float32).reshape(1, 16))
            for t in range(n):
                e = L.elem(s, t)
                T, st = vstep(vo, gray[e], depth[e])
                if not use_map:
                    st.update(vo.local_stats(0))
                T_ref[k, t] = T
                C_ref[k, t] = [st[key] for key in keys]
        except Exception as ex:  # surface, do not let a thread swallow it
            errors.append(ex)

    ths = [threading.Thread(target=worker, args=(k, s)) for k, s in enumerate(streams)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errors:
        raise errors[0]
    Tg = np.stack([T[:n] for T in T_gpu])
    Cg = np.stack([c[:n] for c in C_gpu])
    bad = [(int(streams[k]), int(t), keys[i]) for k, t, i in zip(*np.nonzero(Cg != C_ref))]
    dmax = float(np.abs(Tg - T_ref).max()) if n else 0.0
    gt = np.stack([np.linalg.inv(L.Twc(s, t)) for s in streams for t in range(n)])
    cg = tum.camera_centres(Tg.reshape(-1, 4, 4))
    cr = tum.camera_centres(T_ref.reshape(-1, 4, 4))
    cgt = tum.camera_centres(gt)
    out = {"source": "timed tracker (device-side per-step history)", "streams": [int(s) for s in streams],
            "steps_checked": n, "counts_equal": not bad, "count_mismatches": bad[:10],
            "max_abs_pose_diff_vs_ref": float(f"{dmax:.3e}"), "pose_tol": POSE_TOL,
            "pass": (not bad) and dmax < POSE_TOL,
            "ate_rmse_vs_gt_m": round(tum.ate(cg, cgt)["rmse"], 6) if n > 2 else None,
            "ref_ate_rmse_vs_gt_m": round(tum.ate(cr, cgt)["rmse"], 6) if n > 2 else None,
            "oracle": "MapVO (map model)" if use_map else "LVO"}
    if use_map and n:
        kf = keys.index("keyframes")
        out["keyframes_last_step"] = [int(c) for c in C_ref[:, n - 1, kf]]
        out["keyframes_created"] = int((C_ref[:, :, keys.index("keyframe")] == 1).sum())
    return out


def max_over_ranks(dist, elapsed):
    """The timed region's wall time, max over ranks (gloo all_reduce)."""
    if not dist:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_parity(dist, world, parity):
    """Every rank's parity report on every rank (gloo all_gather_object)."""
    if not dist:
        return parity
    allp = [None] * world
    dist.all_gather_object(allp, parity)
    return {"all_ranks_pass": all(p is not None and p["pass"] for p in allp), "by_rank": allp}


def torchrun_cmd(ngpus, argv, port):
    """The command `--gpus N` runs: one rank per GPU under torch.distributed.run."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={ngpus}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            str(Path(__file__).resolve())] + list(argv)


def share_tree(tree, dist):
    """Rank 0's vocabulary tree on every rank (broadcast)."""
    if dist:
        box = [tree]
        dist.broadcast_object_list(box, src=0)
        tree = box[0]
    return tree


def shared_idf(synth, tree, docs, dist, rccl_device=None):
    """TF-IDF word weights (synth.idf_weights) over every rank's training
    documents: each rank counts the documents its words occur in, one SUM
    all-reduce of the counts (+ the document count) - RCCL on `rccl_device`
    when given, gloo otherwise."""
    nn = len(tree["parent"])
    ni = np.zeros(nn + 1, np.float64)
    for d in docs:
        ni[np.unique(synth.vocabulary_words(tree, d))] += 1
    ni[nn] = len(docs)
    backend = "none"
    if dist:
        import torch
        if rccl_device is not None:
            backend = "rccl"
            if not hasattr(shared_idf, "group"):
                shared_idf.group = dist.new_group(backend="nccl")
            torch.cuda.set_device(rccl_device)
            t = torch.from_numpy(ni).to(f"cuda:{rccl_device}")
            dist.all_reduce(t, group=shared_idf.group)
            ni = t.cpu().numpy()
        else:
            backend = "gloo"
            t = torch.from_numpy(ni)
            dist.all_reduce(t)
            ni = t.numpy()
    n_docs, ni = ni[nn], ni[:nn]
    return synth.idf_weights(tree, ni, n_docs), int(n_docs), backend


def build_vocabulary(pkg, synth, args, rank, world, device, dist):
    """The ORB vocabulary every rank's trackers share: rank 0
    builds the tree (seeded hierarchical k-medians, synth.vocabulary_tree, on
    the GPU extractor's descriptors of its rendered training frames) and
    broadcasts it; the TF-IDF weights come from every rank's own training
    frames through one all-reduce (shared_idf)."""
    k, L = 10, args.vocab_levels
    frames, _ = render_loop(6, seed=100 + rank, workers=min(16, os.cpu_count() or 4))
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, width=W, height=H, device=device)
    docs = [ex(f)[1] for f in frames]
    ex.close()
    tree = share_tree(synth.vocabulary_tree(docs, k=k, L=L, seed=1) if rank == 0 else None, dist)
    rccl = None
    if dist:
        import torch
        if pkg.device_count() >= world and torch.cuda.is_available():
            rccl = device
    w, n_docs, backend = shared_idf(synth, tree, docs, dist, rccl)
    arrays = dict(parent=tree["parent"], leaf=tree["leaf"], desc=tree["desc"], weight=w, k=k, L=L,
                  scoring=0, weighting=0)
    voc = pkg.ORBVocabulary(arrays=arrays, device=device)
    VOCAB["arrays"] = arrays
    info = {"k": k, "L": L, "nodes": voc.n_nodes, "words": voc.n_words,
            "stopped_words": int(((w == 0) & tree["leaf"]).sum()), "levelsup": 4,
            "documents": n_docs, "idf_reduction": backend,
            "source": "synthetic: seeded hierarchical k-medians on rendered frames' ORB "
                      "descriptors (the reference's ORBvoc.txt is not in its checkout)"}
    return voc, info


def run_workload(pkg, synth, args, workload, S, steps, warmup, rank, world, device, dist, voc=None):
    """Time `steps` tracker steps of one workload; returns the measurements."""
    wl = WORKLOADS[workload]
    lines, stereo, cam_name = wl["lines"], wl["stereo"], wl["cam"]
    cams = wl.get("cams", 1)
    F = (args.loop if workload == args.workload else args.loop_other) if cams == 1 else args.rig_loop
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
    d_gray = pkg.DeviceBuffer.from_array(gray[rep], device=device)
    d_depth = pkg.DeviceBuffer.from_array(depth[rep], device=device)
    cam = pkg.make_camera(getattr(synth, cam_name))
    use_map = map_mode(args, wl)
    map_capacity(warmup + steps + (args.isolated_steps if args.isolated_steps > 0 else 0)
                 + (3 if args.trk_load else 0))
    tr = pkg.Tracker(pkg.OrbParams(*wl["orb"]), cam, S, device=device, lines=lines, stereo=stereo,
                     local_map=bool(args.local_map) and not use_map,
                     fixed_line_jac=bool(args.fixed_line_jacobian),
                     refkf=bool(args.refkf and voc is not None), map=use_map)
    if use_map:
        tr.set_fps(wl.get("fps", 30))   # Camera.fps: mMaxFrames (KITTI 10, TUM 30)
    # pipelining overlaps extraction of step t+1 with tracking of step t, for
    # every workload (lines too: the next batch's LSD overlaps this batch's
    # matching and pose, 9.5k -> 9.8k frames/s at 3072 streams)
    pipelined = args.pipelined if args.pipelined >= 0 else 1
    tr.set_pipelined(bool(pipelined))
    if voc is not None:
        tr.set_vocabulary(voc, 4)    # KeyFrame::ComputeBoW of every frame (P18)
    tr.reset(np.stack([np.linalg.inv(L.Twc(s, 0)).astype(np.float32) for s in range(S)]).reshape(S, 16))
    tr.set_history(warmup + steps)
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
    elapsed = max_over_ranks(dist, t1 - t0)
    st = tr.state()
    tim = tr.timings(steps)                            # (steps, 11) ms, in-stream hipEvents
    avg = tim.mean(0)
    stages = dict(zip(tr.STAGES, [round(float(x), 4) for x in avg]))
    stage_avg = dict(zip(tr.STAGES, [float(x) for x in avg]))

    def kernel_sums(kt):
        """GPU time per step of the kernels that run in several stages:
        k_pose summed over its launches, k_match_local alone."""
        k = dict(zip(tr.KERNEL_STAGES, [float(x) for x in kt.mean(0)]))
        return {"pose_all": k["pose_motion"] + k["pose_refkf"] + k["pose_local"],
                "match_local": k["match_local"]}, k

    ksum, kraw = kernel_sums(tr.kernel_timings(steps))
    stage_avg.update(ksum)
    stages.update({f"kernel_{k}": round(v, 4) for k, v in kraw.items()})
    tracking = {"mean_keypoints": float(st["nkeypoints"].mean()),
                "mean_matches": float(st["nmatches"].mean()),
                "mean_inliers": float(st["ninliers"].mean()),
                "ok_frac": float(tr.status()["ok"].mean())}
    if args.local_map or use_map:
        lst = tr.local_stats()
        tracking.update(mean_local_matches=float(lst["local_matches"].mean()),
                        mean_local_inliers=float(lst["local_inliers"].mean()))
        if lines:
            tracking.update(mean_local_line_matches=float(lst["local_line_matches"].mean()),
                            mean_local_line_inliers=float(lst["local_line_inliers"].mean()))
    if lines:
        lt = tr.line_timings(steps).mean(0)
        stages.update(zip(tr.LINE_STAGES, [round(float(x), 4) for x in lt]))
        ls_t = tr.lsd_timings(steps).mean(0)
        stages.update(zip(tr.LSD_STAGES, [round(float(x), 4) for x in ls_t]))
        stage_avg.update(zip(tr.LSD_STAGES, [float(x) for x in ls_t]))
        ls = tr.status()
        tracking.update(mean_lines=float(ls["nlines"].mean()),
                        mean_line_matches=float(ls["line_matches"].mean()))
    if stereo:
        stt = tr.stereo_timings(steps).mean(0)
        stages.update(zip(tr.STEREO_STAGES, [round(float(x), 4) for x in stt]))
    frames = S * steps * world
    value = frames / elapsed

    # device-side history of the timed tracker: streams 0, S/2, S-1
    samp = sorted({0, S // 2, S - 1})
    hist = [(tr.history(s, warmup + steps)[0], tr.map_history(s, warmup + steps)) if use_map
            else tr.history(s, warmup + steps) for s in samp]
    if use_map:
        mh = np.stack([h[1][-1] for h in hist])
        ki = {k: i for i, k in enumerate(tr.MAP_COUNTS)}
        tracking.update(
            sampled_streams_keyframes=[int(x) for x in mh[:, ki["keyframes"]]],
            sampled_streams_map_points=[int(x) for x in mh[:, ki["map_points"]]],
            sampled_streams_map_lines=[int(x) for x in mh[:, ki["map_lines"]]],
            keyframes_created_sampled=int(sum((h[1][:, ki["keyframe"]] == 1).sum() for h in hist)),
            map_capacity_flags=int(tr.map_errors().max()))

    # roofline of the dominant single-stage kernel
    n_kp = float(st["nkeypoints"].mean())
    lsdc = lsd_counts(gray) if lines else None
    ab = algorithmic_bytes(n_kp, fw, fh, wl["orb"])
    # candidates: every kernel's GPU time per step, a kernel launched in
    # several stages (k_pose: motion model, reference keyframe, local map)
    # counted once with all its launches
    # (stereo: the match stage's events also bracket the wait for the right
    # image's extraction and k_stereo, not one kernel: left out)
    cand = ["pyramid", "fast", "octree", "orient_desc"] + ([] if stereo else ["match"]) + ["pose_all"]
    if args.local_map or use_map:
        cand.append("match_local")
    if lines:
        # (line_prepare: its events run from the first LSD half's LBD to the end
        # of k_line_prepare on the line stream, so they bracket the wait for the
        # second half's chain (and, stereo, the right image's lines and
        # k_stereo_lines), not one kernel: left out)
        cand += [k for k in tr.LSD_STAGES if k != "line_prepare"]
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
        iso = dict(zip(tr.STAGES, [float(x) for x in tr.timings(args.isolated_steps).mean(0)]))
        iso.update(kernel_sums(tr.kernel_timings(args.isolated_steps))[0])
        if lines:
            iso.update(zip(tr.LSD_STAGES,
                           [float(x) for x in tr.lsd_timings(args.isolated_steps).mean(0)]))
    trk_load = None
    if (args.trk_load and use_map and voc is not None and args.refkf
            and workload == args.workload):
        # untimed single steps after the timed region, serialised: a plain
        # step, then steps where 10 % / 100 % of the streams lost their
        # velocity (orbpl_tracker_clear_velocity: the state after
        # initialisation or relocalisation) and so run TrackReferenceKeyFrame
        # (SearchByBoW + the reference-keyframe pose) before TrackLocalMap.
        # Parity of this path: test_map_tracker_reference_keyframe_under_load.
        tr.set_pipelined(False)
        k0 = warmup + steps + max(0, args.isolated_steps)

        def one(k):
            tr.synchronize()
            tr.timings_reset()
            t_a = time.perf_counter()
            step(k)
            tr.synchronize()
            ms = (time.perf_counter() - t_a) * 1e3
            kt = dict(zip(tr.KERNEL_STAGES, [float(x) for x in tr.kernel_timings(1)[-1]]))
            return {"step_ms": round(ms, 3), "trk_section_ms": round(kt["pose_refkf"], 4),
                    "ok_frac": round(float(tr.status()["ok"].mean()), 4)}
        trk_load = {"streams": S, "plain": one(k0)}
        for j, frac in enumerate((0.1, 1.0)):
            every = int(round(1 / frac))
            mask = (np.arange(S) % every) == 0
            tr.clear_velocity(mask)
            r = one(k0 + 1 + j)
            r["streams_trk"] = int(mask.sum())
            trk_load[f"{int(frac * 100)}%"] = r
        trk_load["note"] = ("single non-pipelined steps after the timed region; trk_section_ms = "
                            "hipEvents around TrackReferenceKeyFrame (k_trk_bow, line matcher, "
                            "merge, pose) on the tracking stream")
    # the dominant kernel as rocprofv3 --stats ranks it: the most GPU time per
    # step in the timed (pipelined) region; the isolated steps' dominant
    # kernel is reported beside it (roofline.isolated_dominant)
    # frames per launch: the extraction / LSD batches may be split in two
    # offset halves on two streams; their stage events bracket the first half
    orb_fr, lsd_fr = tr.launch_frames()
    def launch_frames(k):
        return (orb_fr if k in ("pyramid", "fast", "octree", "orient_desc") else
                lsd_fr if k in tr.LSD_STAGES else S)
    # launches per step of a stage's kernel: the timed stage is one launch of
    # launch_frames(k) frames; the step runs S frames through the extraction
    # and S (2 S with the right images, stereo) through the LSD chain
    def per_step(k):
        if k in tr.LSD_STAGES:
            return (2 if stereo else 1) * S / lsd_fr
        return S / launch_frames(k) if k in ("pyramid", "fast", "octree", "orient_desc") else 1
    dom = max(cand, key=lambda k: stage_avg[k] * per_step(k))
    dom_iso = max(cand, key=lambda k: iso.get(k, 0.0)) if iso is not None else dom
    dom_ms = stage_avg[dom]          # live: timed region, in-stream hipEvents (one launch)
    bytes_launch = int(ab[dom] * launch_frames(dom))
    achieved = bytes_launch / (dom_ms * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic(KERNELS[dom], workload, launch_frames(dom))
    if traffic and dom == "pose_all":
        traffic *= 2          # the PMC summary is per launch; two full launches per step
    fbytes = frame_bytes(n_kp, fw, fh, wl["orb"], lines, stereo)
    roof = {"bound": "hbm", "kernel": KERNELS[dom], "stage": dom,
            "dominance": "summed per-kernel GPU time per step in the timed region (as "
                         "rocprofv3 --stats ranks kernels): one launch's in-stream time x "
                         "the kernel's launches per step",
            "launches_per_step": round(per_step(dom), 3),
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "traffic_source": tsrc,
            "traffic_over_algorithmic": round(traffic / bytes_launch, 2) if traffic else None,
            "algorithmic_bytes_per_launch": bytes_launch, "avg_launch_ms": round(dom_ms, 4),
            "frames_per_launch": launch_frames(dom),
            "per_kernel_GBps": {k: round(ab[k] * launch_frames(k) / (stage_avg[k] * 1e-3) / 1e9, 1)
                                for k in cand if stage_avg[k] > 0}}
    if lsdc:
        # each LSD kernel's committed PMC traffic against three byte counts per
        # frame: the one-pass bytes (algorithmic_bytes), the
        # unique-bytes floor (distinct addresses the sequential algorithm
        # touches) and the access volume (every access with no reuse)
        uf, av = lsd_unique_floor(lsdc), lsd_access_volume(lsdc)
        per = {}
        for k in uf:
            tb, _ = pmc_traffic(KERNELS[k], workload, launch_frames(k))
            pf = tb / launch_frames(k) if tb else None
            per[k] = {"pmc_bytes_per_frame": int(pf) if pf else None,
                      "one_pass_bytes": int(ab[k]), "unique_bytes": int(uf[k]),
                      "access_volume_bytes": int(av[k]),
                      "over_one_pass": round(pf / ab[k], 2) if pf else None,
                      "over_unique": round(pf / uf[k], 2) if pf else None,
                      "over_access_volume": round(pf / av[k], 2) if pf else None}
        roof["lsd_floor"] = {"counts_per_frame": lsdc, "kernels": per,
                             "source": "oracle.lsd_traffic (oracle/lsd_oracle.cpp LsdTraffic: "
                                       "access counts and touched-address bitmaps) on sampled "
                                       "frames of this workload"}
    # whole pipeline: B_frame x frames/s against 8 TB/s
    per_gpu = S * steps / elapsed
    roof["pipeline"] = {"bytes_per_frame": fbytes, "frames_per_s_per_gpu": round(per_gpu, 1),
                        "achieved": round(fbytes * per_gpu / 1e9, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(fbytes * per_gpu / 1e9 / HBM_PEAK_GBS, 5),
                        "formula": "SURVEY.md 8(d): 7 S - A_last + 60 N (+ LSD/LBD for lines; "
                                   "x2 for stereo)"}
    if iso is not None:
        ims = iso[dom]
        roof["isolated"] = {
            "stage_ms": {k: round(v, 4) for k, v in iso.items()},
            "avg_launch_ms": round(ims, 4),
            "achieved": round(bytes_launch / (ims * 1e-3) / 1e9, 2),
            "frac": round(bytes_launch / (ims * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "steps": args.isolated_steps}
        # the kernel with the most GPU time when the two HIP streams are
        # serialised (no CU sharing), at its isolated launch time
        bl_iso = int(ab[dom_iso] * launch_frames(dom_iso))
        t_iso = iso[dom_iso]
        tr_iso, src_iso = pmc_traffic(KERNELS[dom_iso], workload, launch_frames(dom_iso))
        if tr_iso and dom_iso == "pose_all":
            tr_iso *= 2
        roof["isolated_dominant"] = {
            "kernel": KERNELS[dom_iso], "stage": dom_iso, "avg_launch_ms": round(t_iso, 4),
            "algorithmic_bytes_per_launch": bl_iso,
            "achieved": round(bl_iso / (t_iso * 1e-3) / 1e9, 2),
            "frac": round(bl_iso / (t_iso * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "traffic": tr_iso, "traffic_source": src_iso}
    tr.close()
    del d_gray, d_depth
    return dict(S=S, value=value, layout=L, elapsed=elapsed, stages=stages, tracking=tracking,
                roof=roof, gray=gray, depth=depth, workload=wl["desc"], data=wl["data"],
                image=f"{fw}x{fh}", nfeatures=wl["orb"][0], samp=samp, hist=hist, wname=workload,
                pipelined=bool(pipelined), map=use_map, trk_load=trk_load)


def run_ingress(pkg, synth, args, S, steps, warmup, rank, world, device, dist, voc=None,
                loop=None):
    """The headline workload fed from host memory (GrabImageRGBD's inputs):
    u8 gray + 16-bit TUM depth (DepthMapFactor 5000) in page-locked host
    buffers, each step's batch copied host-to-device on the tracker's copy
    stream while the previous steps' kernels run (orbpl_tracker_step_host),
    depth converted on the device. The timed region includes the copies."""
    wl = WORKLOADS["points"]
    F = args.loop
    if loop is not None:   # the headline's rendered loop (same camera, seed and length)
        gray, depth = loop
    else:
        gray, depth = render_loop(F, seed=1 + rank, workers=min(16, os.cpu_count() or 4))
    d16 = np.clip(np.round(depth * 5000.0), 0, 65535).astype(np.uint16)
    d32 = d16.astype(np.float32) * (np.float32(1.0) / np.float32(5000.0))   # P21
    traj = synth.loop_trajectory(F, seed=1 + rank)
    L = Layout(traj)
    rep = L.replicated(S)
    hg = pkg.HostBuffer((len(rep), H, W), np.uint8)
    hd = pkg.HostBuffer((len(rep), H, W), np.uint16)
    hg.array[:] = gray[rep]
    hd.array[:] = d16[rep]
    use_map = map_mode(args, wl)
    map_capacity(warmup + steps)
    tr = pkg.Tracker(pkg.OrbParams(*wl["orb"]), pkg.make_camera(synth.TUM1), S, device=device,
                     local_map=bool(args.local_map) and not use_map,
                     refkf=bool(args.refkf and voc is not None), map=use_map)
    tr.set_pipelined(True)
    if voc is not None:
        tr.set_vocabulary(voc, 4)
    tr.reset(np.stack([np.linalg.inv(L.Twc(s, 0)).astype(np.float32) for s in range(S)]).reshape(S, 16))
    tr.set_history(warmup + steps)

    def step(k):
        o = k % F
        tr.step_host(hg.ptr + o * W * H, hd.ptr + o * W * H * 2, 5000.0)

    for k in range(warmup):
        step(k)
    tr.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        step(warmup + k)
    tr.synchronize()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, time.perf_counter() - t0)
    samp = sorted({0, S // 2, S - 1})
    hist = [(tr.history(s, warmup + steps)[0], tr.map_history(s, warmup + steps)) if use_map
            else tr.history(s, warmup + steps) for s in samp]
    tr.close()
    step_bytes = S * W * H * 3
    out = dict(S=S, value=S * steps * world / elapsed, elapsed=elapsed, nsteps=steps, samp=samp,
               hist=hist, layout=L, gray=gray, depth=d32, wname="points", map=use_map,
               h2d_GBps=round(step_bytes * steps / elapsed / 1e9, 2), bytes_per_step=step_bytes)
    hg.free()
    hd.free()
    return out


def sweep(pkg, synth, workload, sizes, steps, device, local_map=True, voc=None, refkf=False,
          use_map=False):
    """Per-step latency and throughput at several batch sizes (untimed for the
    headline; each size gets its own tracker, 1 warm-up step)."""
    wl = WORKLOADS[workload]
    F = 8
    gray, depth = render_loop(F, seed=7, workers=min(16, os.cpu_count() or 4), cam_name=wl["cam"],
                              stereo=wl["stereo"])
    fh, fw = gray.shape[1:]
    L = Layout(synth.loop_trajectory(F, seed=7))
    cam = pkg.make_camera(getattr(synth, wl["cam"]))
    out = []
    for S in sizes:
        rep = L.replicated(S)
        d_gray = pkg.DeviceBuffer.from_array(gray[rep], device=device)
        d_depth = pkg.DeviceBuffer.from_array(depth[rep], device=device)
        map_capacity(1 + 2 * steps)
        tr = pkg.Tracker(pkg.OrbParams(*wl["orb"]), cam, S, device=device, lines=wl["lines"],
                         stereo=wl["stereo"], local_map=local_map and not use_map,
                         refkf=bool(refkf and voc is not None), map=use_map)
        tr.set_pipelined(True)
        if voc is not None:
            tr.set_vocabulary(voc, 4)
        tr.reset(np.stack([np.linalg.inv(L.Twc(s, 0)).astype(np.float32)
                           for s in range(S)]).reshape(S, 16))
        fb, db = fw * fh, fw * fh * depth.itemsize

        def step(k):
            o = k % F
            if wl["stereo"]:
                tr.step_stereo_device(d_gray.ptr + o * fb, d_depth.ptr + o * db)
            else:
                tr.step_device(d_gray.ptr + o * fb, d_depth.ptr + o * db)

        step(0)
        tr.synchronize()
        lat = []
        for k in range(steps):     # latency: one step issued and waited for
            t0 = time.perf_counter()
            step(1 + k)
            tr.synchronize()
            lat.append(time.perf_counter() - t0)
        t0 = time.perf_counter()   # throughput: steps back to back
        for k in range(steps):
            step(1 + steps + k)
        tr.synchronize()
        thr = S * steps / (time.perf_counter() - t0)
        out.append({"streams": S, "latency_ms_per_step": round(1e3 * float(np.median(lat)), 3),
                    "fps": round(thr, 1)})
        tr.close()
        del d_gray, d_depth
    return out


def host_info():
    """Host CPU facts for the CPU baseline: model, logical CPUs (nproc), the
    CPUs this process may use (affinity) and the cgroup CPU quota."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(p)
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0))
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    # the GPU box gives a one-GPU job a 16-CPU share (nproc shows the whole
    # machine there); OMP_NUM_THREADS carries that share
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit():
        usable = min(usable, int(share))
    return {"model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_quota": quota,
            "usable_cores": usable}


def cpu_baseline(seconds, threads, gray, depth, L, workload="points", flags=0, use_map=False):
    """Throughput mode (BASELINE.md §2 mode 2): the CPU oracle running the
    same per-frame step, one stream per host thread, for a bounded wall time."""
    from _pkg import load_oracle
    O = load_oracle()
    wl = WORKLOADS[workload]
    counts = [0] * threads
    stop = time.time() + seconds

    def worker(k):
        vo, vstep = oracle_vo(O, wl, flags, use_map)
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


def dropin_frame_latency(gray, depth, L, workload, reps=30):
    """Single-frame latency of the compiled drop-in ORB_SLAM2::Frame (ORB ||
    LineExtractor on two host threads + the frame glue, dropin/Frame.cc, one
    frame at a time as the reference's Tracking builds it): dropin_driver
    --time on three frames of the workload's loop; host buffers in and out,
    so the PCIe copies are inside. Returns the driver's median / mean ms."""
    import struct
    import tempfile
    import orbpl.synth as synth
    from _pkg import load_pkg
    pkg_th_depth = load_pkg().th_depth
    drv = ROOT / "orb_slam2_modification_with-point-and-line-feature_amd" / "dropin_driver"
    if not drv.exists():
        return None
    wl = WORKLOADS[workload]
    cfg = getattr(synth, wl["cam"])
    fh, fw = gray.shape[1:]
    with tempfile.TemporaryDirectory() as td:
        voc = Path(td) / "voc.txt"
        voc.write_text("10 1 0 0\n")   # never opened: the timing mode loads no vocabulary
        inp = Path(td) / "in.bin"
        with open(inp, "wb") as f:
            f.write(struct.pack("<2i", fw, fh))
            camv = [cfg["fx"], cfg["fy"], cfg["cx"], cfg["cy"], cfg["k1"], cfg["k2"], cfg["p1"],
                    cfg["p2"], cfg["k3"], cfg["bf"], pkg_th_depth(cfg)]
            f.write(np.asarray(camv, np.float32).tobytes())
            o = wl["orb"]
            f.write(struct.pack("<ifiii", o[0], o[1], o[2], o[3], o[4]))
            f.write(np.eye(4, dtype=np.float32).tobytes())
            for t in range(3):
                e = L.elem(0, t)
                f.write(np.ascontiguousarray(gray[e], np.uint8).tobytes())
                f.write(np.ascontiguousarray(depth[e], np.float32).tobytes())
            pb = str(voc).encode()
            f.write(struct.pack("<i", len(pb)) + pb)
        r = subprocess.run([str(drv), "--time", str(inp), str(reps)], capture_output=True, text=True,
                           timeout=300)
    if r.returncode != 0 or "median" not in r.stdout:
        return {"error": (r.stderr or r.stdout)[-200:]}
    w = r.stdout.split()
    return {"median_ms_per_frame": float(w[w.index("median") + 1]),
            "mean_ms_per_frame": float(w[w.index("mean") + 1]), "frames": reps,
            "what": "compiled drop-in ORB_SLAM2::Frame (ORB || LineExtractor threads + frame "
                    "glue over the C ABI, host images in, host keypoints / lines out)"}


def cpu_reference_faithful(gray, depth, L, workload, flags=0, warmup=20, frames=300,
                           use_map=False):
    """BASELINE.md §2 mode 1: one stream as the reference runs it, ORB and
    the LineExtractor on two host threads per frame (Frame.cc:152-155),
    matching and pose on the tracking thread; per-frame latency with
    std::chrono-like perf_counter over `frames` frames after `warmup` untimed
    ones (20 warm-up, >= 300 timed; the loop wraps).
    Measured in a child process of its own (tools/cpu_faithful.py) on the
    stream's frames and the bench's vocabulary: inside the bench process,
    after the GPU legs and the threaded CPU baseline, the same loop ran 2.6x
    slower on the lines workload (81 vs 31 ms median on one box)."""
    import tempfile
    seq = [L.elem(0, i) for i in range(warmup + frames)]
    uniq = sorted(set(seq))
    pos = {e: k for k, e in enumerate(uniq)}
    with tempfile.TemporaryDirectory() as td:
        f = os.path.join(td, "faithful.npz")
        extra = {}
        if VOCAB["arrays"] is not None:
            extra = {"voc_" + k: np.asarray(v) for k, v in VOCAB["arrays"].items()}
        np.savez(f, gray=gray[uniq], depth=depth[uniq], order=np.array([pos[e] for e in seq]),
                 Tcw0=np.linalg.inv(L.Twc(0, 0)).astype(np.float32).reshape(1, 16),
                 workload=workload, flags=flags, warmup=warmup, use_map=use_map, **extra)
        r = subprocess.run([sys.executable, str(ROOT / "tools" / "cpu_faithful.py"), "--npz", f],
                           capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise RuntimeError(f"cpu_faithful failed: {r.stderr[-2000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def _cpu_list(text):
    out = []
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def _parent_cpus():
    """The CPUs the parent process's threads last ran on (/proc stat field
    39): the bench's own threads, HIP runtime threads included."""
    out = set()
    try:
        ppid = os.getppid()
        for tid in os.listdir(f"/proc/{ppid}/task"):
            st = open(f"/proc/{ppid}/task/{tid}/stat").read()
            out.add(int(st.rsplit(")", 1)[1].split()[36]))
    except (OSError, ValueError, IndexError):
        pass
    return out


def pin_one_ccd(avoid_parent=True):
    """Pin this process (before any thread starts) to the allowed CPUs of one
    last-level-cache domain (a CCD on EPYC), one logical CPU per physical core
    (no SMT sibling shares a core with another of our threads), preferring a
    domain none of the parent's threads ran on (the bench process and its HIP
    runtime threads). Returns what was done: the CPUs before / after, the LLC
    group and the parent's CPUs."""
    before = sorted(os.sched_getaffinity(0))
    rec = {"allowed_before_count": len(before)}
    try:
        groups = {}
        for c in before:
            llc = open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list").read()
            groups.setdefault(llc.strip(), []).append(c)
        par = _parent_cpus() if avoid_parent else set()
        rec["parent_cpus"] = sorted(par)
        free = {k: v for k, v in groups.items() if not (set(_cpu_list(k)) & par)}
        pool = free if any(len(v) >= 2 for v in free.values()) else groups
        llc, cpus = max(pool.items(), key=lambda kv: (len(kv[1]), -kv[1][0]))
        cores, seen = [], set()
        for c in cpus:
            sib = _cpu_list(open(f"/sys/devices/system/cpu/cpu{c}/topology/"
                                 "thread_siblings_list").read())
            key = min(sib)
            if key not in seen:
                seen.add(key)
                cores.append(c)
        if len(cores) >= 2:
            os.sched_setaffinity(0, cores)
        rec.update(pinned=sorted(os.sched_getaffinity(0)), llc_group=llc,
                   llc_groups=len(groups), physical_cores_in_group=len(cores))
    except (OSError, ValueError) as e:
        rec.update(pinned=None, note=f"not pinned: {e}")
    return rec


def faithful_run(npz, pin=True):
    """The child side of cpu_reference_faithful (tools/cpu_faithful.py --npz):
    pinned to one CCD's physical cores before the oracle starts any thread,
    per-frame latency plus the per-thread stage times (ORB thread, LSD thread,
    the ORB thread's join wait, tracking = the rest of the step)."""
    affinity = pin_one_ccd() if pin else {"pinned": None, "note": "not pinned (--no-pin)"}
    from _pkg import load_oracle
    import orbpl.synth as synth
    d = np.load(npz)
    O = load_oracle()
    O.use_variant("best")
    workload = str(d["workload"])
    wl = WORKLOADS[workload]
    use_map = bool(d["use_map"])
    warmup = int(d["warmup"])
    cam = O.camera(getattr(synth, wl["cam"]))
    mk = O.MapVO if use_map else O.LVO
    st_flag = O.TRACK_STEREO if (use_map and wl["stereo"]) else 0
    vo = mk(O.params(*wl["orb"]), cam, 1, use_lines=wl["lines"],
            flags=O.TWO_THREADS | int(d["flags"]) | st_flag)
    if use_map:
        vo.set_fps(wl.get("fps", 30))
    if "voc_parent" in d.files:
        arrays = {k[4:]: (d[k].item() if d[k].ndim == 0 else d[k]) for k in d.files
                  if k.startswith("voc_")}
        vo.set_vocabulary(O.Vocabulary(arrays=arrays))
    vo.reset(d["Tcw0"])
    gray, depth, order = d["gray"], d["depth"], d["order"]
    lat, stages = [], []
    for i, k in enumerate(order):
        t0 = time.perf_counter()
        if wl["stereo"]:
            vo.step_stereo(0, gray[k], depth[k])
        else:
            vo.step(0, gray[k], depth[k])
        if i >= warmup:
            lat.append(time.perf_counter() - t0)
            if use_map:
                stages.append(vo.stage_times())
    lat = np.array(lat) * 1e3
    out = {"value": round(1e3 / float(lat.mean()), 2), "unit": "frames/s",
           "threads_per_frame": 2 if wl["lines"] else 1,
           "median_ms_per_frame": round(float(np.median(lat)), 3),
           "mean_ms_per_frame": round(float(lat.mean()), 3), "frames": int(len(lat)),
           "p10_p90_ms": [round(float(np.percentile(lat, 10)), 3),
                          round(float(np.percentile(lat, 90)), 3)],
           "affinity": affinity,
           "sample": f"one stream, {len(lat)} frames after {warmup} warm-up frames, "
                     f"in a process of its own"}
    if stages:
        st = {k: np.array([x[k] for x in stages]) for k in stages[0]}
        st["tracking"] = st["step"] - st["orb"] - st["join_wait"]
        out["stage_median_ms"] = {k: round(float(np.median(v)), 3) for k, v in st.items()}
        out["stage_note"] = ("orb = ORB extraction on the tracking thread; lines = LineExtractor "
                             "on its own thread (Frame.cc:152-155); join_wait = the tracking "
                             "thread's wait for it; tracking = step - orb - join_wait")
    return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, default=2048,
                    help="streams (frames per step) per GPU; the sweep reports 1..1024 with the "
                         "per-step latency (12.6 ms at 2048: each stream still runs at ~79 Hz, "
                         "above a TUM camera's 30 Hz; 1024: 155.7k, 2048: 162.2k, 3072: 163.1k "
                         "frames/s, profiles/r06/ab/streams_ab.txt)")
    ap.add_argument("--loop", type=int, default=300,
                    help="frames in the headline workload's synthetic closed loop (each stream "
                         "starts at its own frame and walks along it)")
    ap.add_argument("--loop-other", type=int, default=32,
                    help="frames in the other single-camera legs' loops")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host's usable cores")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-ref-frames", type=int, default=300,
                    help="timed frames of the reference-faithful one-stream CPU run (BASELINE.md "
                         "§2: >= 300 after 20 warm-up)")
    ap.add_argument("--cpu-ref-warmup", type=int, default=20)
    ap.add_argument("--workload", choices=tuple(WORKLOADS), default="points",
                    help="points = configs[1] (headline); lines = configs[2] ORB + LSD/LBD; "
                         "kitti = configs[3] stereo points+lines; rig = configs[4] 1280x720 rig")
    ap.add_argument("--rig-loop", type=int, default=12,
                    help="rig frames in the synthetic loop (x8 camera renders)")
    ap.add_argument("--secondary-steps", type=int, default=5,
                    help="steps of the configs[2] lines workload reported under 'secondary' "
                         "(points runs only; 0 = skip)")
    ap.add_argument("--lines-streams", type=int, default=4096,
                    help="streams of the lines workload: the LSD seed loop is one wave per "
                         "frame, latency-bound, so it needs many frames in flight (round 6, "
                         "after the one-wave LDS sort: 3072 17.6-18.3k, 4096 18.3-18.7k, "
                         "5120 19.5k frames/s, profiles/r06/ab/streams_ab.txt)")
    ap.add_argument("--stereo-steps", type=int, default=5,
                    help="steps of the configs[3] stereo workload reported under 'stereo' "
                         "(points runs only; 0 = skip)")
    ap.add_argument("--stereo-streams", type=int, default=3072,
                    help="stereo pairs per GPU: the leg is bound by the two images' LSD "
                         "chains (before the round-6 LDS sort: 1024: 6.03k, 1536: 6.67k, "
                         "2048: 6.75-6.80k, 2560: 6.74k; after it: 2048: 7.35-7.50k, 3072: "
                         "7.65-7.72k frames/s, profiles/r06/ab/streams_ab.txt)")
    ap.add_argument("--rig-steps", type=int, default=5,
                    help="steps of the configs[4] 8-camera rig workload reported under 'rig' "
                         "(points runs only; 0 = skip)")
    ap.add_argument("--rig-streams", type=int, default=512, help="rig cameras per GPU (x8)")
    ap.add_argument("--isolated-steps", type=int, default=5,
                    help="untimed non-pipelined steps after the timed region: per-kernel "
                         "times without the other stream's interference (roofline.isolated)")
    ap.add_argument("--pipelined", type=int, default=-1,
                    help="1 = overlap extraction of step t+1 with tracking of step t; 0 = no; "
                         "-1 = per workload (on, except for the LSD-bound line workloads)")
    ap.add_argument("--sweep", type=int, default=1,
                    help="1 = per-step latency / fps at batch 1..2048 (points) and 1..256 "
                         "(lines) after the timed runs (points runs, rank 0 only)")
    ap.add_argument("--local-map", type=int, default=1,
                    help="1 = every step runs TrackWithMotionModel + TrackLocalMap (the "
                         "reference's per-frame Track, Tracking.cc:1332-1420; local map = the "
                         "last 4 frames, DESIGN.md P18); 0 = TrackWithMotionModel only")
    ap.add_argument("--map", type=int, default=1,
                    help="1 = Tracking::Track with the reference's map model (ORBPL_TRACK_MAP: "
                         "UpdateLastFrame, covisibility local map, NeedNewKeyFrame, "
                         "CreateNewKeyFrame; RGB-D workloads; the stereo leg keeps P18); "
                         "0 = the P18 per-frame local map (--local-map)")
    ap.add_argument("--fixed-line-jacobian", type=int, default=0,
                    help="1 = the analytic line-edge Jacobian instead of the reference's "
                         "as-written one (pinned P7)")
    ap.add_argument("--bow", type=int, default=1,
                    help="1 = every frame's KeyFrame::ComputeBoW with a shared synthetic "
                         "vocabulary (broadcast + IDF all-reduce over ranks); 0 = off")
    ap.add_argument("--vocab-levels", type=int, default=6,
                    help="vocabulary depth L (k = 10; 6 = ORBvoc's shape: with levelsup 4 the "
                         "FeatureVector nodes SearchByBoW walks sit at level 2)")
    ap.add_argument("--trk-load", type=int, default=1,
                    help="1 = after the timed region, time single steps in which 10 %% / 100 %% "
                         "of the streams run TrackReferenceKeyFrame (headline, map model)")
    ap.add_argument("--refkf", type=int, default=1,
                    help="1 = Tracking::Track's TrackReferenceKeyFrame for the first tracked "
                         "frame and motion-model failures (needs --bow; DESIGN.md P22)")
    ap.add_argument("--ingress-steps", type=int, default=20,
                    help="steps of the host-memory ingress leg (u8 gray + u16 depth copied "
                         "host-to-device inside the timed region; points runs only; 0 = skip)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the oracle replay of the timed trackers' sampled streams")
    ap.add_argument("--detail", default="gpurun_out/bench_detail.json",
                    help="side file for the full report (stage times, sweeps, LSD floors, "
                         "per-kernel GB/s); stdout's last line is the compact record")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started before anything here touches the GPU
        sys.exit(subprocess.call(torchrun_cmd(args.gpus, sys.argv[1:], _free_port())))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch  # noqa: F401
        import torch.distributed as dist
        dist.init_process_group("gloo")

    from _pkg import load_oracle, load_pkg
    pkg = load_pkg()
    import orbpl.synth as synth
    O = load_oracle()
    oracle_build = O.use_variant("best")   # -O3 -march build for the CPU legs
    ndev = pkg.device_count()
    device = local_rank % max(1, ndev)

    voc, voc_info = build_vocabulary(pkg, synth, args, rank, world, device, dist) if args.bow \
        else (None, None)
    res = run_workload(pkg, synth, args, args.workload, args.streams, args.steps, args.warmup,
                       rank, world, device, dist, voc)
    res["nsteps"] = args.steps
    # other BASELINE configs, same clock discipline, fewer steps (points runs only)
    others = {}
    if args.workload == "points" and args.secondary_steps > 0:
        others["secondary"] = run_workload(pkg, synth, args, "lines", args.lines_streams,
                                           args.secondary_steps, max(1, args.warmup // 2), rank,
                                           world, device, dist, voc)
        others["secondary"]["nsteps"] = args.secondary_steps
    if args.workload == "points" and args.stereo_steps > 0:
        others["stereo"] = run_workload(pkg, synth, args, "kitti", args.stereo_streams,
                                        args.stereo_steps, max(1, args.warmup // 2), rank, world,
                                        device, dist, voc)
        others["stereo"]["nsteps"] = args.stereo_steps
    if args.workload == "points" and args.rig_steps > 0:
        others["rig"] = run_workload(pkg, synth, args, "rig", args.rig_streams, args.rig_steps,
                                     max(1, args.warmup // 2), rank, world, device, dist, voc)
        others["rig"]["nsteps"] = args.rig_steps

    ingress = None
    if args.workload == "points" and args.ingress_steps > 0:
        ingress = run_ingress(pkg, synth, args, args.streams, args.ingress_steps,
                              args.warmup, rank, world, device, dist, voc,
                              loop=(res["gray"], res["depth"]))
    # parity of every timed tracker's sampled streams against the oracle
    for r in [res] + list(others.values()) + ([ingress] if ingress else []):
        if args.no_parity:
            r["parity"] = None
            continue
        r["parity"] = gather_parity(dist, world, parity_check(
            [h[0] for h in r["hist"]], [h[1] for h in r["hist"]], r["samp"], r["gray"], r["depth"],
            r["layout"], r["wname"], oracle_flags(O, args), r.get("map", False)))

    sweeps = None
    if rank == 0 and world == 1 and args.sweep and args.workload == "points":
        lmf = bool(args.local_map)
        rk = bool(args.refkf)
        mp = bool(args.map)
        sweeps = {"points": sweep(pkg, synth, "points", (1, 16, 64, 256, 1024, 2048), 5, device, lmf,
                                  voc, rk, mp),
                  "lines": sweep(pkg, synth, "lines", (1, 16, 64, 256), 2, device, lmf, voc, rk,
                                 mp)}

    cpu = None
    host = host_info()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        thr = args.cpu_threads or host["usable_cores"]
        ofl = oracle_flags(O, args)
        fps, nfr, dt = cpu_baseline(args.cpu_seconds, thr, res["gray"], res["depth"],
                                    res["layout"], args.workload, ofl, res["map"])
        cpu = {"value": round(fps, 2), "unit": "frames/s", "cores": thr, "kind": "port",
               "sample": f"{nfr} frames of the same {res['image']} loop in {dt:.1f} s, oracle/ "
                         f"C++ restatement ({args.workload} workload), one stream per thread",
               "build": f"oracle/_build ({oracle_build}: -O3 -march=x86-64-{oracle_build})"
                        if oracle_build != "O2" else "oracle/_build (-O2)",
               "host": host,
               "reference_faithful": cpu_reference_faithful(res["gray"], res["depth"],
                                                            res["layout"], args.workload, ofl,
                                                            args.cpu_ref_warmup,
                                                            args.cpu_ref_frames, res["map"])}

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
                       "frames_per_step": S * world, "parallelism": f"streams sharded x{world}",
                       "pipelined": res["pipelined"],
                       "track_map": res["map"],
                       "track_local_map": bool(args.local_map) or res["map"],
                       "fixed_line_jacobian": bool(args.fixed_line_jacobian),
                       "keyframe_bow": bool(args.bow),
                       "track_reference_keyframe": bool(args.bow and args.refkf)},
            "vocabulary": voc_info,
            "stage_ms": res["stages"],
            "tracking": res["tracking"],
            "roofline": res["roof"],
            "parity": res["parity"],
            "cpu_baseline": cpu,
        }
        if res.get("trk_load"):
            out["trk_load"] = res["trk_load"]
        if sweeps:
            out["sweep"] = sweeps
        if ingress:
            out["ingress"] = {
                "workload": "the headline workload from page-locked host memory: u8 gray + "
                            "16-bit depth (DepthMapFactor 5000) copied host-to-device on a copy "
                            "stream overlapped with the kernels, depth converted on the device; "
                            "copies inside the timed region",
                "value": round(ingress["value"], 2), "unit": "frames/s",
                "streams_per_gpu": ingress["S"], "steps": ingress["nsteps"],
                "ms_per_step": round(ingress["elapsed"] / ingress["nsteps"] * 1e3, 3),
                "h2d_bytes_per_step": ingress["bytes_per_step"],
                "h2d_GBps_per_gpu": ingress["h2d_GBps"], "parity": ingress["parity"]}
        for key, o in others.items():
            out[key] = {
                "workload": o["workload"], "value": round(o["value"], 2),
                "unit": "frames/s", "image": o["image"], "nfeatures": o["nfeatures"],
                "steps": o["nsteps"], "streams_per_gpu": o["S"],
                "ms_per_step": round(o["elapsed"] / o["nsteps"] * 1e3, 3),
                "stage_ms": o["stages"], "tracking": o["tracking"], "roofline": o["roof"],
                "parity": o["parity"], "data": o["data"], "track_map": o["map"]}
            if cpu is not None:
                thr = cpu["cores"]
                fps, nfr, dt = cpu_baseline(args.cpu_seconds / 2, thr, o["gray"], o["depth"],
                                            o["layout"], o["wname"], ofl, o["map"])
                out[key]["cpu_baseline"] = {
                    "value": round(fps, 2), "unit": "frames/s", "cores": thr, "kind": "port",
                    "sample": f"{nfr} frames in {dt:.1f} s, oracle/ C++ restatement "
                              f"({o['wname']} workload), one stream per thread",
                    "reference_faithful": cpu_reference_faithful(
                        o["gray"], o["depth"], o["layout"], o["wname"], ofl, args.cpu_ref_warmup,
                        args.cpu_ref_frames, o["map"])}
                if key == "secondary":
                    out[key]["dropin_frame"] = dropin_frame_latency(o["gray"], o["depth"],
                                                                    o["layout"], o["wname"])
        out["summary"] = leg_summary(out)
        detail = Path(args.detail)
        if not detail.is_absolute():
            detail = ROOT / detail
        detail.parent.mkdir(parents=True, exist_ok=True)
        detail.write_text(json.dumps(out) + "\n")
        line = json.dumps(compact_line(out, str(detail.relative_to(ROOT))
                                       if detail.is_relative_to(ROOT) else str(detail)))
        print(line, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
