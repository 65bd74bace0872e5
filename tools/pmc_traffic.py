"""Summarise a tools/prof.sh run into per-kernel HBM traffic per launch.

Reads gpurun_out/prof_<tag>/{trace,fetch,write}/ (rocprofv3 csv) and writes
profiles/<round>/pmc_traffic.json:
  {kernel: {"launches", "avg_ns", "fetch_bytes", "write_bytes", "traffic_bytes"}}
per launch, averaged over the launches of the profiled bench command (per
extraction step for k_pyramid / k_fast_cells / k_octree / k_orient_desc,
which the level pipeline launches once per group of levels: "group_launches"
per step).
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half
the bytes of wide coalesced reads, so fetch_bytes = 2 * FETCH_SIZE; WRITE_SIZE
is taken as is. Both counters are in KiB.

usage: python tools/pmc_traffic.py <tag> <round> [streams] [workload] [orb_frames,lsd_frames]
(workload: points -> pmc_traffic_points.json, lines, kitti, ...; the last
argument: frames per launch of the extraction / LSD kernels when the tracker
split those batches in two halves, stored per kernel as "frames_per_launch")
"""
import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("orbpl::", "")
    n = n.split("<")[0]
    # the paired variant of the orientation / descriptor kernel is the same stage
    return "k_orient_desc" if n == "k_orient_desc2" else n


ORB_KERNELS = ("k_pyramid", "k_fast_cells", "k_octree", "k_orient_desc")
LSD_KERNELS = ("k_lsd_prep", "k_lsd_sort", "k_lsd_sort_local", "k_lsd_sort_wave", "k_lsd_fill",
               "k_lsd_spec", "k_lsd_validate",
               "k_lsd_compact", "k_keylines", "k_blur_sobel", "k_lbd")


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    base = ROOT / "gpurun_out" / f"prof_{tag}"
    out = {}
    # per kernel, its launches in dispatch order: (duration, grid threads)
    launches = collections.defaultdict(list)
    rows = sorted(csv.DictReader(open(base / "trace" / "run_kernel_trace.csv")),
                  key=lambda r: int(r["Dispatch_Id"]))
    # the bench workload's window: from the tracker's reset (k_map_reset, the
    # map model every bench leg runs) on; the vocabulary training's one-frame
    # extractions before it are left out
    starts = [int(r["Dispatch_Id"]) for r in rows if short(r["Kernel_Name"]) == "k_map_reset"]
    d0 = starts[0] if starts else None
    if d0 is None:
        print("pmc_traffic: WARNING no k_map_reset launch: keeping launches with grids "
              ">= 1/10 of the kernel's largest", file=sys.stderr)
    for r in rows:
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        launches[short(r["Kernel_Name"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), grid, int(r["Dispatch_Id"])))
    cnt = {}
    for part in ("fetch", "write"):
        vals = collections.defaultdict(list)
        for r in sorted(csv.DictReader(open(base / part / "run_counter_collection.csv")),
                        key=lambda r: int(r["Dispatch_Id"])):
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        cnt[part] = vals
    for k, v in launches.items():
        if "rocclr" in k:
            continue
        # the bench workload's launches only: the runs dispatch the same
        # sequence, so the i-th launch of a kernel is the same in every pass
        if d0 is not None:
            keep = [i for i, (_, _, di) in enumerate(v) if di >= d0]
        else:
            gmax = max(g for _, g, _ in v)
            keep = [i for i, (_, g, _) in enumerate(v) if g >= gmax // 10]
        if not keep:
            continue
        f = cnt["fetch"].get(k, [])
        w = cnt["write"].get(k, [])
        if len(f) == len(v):
            f = [f[i] for i in keep]
        if len(w) == len(v):
            w = [w[i] for i in keep]
        d = [v[i][0] for i in keep]
        fb = 2.0 * 1024.0 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        out[k] = {"launches": len(d), "avg_ns": sum(d) / len(d),
                  "fetch_bytes": fb, "write_bytes": wb,
                  "traffic_bytes": (fb + wb) if fb is not None and wb is not None else None}
    # the ORB level pipeline launches k_pyramid, k_fast_cells, k_octree and
    # k_orient_desc once per group of levels: their entries are per step (the
    # sum over a step's group launches, "group_launches" of them)
    # (k_frame_prepare runs once per step; the octree and orientation are
    # group-launched too since round 5)
    steps = out.get("k_frame_prepare", {}).get("launches", 0)
    for k in ("k_pyramid", "k_fast_cells", "k_octree", "k_orient_desc"):
        e = out.get(k)
        if e and steps and e["launches"] > steps and e["launches"] % steps != 0:
            print(f"pmc_traffic: WARNING {k}: {e['launches']} launches is not a multiple of "
                  f"the {steps} steps; left per launch", file=sys.stderr)
        if e and steps and e["launches"] > steps and e["launches"] % steps == 0:
            m = e["launches"] // steps
            e["group_launches"] = m
            e["launches"] = steps
            e["avg_ns"] *= m
            for q in ("fetch_bytes", "write_bytes", "traffic_bytes"):
                if e[q] is not None:
                    e[q] *= m
    wl = sys.argv[4] if len(sys.argv) > 4 else "points"
    streams = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    of, lf = (int(x) for x in sys.argv[5].split(",")) if len(sys.argv) > 5 else (streams, streams)
    for k, e in out.items():
        e["frames_per_launch"] = of if k in ORB_KERNELS else lf if k in LSD_KERNELS else streams
    out["_meta"] = {"streams": streams, "workload": wl,
                    "source": f"gpurun_out/prof_{tag}", "correction": "fetch x2 (gfx950)"}
    dst = ROOT / "profiles" / rnd / f"pmc_traffic_{wl}.json"
    dst.parent.mkdir(parents=True, exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    for k in sorted((k for k in out if k != "_meta"),
                    key=lambda k: -out[k]["avg_ns"] * out[k]["launches"])[:14]:
        e = out[k]
        tb = e["traffic_bytes"]
        print(f"{k:28s} n={e['launches']:3d} avg {e['avg_ns'] / 1e3:9.1f} us  traffic "
              f"{(tb or 0) / 1e6:9.2f} MB/launch")


if __name__ == "__main__":
    main()
