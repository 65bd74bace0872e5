"""Summarise the FETCH_SIZE calibration run (tools/calib/fetch_calib.hip).

usage: python tools/calib/fetch_calib.py <rocprofv3 counter_collection.csv> <out.json>
Every measured kernel reads a known byte count from HBM (1 GiB; k_sparse16:
one 16-B piece of each of the 2^23 lines). Reports FETCH_SIZE (KiB x 1024) /
known bytes per kernel: the factor to divide a counter reading by, per access
shape.
"""
import collections
import csv
import json
import sys

KNOWN = {"k_stream16": 1 << 30, "k_gather<16>": 1 << 30, "k_gather<8>": 1 << 30,
         "k_gather<4>": 1 << 30, "k_sparse16": (1 << 30) // 128 * 16}
SHAPE = {"k_stream16": "coalesced 16 B/lane stream",
         "k_gather<16>": "16 B/lane gather, 8 lanes per 128-B line, 8 scattered lines per wave",
         "k_gather<8>": "8 B/lane gather, 16 lanes per line, 4 scattered lines per wave",
         "k_gather<4>": "4 B/lane gather, 32 lanes per line, 2 scattered lines per wave",
         "k_sparse16": "16 B/lane, one piece per line, 64 scattered lines per wave"}


def short(n):
    return n.split("(")[0].replace("void ", "").strip()


def main():
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    out = {}
    for k, known in KNOWN.items():
        if k not in vals:
            continue
        v = sorted(vals[k])
        med = v[len(v) // 2]
        out[k] = {"shape": SHAPE[k], "known_bytes": known, "fetch_size_bytes_median": med,
                  "counter_over_known": round(med / known, 4), "runs": len(v)}
        if k == "k_sparse16":
            out[k]["counter_bytes_per_request"] = round(med / (known // 16), 2)
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    for k, e in out.items():
        print(f"{k:14s} counter/known {e['counter_over_known']:.3f}  ({e['shape']})")


if __name__ == "__main__":
    main()
