"""Per-kernel SQ counter table from one rocprofv3 --pmc counter_collection.csv
(tools/prof.sh SQ=1 pass): VALU totals, share, LDS, waves, wave cycles,
wait fraction and VALU instructions per wave cycle.

usage: python tools/sq_table.py <counter_collection.csv> [out.txt] [header line ...]
"""
import collections
import csv
import sys


def table(path, top=14):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbpl::", "").split("<")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = sum(c["SQ_INSTS_VALU"] for c in acc.values()) or 1.0
    out = ["%-24s %9s %6s %9s %9s %10s %8s %8s" % ("kernel", "VALU", "share", "LDS", "waves",
                                                  "wave_cyc", "wait_any", "valu/cyc")]
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU"])[:top]:
        wc = c["SQ_WAVE_CYCLES"] or 1.0
        out.append("%-24s %9.3g %5.1f%% %9.3g %9.3g %10.3g %7.1f%% %8.3f" % (
            k[:24], c["SQ_INSTS_VALU"], 100 * c["SQ_INSTS_VALU"] / tot, c["SQ_INSTS_LDS"],
            c["SQ_WAVES"], wc, 100 * c["SQ_WAIT_ANY"] / wc, c["SQ_INSTS_VALU"] / wc))
    return out


if __name__ == "__main__":
    lines = sys.argv[3:] + table(sys.argv[1])
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))
