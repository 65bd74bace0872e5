"""Per-kernel sums of the counters in gpurun_out/pmc_<tag>/counters.csv (dev tool)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
want = sys.argv[2].split(",") if len(sys.argv) > 2 else None
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    if want and not any(w in k for w in want):
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, c in acc.items():
    n = len(disp[k])
    print(k, f"dispatches={n}", " ".join(f"{a}={v / n:.4g}" for a, v in sorted(c.items())))
