"""Per-dispatch mean durations by (kernel, grid) from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    g = (r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"])
    d[(n, g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v) / len(v) / 1000:9.1f} us x{len(v):3d}  {k}")
