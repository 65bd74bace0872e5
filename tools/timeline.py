"""Per-stream kernel timeline of a rocprofv3 kernel_trace.csv: the last N
dispatches in start order with start / end (ms from the first shown), duration,
queue and grid; used to see how the pipelined tracker's two streams overlap."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 120
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if not r["Kernel_Name"].startswith("__amd")][-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    name = r["Kernel_Name"].split("(")[0].replace("orbpl::", "").replace("void ", "")
    print(f"q{r['Queue_Id']:>2} {s:9.3f} {e:9.3f} {e - s:8.3f}  {name[:34]:34s} grid {r['Grid_Size_X']}x{r['Grid_Size_Y']} wg {r['Workgroup_Size_X']} vgpr {r['VGPR_Count']}+{r['Accum_VGPR_Count']} lds {r['LDS_Block_Size']}")
