"""Timeline of one iteration from a rocprofv3 kernel trace (diagnostic): kernels between the k-th and
(k+1)-th dispatch of a marker kernel, with queue, start / end relative to the marker (us), and the
idle gaps of the busiest queue.
  python tools/trace_timeline.py TRACE.csv MARKER_SUBSTRING [k]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mark = sys.argv[2]
k = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
i0, i1 = starts[k], starts[k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
span = (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3
print(f"iteration {k}: {span:.1f} us between consecutive '{mark}' dispatches")
for r in rows[i0:i1]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    name = r["Kernel_Name"].replace("void mfgp::", "").replace("mfgp::", "")
    name = name.split("(")[0] + ("(" + r["Grid_Size_X"] + "x" + r["Grid_Size_Z"] + ")")
    print(f"  q{r['Queue_Id']:>2} {s:8.1f} {e:8.1f} {e - s:7.1f}  {name[:70]}")
