"""Summarise a rocprofv3 counter CSV per (kernel, grid): median serialised duration and SQ counters
per dispatch (tools/pmc_kernel_ab.sh)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tag = sys.argv[2] if len(sys.argv) > 2 else ""
dur = collections.defaultdict(dict)
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = (r["Kernel_Name"].split("(")[0][-28:], r["Grid_Size"])
    dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(dur):
    v = sorted(dur[k].values())
    c = {n.replace("SQ_", ""): sum(x) / len(x) for n, x in cnt[k].items()}
    wc = c.get("WAVE_CYCLES", 1.0)
    print(f"{tag:10s} {k[0]:28s} grid {k[1]:>8s} n {len(v):3d} median {v[len(v) // 2]:8.1f} us  "
          f"wait {c.get('WAIT_ANY', 0) / wc:.2f} stall {c.get('WAIT_INST_ANY', 0) / wc:.2f} "
          f"active {c.get('ACTIVE_INST_ANY', 0) / wc:.2f} valu_insts {c.get('INSTS_VALU', 0):.3g} "
          f"mfma_busy {c.get('VALU_MFMA_BUSY_CYCLES', 0):.3g}")
