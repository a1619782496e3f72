#!/usr/bin/env python
"""Summarise one round's rocprofv3 output (tools/profile_round.sh) into profiles/<round>/<config>/.

Writes kernel_stats.csv (copy of the --kernel-trace --stats summary) and
pmc_summary.json: per kernel, the mean FETCH_SIZE / WRITE_SIZE per dispatch from
the two separate --pmc passes, in bytes, with the gfx950 correction of
MI355X_MICROARCH.md ("HBM [CDNA4]"): FETCH_SIZE (KiB, from TCC_EA0_RDREQ x 64 B)
reports half the bytes of wide coalesced reads -> x2; WRITE_SIZE is taken as is.
With the MFMA pass: MFMA flops per dispatch (SQ_INSTS_VALU_MFMA_MOPS_* x 512, the
MfmaFlops definition of rocprofv3 -L), SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES and
GRBM_GUI_ACTIVE (summed over the XCDs by rocprofv3), and the kernel's mean duration
from the trace pass, so mfma_tflops = flops / duration.
"""
import csv
import json
import os
import shutil
import sys


def per_kernel(path, counter=None):
    """{kernel: (mean value per dispatch, dispatches)} (one counter, summed over its rows per dispatch)."""
    per_disp = {}
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if counter and r.get("Counter_Name") != counter:
                continue
            key = (r["Kernel_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            per_disp[key] = per_disp.get(key, 0.0) + float(r["Counter_Value"])
    agg = {}
    for (name, _), v in per_disp.items():
        agg.setdefault(name, []).append(v)
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


def durations(path):
    """{kernel: mean duration ns} from the --stats summary."""
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            out[r["Name"]] = float(r["AverageNs"])
    return out


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    for f in ("bench.json", "bench_under_rocprof.json"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    fetch = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    mf = os.path.join(src, "pmc_mfma", "run_counter_collection.csv")
    mfma = {c: per_kernel(mf, c) for c in ("SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_INSTS_VALU_MFMA_MOPS_F32",
                                           "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")}
    dur = durations(os.path.join(src, "trace", "run_kernel_stats.csv"))
    out = {"units": "bytes per dispatch (mean over dispatches)",
           "correction": "fetch_bytes = 2 x FETCH_SIZE[KiB] x 1024 (gfx950 wide-read halving); "
                         "write_bytes = WRITE_SIZE[KiB] x 1024",
           "command": "tools/profile_round.sh: rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE | --pmc <MFMA counters> "
                      "(separate passes) -- python3 bench.py --config <config> <short args>",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(("void mfgp::", "mfgp::")):
            continue
        fk, nf = fetch.get(k, (0.0, 0))
        wk, nw = write.get(k, (0.0, 0))
        e = {"dispatches": max(nf, nw), "fetch_size_kib_raw": round(fk, 3),
             "fetch_bytes": round(2 * fk * 1024), "write_bytes": round(wk * 1024),
             "hbm_bytes": round(2 * fk * 1024 + wk * 1024)}
        if any(k in v for v in mfma.values()):
            m64 = mfma["SQ_INSTS_VALU_MFMA_MOPS_F64"].get(k, (0.0, 0))[0]
            m32 = mfma["SQ_INSTS_VALU_MFMA_MOPS_F32"].get(k, (0.0, 0))[0]
            e["mfma_flops_f64"] = m64 * 512
            e["mfma_flops_f32"] = m32 * 512
            for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
                e[c] = mfma[c].get(k, (0.0, 0))[0]
            if k in dur and dur[k] > 0:
                e["avg_duration_ns"] = dur[k]
                e["mfma_tflops"] = round((m64 + m32) * 512 / dur[k] / 1e3, 3)
        out["kernels"][k] = e
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
