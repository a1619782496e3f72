#!/usr/bin/env python
"""Summarise one round's rocprofv3 output (tools/profile_round.sh) into profiles/<round>/.

Writes kernel_stats.csv (copy of the --kernel-trace --stats summary) and
pmc_summary.json: per kernel, the mean FETCH_SIZE / WRITE_SIZE per dispatch from
the two separate --pmc passes, in bytes, with the gfx950 correction of
MI355X_MICROARCH.md ("HBM [CDNA4]"): FETCH_SIZE (KiB, from TCC_EA0_RDREQ x 64 B)
reports half the bytes of wide coalesced reads -> x2; WRITE_SIZE is taken as is.
"""
import csv
import json
import os
import shutil
import sys


def per_kernel(path):
    agg = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            agg.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    for f in ("bench.json", "bench_under_rocprof.json"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    fetch = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    out = {"units": "bytes per dispatch (mean over dispatches)",
           "correction": "fetch_bytes = 2 x FETCH_SIZE[KiB] x 1024 (gfx950 wide-read halving); "
                         "write_bytes = WRITE_SIZE[KiB] x 1024",
           "command": "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate passes) -- "
                      "python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train-predict",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(("void mfgp::", "mfgp::")):
            continue
        fk, nf = fetch.get(k, (0.0, 0))
        wk, nw = write.get(k, (0.0, 0))
        out["kernels"][k] = {"dispatches": max(nf, nw), "fetch_size_kib_raw": round(fk, 3),
                             "fetch_bytes": round(2 * fk * 1024), "write_bytes": round(wk * 1024),
                             "hbm_bytes": round(2 * fk * 1024 + wk * 1024)}
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
