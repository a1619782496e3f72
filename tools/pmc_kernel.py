"""PMC counters of one LML value+grad evaluation's kernels (Goku), one rocprofv3 pass
per counter group.  On the GPU box, from the repo root:

  python tools/pmc_kernel.py run gpurun_out/pmc     # rocprofv3 passes
  python tools/pmc_kernel.py sum gpurun_out/pmc     # per-kernel averages (JSON)
  python tools/pmc_kernel.py work                    # the profiled workload itself
"""
import csv
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GROUPS = [
    ["SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"],
    ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CU_CYCLES", "SQ_INSTS_VALU_MFMA_F64"],
    ["SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"],
    ["TCC_HIT_sum", "TCC_MISS_sum"],
    ["SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"],
    ["SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA",
     "SQ_IFETCH", "SQ_INST_CYCLES_VMEM_WR", "SQ_ACTIVE_INST_ANY"],
    ["SQ_VMEM_WR_TA_DATA_FIFO_FULL", "SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_VMEM_TA_CMD_FIFO_FULL", "SQ_INSTS_VMEM_WR",
     "SQ_INSTS_SMEM", "SQ_INST_CYCLES_SMEM", "SQ_LDS_DATA_FIFO_FULL", "SQ_LDS_CMD_FIFO_FULL"],
]


def work(reps=30):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import bench
    from multi_fidelity_gpflow_amd.engine import gpr_phase_times
    arrs = bench.load_goku()
    model = bench.make_model(arrs[0], arrs[1])
    eng, X, Y = model._device_data()
    theta = torch.tensor(model._theta_map().theta(), dtype=torch.float64, device=eng.device)
    for _ in range(reps):
        gpr_phase_times(eng, X, Y, theta)
    torch.cuda.synchronize()


def run(out):
    env = dict(os.environ, TMPDIR="/tmp")
    for g, counters in enumerate(GROUPS):
        cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", os.path.join(out, f"g{g}"),
               "-o", "run", "--", sys.executable, os.path.abspath(__file__), "work"]
        r = subprocess.run(cmd, env=env, timeout=300, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stderr[-3000:])
            raise SystemExit(f"pass {g} failed ({r.returncode})")


def summarize(out):
    agg = {}
    for path in glob.glob(os.path.join(out, "g*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "work":
        work()
    elif sys.argv[1] == "run":
        run(sys.argv[2])
        summarize(sys.argv[2])
    else:
        summarize(sys.argv[2])
