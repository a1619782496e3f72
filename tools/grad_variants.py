"""Experiment: k_grad variants (compile-time switches) timed by the LML phase times.

  python tools/grad_variants.py build        # here: hipcc each variant -> tools/variants/
  python tools/grad_variants.py run          # GPU box: phase times per variant (Goku)
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "multi_fidelity_gpflow_amd", "variants")   # travels to the GPU box
VARIANTS = {
    "cur": [],
    "noepi": ["-DGRAD_ABL=1"],
    "nomfma": ["-DGRAD_ABL=2"],
}


def build():
    from multi_fidelity_gpflow_amd.build import build_lib, SOURCES
    os.makedirs(VDIR, exist_ok=True)
    if os.environ.get("GV_REF"):   # also build the committed sources at this git ref
        ref = os.environ["GV_REF"]
        src = os.path.join(VDIR, "ref", "csrc")   # csrc includes ../../include/mfgp.h
        os.makedirs(src, exist_ok=True)
        os.makedirs(os.path.join(VDIR, "include"), exist_ok=True)
        files = [(f"multi_fidelity_gpflow_amd/csrc/{f}", os.path.join(src, f))
                 for f in SOURCES + ["mfgp_device.h", "mfgp_internal.h"]]
        files.append(("include/mfgp.h", os.path.join(VDIR, "include", "mfgp.h")))
        for gpath, dst in files:
            with open(dst, "w") as fh:
                fh.write(subprocess.run(["git", "-C", ROOT, "show", f"{ref}:{gpath}"],
                                        capture_output=True, text=True, check=True).stdout)
        build_lib(force=True, out=os.path.join(VDIR, "libmfgp_ref.so"), csrc=src)
        print("built ref", ref)
    for name, flags in VARIANTS.items():
        build_lib(force=True, extra_flags=flags, out=os.path.join(VDIR, f"libmfgp_{name}.so"))
        print("built", name)


def load_goku_xy(bench):
    arrs = bench.load_goku()
    return arrs[0], arrs[1]


def one(name, chunk):
    import numpy as np
    import torch
    os.environ["MFGP_GRAD_CHUNK"] = str(chunk)
    from multi_fidelity_gpflow_amd import _lib
    _lib.load(os.path.join(VDIR, f"libmfgp_{name}.so"))
    import bench
    from multi_fidelity_gpflow_amd.engine import gpr_phase_times
    X, Y = load_goku_xy(bench)
    model = bench.make_model(X, Y)
    eng, X, Y = model._device_data()
    theta = torch.tensor(model._theta_map().theta(), dtype=torch.float64, device=eng.device)
    for _ in range(3):
        gpr_phase_times(eng, X, Y, theta)
    ms = np.mean([gpr_phase_times(eng, X, Y, theta) for _ in range(20)], axis=0)
    print(json.dumps({"variant": name, "chunk": chunk, "grad_us": round(ms[3] * 1e3, 2),
                      "chol_us": round(ms[2] * 1e3, 2)}))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    elif sys.argv[1] == "one":
        one(sys.argv[2], int(sys.argv[3]))
    else:
        chunks = [int(c) for c in (sys.argv[2:] or ["16"])]
        names = (["ref"] if os.path.exists(os.path.join(VDIR, "libmfgp_ref.so")) else []) + list(VARIANTS)
        for name in names:
            for c in chunks:
                subprocess.run([sys.executable, __file__, "one", name, str(c)], check=True, timeout=300)
