"""Build libmfgp.so in-tree with hipcc for gfx950 (CDNA4 / MI355X)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
SOURCES = ["mfgp_kernels.hip", "mfgp_flow.hip", "mfgp_capi.hip", "mfgp_svgp.hip", "mfgp_svgp_grad.hip", "mfgp_f32.hip"]
OUT = os.path.join(HERE, "libmfgp.so")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def needs_rebuild() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(ROOT, "include", "mfgp.h")]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build_lib(force: bool = False, extra_flags=None, out: str = OUT, csrc: str = CSRC) -> str:
    if not force and out == OUT and not needs_rebuild():
        return out
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + os.path.join(ROOT, "include"), "-Wno-unused-result"]
    cmd += list(extra_flags or [])
    cmd += [os.path.join(csrc, s) for s in SOURCES] + ["-o", out]
    r = subprocess.run(cmd, cwd=csrc, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc build of libmfgp.so failed")
    return out


if __name__ == "__main__":
    print(build_lib(force="--force" in sys.argv))
