"""Build libmfgp.so in-tree with hipcc for gfx950 (CDNA4 / MI355X)."""
from __future__ import annotations

import hashlib
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


def source_files(csrc: str = CSRC):
    """Every file the library is compiled from: csrc/* and include/mfgp.h."""
    return sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                  if os.path.isfile(os.path.join(csrc, f))) + [os.path.join(ROOT, "include", "mfgp.h")]


def source_hash(csrc: str = CSRC) -> str:
    """Content hash of the library's sources (names and bytes; 16 hex digits).  Compiled into the
    library (mfgp_build_id), so a test can tell whether the .so it loaded was built from the
    sources checked out beside it."""
    h = hashlib.sha256()
    for p in source_files(csrc):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def built_id(path: str = OUT):
    """The build id marker inside a built library file, read without loading it (None if absent)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(b"mfgp-build-id:")
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + 14:j].decode(errors="replace")


def needs_rebuild() -> bool:
    return built_id(OUT) != source_hash()


def build_lib(force: bool = False, extra_flags=None, out: str = OUT, csrc: str = CSRC) -> str:
    """Compile every source to an object in parallel (they are separate translation units in any
    case), then link the shared library."""
    if not force and out == OUT and not needs_rebuild():
        return out
    from concurrent.futures import ThreadPoolExecutor
    out = os.path.abspath(out)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include"),
             "-Wno-unused-result", '-DMFGP_BUILD_ID="%s"' % source_hash(csrc)] + list(extra_flags or [])
    objdir = out + ".objs"
    os.makedirs(objdir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        r = subprocess.run([hipcc()] + flags + ["-c", os.path.join(csrc, src), "-o", obj], cwd=csrc,
                           capture_output=True, text=True)
        return obj, r

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1, 8)) as ex:
        results = list(ex.map(compile_one, SOURCES))
    for _, r in results:
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("hipcc build of libmfgp.so failed")
    r = subprocess.run([hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC"] + [o for o, _ in results] + ["-o", out],
                       capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc link of libmfgp.so failed")
    for o, _ in results:
        os.remove(o)
    os.rmdir(objdir)
    return out


if __name__ == "__main__":
    print(build_lib(force="--force" in sys.argv))
