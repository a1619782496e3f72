"""Build A/B variants of libmfgp.so in parallel (CPU, in this container):
    python tools/build_variants.py name=-DFLAG[,-DFLAG2] ...
-> multi_fidelity_gpflow_amd/variants/libmfgp_<name>.so (tools/ab.sh runs them)."""
import concurrent.futures as cf
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multi_fidelity_gpflow_amd.build import build_lib  # noqa: E402

OUT = os.path.join(ROOT, "multi_fidelity_gpflow_amd", "variants")


def one(spec):
    name, _, flags = spec.partition("=")
    return build_lib(force=True, extra_flags=[f for f in flags.split(",") if f],
                     out=os.path.join(OUT, f"libmfgp_{name}.so"))


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    with cf.ProcessPoolExecutor(min(6, len(sys.argv) - 1)) as ex:
        for r in ex.map(one, sys.argv[1:]):
            print(r)
