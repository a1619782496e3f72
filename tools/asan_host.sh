#!/usr/bin/env bash
# Host AddressSanitizer build of libmfgp.so (SURVEY §5 "Race detection / sanitizers"),
# run over the CPU tests that drive the library's host side: argument validation, workspace layout
# (gpr_layout / pred_layout / the fp32 and SVGP carves), handle settings and the flow fence.
# GPU code is compiled as usual (-fsanitize only after -Xarch_host: GPU ASan is not available on
# this pool); no GPU is needed.  Python is not instrumented, so the ASan runtime is preloaded.
# Usage (repo root, build container):  tools/asan_host.sh [extra pytest args]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT="$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_asan.so"
mkdir -p "$(dirname "$OUT")"
python - <<EOF
from multi_fidelity_gpflow_amd.build import build_lib
build_lib(force=True, out="$OUT",
          extra_flags=["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer",
                       "-shared-libsan", "-g"])
EOF
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
mkdir -p gpurun_out
LOG=gpurun_out/asan_host.log
# detect_leaks=0: CPython's own allocations are not instrumented and report as leaks at exit
MFGP_LIB_PATH="$OUT" LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
    python -m pytest tests/test_capi.py tests/test_asan_host.py -q -p no:cacheprovider "$@" 2>&1 | tee "$LOG"
echo "ASan runtime: $RT" | tee -a "$LOG"
