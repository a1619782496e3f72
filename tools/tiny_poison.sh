#!/usr/bin/env bash
# k_gpr_tiny LDS-hazard check (VERDICT r4 #1b).  `build` (build container): libmfgp.so with
# -DTINY_POISON=1, where every LDS slot reuse of k_gpr_tiny is preceded by overwriting the dead
# slots with a signalling NaN between two extra barriers (mfgp_kernels.hip TINY_REUSE): a read not
# ordered before the reuse by the barrier named there sees NaN and the parity tests fail.
# `run` (GPU box): the small-problem parity tests against that build.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT="$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_poison.so"
case "${1:-run}" in
  build)
    mkdir -p "$(dirname "$OUT")"
    python -c "from multi_fidelity_gpflow_amd.build import build_lib; build_lib(force=True, out='$OUT', extra_flags=['-DTINY_POISON=1'])"
    ;;
  run)
    mkdir -p gpurun_out
    MFGP_LIB_PATH="$OUT" timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
      -k "tiny or (test_lml_and_grad and nb32-tiny) or (test_predict_f and nb32-tiny) or test_lbfgs_forrester_kat" \
      tests/test_gpu_parity.py 2>&1 | tee gpurun_out/tiny_poison.log
    ;;
esac
