#!/bin/bash
# k_grad / k_grad_w ablations (tools/grad_variants.py variants): gradient phase time per variant
set -o pipefail
mkdir -p gpurun_out
for w in 0 10; do
  for v in cur noepi nomfma; do
    MFGP_GRAD_WIDE=$w MFGP_LIB_PATH=multi_fidelity_gpflow_amd/variants/libmfgp_$v.so timeout -k 10 120 \
      python tools/phase_times.py 50 > gpurun_out/abl_${w}_$v.txt 2>&1 || exit $?
    echo "wide=$w $v $(tail -1 gpurun_out/abl_${w}_$v.txt)"
  done
done
