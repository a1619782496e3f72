#!/bin/bash
# k_gram_flow variant A/B (GPU box, repo root): timeline of each variant, then interleaved bench lines
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  MFGP_LIB_PATH=multi_fidelity_gpflow_amd/variants/libmfgp_$v.so timeout -k 10 60 python tools/gram_trace.py 3 2>&1 | grep -v amdgpu.ids | tail -4 || exit $?
done
bash tools/ab_bench.sh "$@"
