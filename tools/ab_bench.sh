#!/bin/bash
# A/B of library variants (run on the GPU box from the repo root):
#   bash tools/ab_bench.sh S1 S4 ...   (multi_fidelity_gpflow_amd/variants/libmfgp_<name>.so)
# Interleaved rounds, one bench line per variant per round (evals/s and the flow launch time).
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    MFGP_LIB_PATH=multi_fidelity_gpflow_amd/variants/libmfgp_$v.so timeout -k 10 120 \
      python bench.py --no-cpu-baseline --no-train-predict > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['value'],1), d['roofline']['avg_launch_us'], d['roofline']['phase_ms'])"
  done
done
