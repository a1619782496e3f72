#!/bin/bash
# A/B of library variants on the Goku SVGP bench leg (run on the GPU box from the repo root):
#   bash tools/ab_svgp.sh V1 V2 ...   (multi_fidelity_gpflow_amd/variants/libmfgp_<name>.so)
# Interleaved rounds, one line per variant per round: single-bin and latent ms per iteration.
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    MFGP_LIB_PATH=multi_fidelity_gpflow_amd/variants/libmfgp_$v.so timeout -k 10 180 \
      python bench.py --config goku_svgp --steps 40 --warmup 10 --no-train-predict \
      > gpurun_out/abs_$v.json 2> gpurun_out/abs_$v.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/abs_$v.json')); print('$v', d['ms_per_step'], d['latent_l15']['ms_per_step'])"
  done
done
