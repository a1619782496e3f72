#!/bin/bash
# SVGP A/B of library variants (GPU box, repo root): interleaved goku_svgp bench lines
#   bash tools/svgp_ab.sh V1 V2 ...   (multi_fidelity_gpflow_amd/variants/libmfgp_<V>.so)
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    MFGP_LIB_PATH=multi_fidelity_gpflow_amd/variants/libmfgp_$v.so timeout -k 10 200 \
      python bench.py --config goku_svgp --steps 30 --warmup 10 --no-train-predict --no-cpu-baseline \
      > gpurun_out/svab_$v.json 2> gpurun_out/svab_$v.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/svab_$v.json')); print('$v', d['ms_per_step'], d.get('latent_l15', {}).get('ms_per_step'))"
  done
done
