#!/bin/bash
# --config goku_svgp with the latent L = 15 model, in-tree library vs variants
set -o pipefail
mkdir -p gpurun_out/svlat
for v in "$@"; do
  if [ "$v" = tree ]; then L=""; else L="MFGP_LIB_PATH=$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_$v.so"; fi
  env $L timeout -k 10 300 python bench.py --config goku_svgp --steps 50 --warmup 10 --no-train-predict --no-cpu-baseline > gpurun_out/svlat/$v.json 2> gpurun_out/svlat/$v.err || exit 5
  python -c "import json; d=json.load(open('gpurun_out/svlat/$v.json')); print('$v', d['ms_per_step'], 'l15', d['latent_l15']['ms_per_step'])"
done
