#!/bin/bash
# Default bench line (Goku + hbs / synth / goku_svgp sub-objects) for the in-tree library and variants
#   bash tools/gpu_r5_defab.sh V1 V2 ...   ("tree" = the in-tree libmfgp.so)
set -o pipefail
mkdir -p gpurun_out/defab
for v in "$@"; do
  if [ "$v" = tree ]; then L=""; else L="MFGP_LIB_PATH=$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_$v.so"; fi
  env $L timeout -k 10 400 python bench.py > gpurun_out/defab/$v.json 2> gpurun_out/defab/$v.err || exit 5
  python -c "import json; d=json.load(open('gpurun_out/defab/$v.json')); s=d['goku_svgp']; print('$v', d['value'], 'svgp', s['ms_per_step'], 'l15', s['latent_l15']['ms_per_step'], 'synth', d['synth']['ms_per_step'])"
done
