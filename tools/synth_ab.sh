#!/bin/bash
# Synth fp32 A/B of library variants (GPU box, repo root): interleaved bench lines
#   bash tools/synth_ab.sh V1 V2 ...   (multi_fidelity_gpflow_amd/variants/libmfgp_<V>.so)
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    MFGP_LIB_PATH=multi_fidelity_gpflow_amd/variants/libmfgp_$v.so timeout -k 10 200 \
      python bench.py --config synth --steps 6 --warmup 2 --no-cpu-baseline \
      > gpurun_out/syab_$v.json 2> gpurun_out/syab_$v.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/syab_$v.json')); r=d['roofline']; print('$v', d['ms_per_step'], round(r['frac'],4), r['phase_ms'].get('update_out'), r['phase_ms'].get('grad'))"
  done
done
