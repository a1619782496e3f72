#!/bin/bash
# Synth fp32 A/B of library variants with the serial phase split (diag / panel / updates)
#   bash tools/synth_ab2.sh V1 V2 ...   (multi_fidelity_gpflow_amd/variants/libmfgp_<V>.so)
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    MFGP_LIB_PATH=multi_fidelity_gpflow_amd/variants/libmfgp_$v.so timeout -k 10 200 \
      python bench.py --config synth --steps 6 --warmup 2 --no-cpu-baseline --no-train-predict \
      > gpurun_out/syab_$v.json 2> gpurun_out/syab_$v.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/syab_$v.json')); r=d['roofline']; p=r['phase_ms']; print('$v', d['ms_per_step'], round(r['frac'],4), {k: round(x, 3) for k, x in p.items()})"
  done
done
