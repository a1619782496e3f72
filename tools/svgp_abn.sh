#!/bin/bash
# Goku SVGP A/B over library variants, interleaved (GPU box, repo root):
#   bash tools/svgp_abn.sh V1 V2 ...   (multi_fidelity_gpflow_amd/variants/libmfgp_<V>.so)
set -o pipefail
mkdir -p gpurun_out/svabn
A="--config goku_svgp --steps 50 --warmup 10 --no-train-predict --no-latent --no-cpu-baseline"
for round in 1 2 3; do
  line=""
  for v in "$@"; do
    MFGP_LIB_PATH=$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_$v.so timeout -k 10 200 python bench.py $A \
      > gpurun_out/svabn/$v.json 2> gpurun_out/svabn/$v.err || exit 5
    line="$line $v $(python -c "import json; print(json.load(open('gpurun_out/svabn/$v.json'))['ms_per_step'])")"
  done
  echo "AB$line"
done
