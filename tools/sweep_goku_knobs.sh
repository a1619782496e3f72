#!/bin/bash
# Goku step knob sweep (GPU box, repo root): k_gram workgroups and the k_grad m-chunk.
#   bash tools/sweep_goku_knobs.sh
set -o pipefail
mkdir -p gpurun_out
run() {   # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-train-predict > gpurun_out/sw_$name.json 2> gpurun_out/sw_$name.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/sw_$name.json')); print('$name', round(d['value'],1), d['roofline']['phase_ms'])"
}
for round in 1 2; do
  run gw0 MFGP_GRAM_WGS=0
  run gw384 MFGP_GRAM_WGS=384
  run gw512 MFGP_GRAM_WGS=512
  run gwtile MFGP_GRAM_WGS=-1
done
run gc16 MFGP_GRAD_CHUNK=16
run gc32 MFGP_GRAD_CHUNK=32
run gc24 MFGP_GRAD_CHUNK=24
