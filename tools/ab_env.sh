#!/bin/bash
# A/B of an environment knob on the Goku bench line (run on the GPU box from the repo root):
#   bash tools/ab_env.sh VAR "v1 v2 ..."   -> interleaved rounds, evals/s and the flow launch time
set -o pipefail
mkdir -p gpurun_out
var=$1; shift
for round in 1 2 3; do
  for v in $1; do
    env "$var=$v" timeout -k 10 120 python bench.py --no-cpu-baseline --no-train-predict --no-extras \
      > gpurun_out/abe_$v.json 2> gpurun_out/abe_$v.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/abe_$v.json')); print('$var=$v', round(d['value'],1), d['roofline']['avg_launch_us'], d['roofline']['phase_ms'])"
  done
done
