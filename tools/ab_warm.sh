#!/bin/bash
# Goku line at the driver's --steps 20: capture-first order on / off and the warm-up length
set -o pipefail
O=${1:-gpurun_out/r06g}; mkdir -p $O
for r in 1 2 3; do for cfg in "1 5" "0 5" "1 30"; do set -- $cfg
  MFGP_BENCH_CAPTURE_FIRST=$1 timeout -k 10 120 python bench.py --steps 20 --warmup $2 --no-cpu-baseline --no-train-predict --no-extras > $O/w_$1_$2_$r.json 2> $O/w_$1_$2_$r.err || exit 4
  python -c "import json; d=json.load(open('$O/w_$1_$2_$r.json')); print('capture_first=$1 warmup=$2', d['value'], d['ms_per_step'])"
done; done
