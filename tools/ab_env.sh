#!/bin/bash
# Interleaved A/B of environment settings on the Goku headline step (GPU box, repo root):
#   bash tools/ab_env.sh OUTDIR ROUNDS "ENV_A" "ENV_B" ...   (ENV: space-separated VAR=value, or "-")
# Each round runs every setting once (bench.py --no-extras, 300 steps); prints ms/step per run.
set -o pipefail
O=${1:?}; R=${2:?}; shift 2
mkdir -p "$O"
for r in $(seq 1 "$R"); do
  k=0
  for e in "$@"; do
    k=$((k + 1))
    envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --no-train-predict \
      > "$O/ab_${k}_$r.json" 2> "$O/ab_${k}_$r.err" || exit 3
    python -c "import json,sys; d=json.load(open('$O/ab_${k}_$r.json')); print('round $r [$e]', d['value'], 'evals/s', d['ms_per_step'], 'ms', 'phases', d['roofline'].get('phase_ms'))"
  done
done
