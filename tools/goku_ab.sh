#!/bin/bash
# Goku headline A/B of library builds (GPU box, repo root): interleaved default-line timings
#   bash tools/goku_ab.sh ROUNDS LIB1 LIB2 ...   (paths of libmfgp.so builds, MFGP_LIB_PATH)
set -o pipefail
R=$1; shift
for round in $(seq 1 "$R"); do
  for v in "$@"; do
    MFGP_LIB_PATH=$v timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict \
      > /tmp/gab.json 2>/tmp/gab.err || exit 3
    python -c "import json; d=json.loads(open('/tmp/gab.json').read().splitlines()[-1]); print('$v', d['value'], 'evals/s', d['ms_per_step'], 'ms', 'grad phase', d['roofline']['phase_ms']['grad'])"
  done
done
