#!/bin/bash
# SVGP A/B of library builds (GPU box, repo root): interleaved single-bin SVGP iteration times
#   bash tools/svgp_ab.sh ROUNDS LIB1 LIB2 ...   (paths of libmfgp.so builds, MFGP_LIB_PATH)
set -o pipefail
R=$1; shift
for round in $(seq 1 "$R"); do
  for v in "$@"; do
    MFGP_LIB_PATH=$v timeout -k 10 200 python tools/bench_svgp.py --which single --iters 40 > /tmp/svab.json 2>/tmp/svab.err || exit 3
    python -c "import json; d=json.loads(open('/tmp/svab.json').read().splitlines()[-1]); print('$v', round(d['s_per_iter']*1e3, 4), 'ms')"
  done
done
