#!/bin/bash
# k_gram_flow ablations (diagnostic; results are wrong under them): 1 no entry stores, 2 no exp,
# 4 no sentinel fill, 8 no Y copy.  GPU box, repo root.
set -o pipefail
for e in 0 1 2 4 8 15; do
  echo "== MFGP_GRAM_EXPERIMENT=$e"
  MFGP_GRAM_EXPERIMENT=$e timeout -k 10 60 python tools/gram_trace.py 3 2>&1 | grep -v amdgpu.ids | tail -4 || exit $?
done
