#!/bin/bash
# Isolated (counter-collection, serialised) kernel durations + SQ cycles of library builds (GPU box):
#   bash tools/pmc_kernel_ab.sh OUTDIR REGEX LIB1 LIB2 ...   (single-bin Goku SVGP, 10 iterations)
set -o pipefail
export TMPDIR=/tmp
O=$(realpath -m "$1"); RX=$2; shift 2
mkdir -p "$O"
for v in "$@"; do
  n=$(basename "$v" .so)
  ( cd /tmp && MFGP_LIB_PATH=$v timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
      --kernel-include-regex "$RX" --output-format csv -d "$O/$n" -o run -- \
      python "$GRAFT_REPO_ROOT/tools/bench_svgp.py" --which single --iters 10 > "$O/$n.log" 2>&1 ) || exit 3
  python "$GRAFT_REPO_ROOT/tools/pmc_summary_ab.py" "$O/$n/run_counter_collection.csv" "$n"
done
