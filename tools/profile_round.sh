#!/bin/bash
# Round profile recipe (run on the GPU box from the repo root).  Usage:
#   bash tools/profile_round.sh OUTDIR CONFIG "BENCH ARGS" "SHORT BENCH ARGS" ["TRACE ARGS"]
# 1. the bench JSON line;  2. rocprofv3 --kernel-trace --stats of the same command;
# 3./4. HBM traffic FETCH_SIZE / WRITE_SIZE, 5. MFMA counters -- each in a separate --pmc pass of
# the short command (MI355X_MICROARCH.md: counters in their own runs, no trace domains with --pmc).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r02}
CFG=${2:-goku}
ARGS=${3:-}
SHORT=${4:-"--steps 20 --warmup 5 --no-cpu-baseline --no-train-predict"}
TRACE=${5:-$ARGS}
mkdir -p "$OUT"
timeout -k 10 400 python3 bench.py --config "$CFG" $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --config "$CFG" $TRACE > "$OUT/bench_under_rocprof.json" 2> "$OUT/trace.err"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --config "$CFG" $SHORT > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py --config "$CFG" $SHORT > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_mfma" -o run -- \
    python3 bench.py --config "$CFG" $SHORT > "$OUT/pmc_mfma.json" 2> "$OUT/pmc_mfma.err"
