#!/bin/bash
# Round profile recipe (run on the GPU box from the repo root):
#   1. the bench JSON line;  2. rocprofv3 kernel-trace --stats of the same command;
#   3./4. HBM traffic counters FETCH_SIZE / WRITE_SIZE in separate passes (short run).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r01}
mkdir -p "$OUT"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py > "$OUT/bench_under_rocprof.json" 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train-predict > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train-predict > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
