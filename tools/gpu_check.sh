#!/bin/bash
# One GPU call: the -m gpu suite, then a default bench line (each step time-limited; stop at the
# first failure).  Usage: bash tools/gpu_check.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K \
    > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK \
&& timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err \
&& echo BENCH_OK && cat gpurun_out/bench_default.json
