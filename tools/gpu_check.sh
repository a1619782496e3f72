#!/bin/bash
# Quick GPU check (run on the GPU box from the repo root): parity tests (optionally a -k
# filter as $1) then one short bench line.
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
