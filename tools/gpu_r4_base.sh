set -o pipefail
mkdir -p gpurun_out/r4base
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4base/gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python -u bench.py > gpurun_out/r4base/bench.json 2> gpurun_out/r4base/bench.err && echo BENCH_OK && cat gpurun_out/r4base/bench.json
