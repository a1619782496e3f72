set -o pipefail
mkdir -p gpurun_out/r4oh
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4oh/parity.log 2>&1 && echo PARITY_OK && tail -1 gpurun_out/r4oh/parity.log && \
timeout -k 10 700 bash tools/ab_bench.sh oh1 oh0 > gpurun_out/r4oh/ab.txt 2>&1 && echo AB_OK && cat gpurun_out/r4oh/ab.txt
