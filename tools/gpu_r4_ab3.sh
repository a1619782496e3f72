set -o pipefail
mkdir -p gpurun_out/r4ab3
V=multi_fidelity_gpflow_amd/variants
MFGP_LIB_PATH=$V/libmfgp_w4s5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4ab3/parity_w4s5.log 2>&1 && echo PARITY_W4S5_OK && tail -1 gpurun_out/r4ab3/parity_w4s5.log && \
timeout -k 10 700 bash tools/ab_bench.sh base w4 s2 s5 s8 w4s5 > gpurun_out/r4ab3/ab.txt 2>&1 && echo AB_OK && cat gpurun_out/r4ab3/ab.txt && \
MFGP_LIB_PATH=$V/libmfgp_s5.so timeout -k 10 120 python tools/flow_trace.py 5 > gpurun_out/r4ab3/trace_s5.txt 2>&1 && echo TRACE_OK && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_svgp.py tests/test_gpu_api_surface.py -x -q --timeout 120 --timeout-method thread -k "shared_inducing or pool" > gpurun_out/r4ab3/new_tests.log 2>&1 && echo NEWTESTS_OK && tail -2 gpurun_out/r4ab3/new_tests.log && \
timeout -k 10 120 python tools/flow_trace.py 5 > gpurun_out/r4ab3/trace_base.txt 2>&1 && echo TRACE_BASE_OK
