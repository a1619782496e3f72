set -o pipefail
mkdir -p gpurun_out/r4split2
V=multi_fidelity_gpflow_amd/variants
timeout -k 10 60 ./tools/ubench_rsplit > gpurun_out/r4split2/ubench.txt 2>&1 && echo UB_OK && cat gpurun_out/r4split2/ubench.txt && \
MFGP_LIB_PATH=$V/libmfgp_r2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4split2/parity_r2.log 2>&1 && echo PARITY_R2_OK && tail -1 gpurun_out/r4split2/parity_r2.log && \
MFGP_LIB_PATH=$V/libmfgp_s2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4split2/parity_s2.log 2>&1 && echo PARITY_S2_OK && tail -1 gpurun_out/r4split2/parity_s2.log && \
MFGP_LIB_PATH=$V/libmfgp_r2b3s2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4split2/parity_r2b3s2.log 2>&1 && echo PARITY_R2B3S2_OK && tail -1 gpurun_out/r4split2/parity_r2b3s2.log && \
timeout -k 10 700 bash tools/ab_bench.sh base b3 r2 r2b3 r3b3 s2 s3 r2b3s2 > gpurun_out/r4split2/ab.txt 2>&1 && echo AB_OK && cat gpurun_out/r4split2/ab.txt && \
MFGP_LIB_PATH=$V/libmfgp_r2b3.so timeout -k 10 120 python tools/flow_trace.py 5 > gpurun_out/r4split2/trace_r2b3.txt 2>&1 && echo TRACE_OK && \
timeout -k 10 120 python tools/tp_breakdown.py hbs > gpurun_out/r4split2/tp_hbs.txt 2>&1 && echo TP_OK && cat gpurun_out/r4split2/tp_hbs.txt && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_svgp.py tests/test_gpu_api_surface.py -x -q --timeout 120 --timeout-method thread -k "shared_inducing or pool" > gpurun_out/r4split2/new_tests.log 2>&1 && echo NEWTESTS_OK && tail -2 gpurun_out/r4split2/new_tests.log
