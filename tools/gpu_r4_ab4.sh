# wave-5 variants: parity on the most different one, A/B, traces
set -o pipefail
mkdir -p gpurun_out/r4ab4
V=multi_fidelity_gpflow_amd/variants
MFGP_LIB_PATH=$V/libmfgp_w5ng.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4ab4/parity_w5ng.log 2>&1 && echo PARITY_OK && tail -1 gpurun_out/r4ab4/parity_w5ng.log && \
MFGP_LIB_PATH=$V/libmfgp_w5b3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4ab4/parity_w5b3.log 2>&1 && echo PARITY2_OK && tail -1 gpurun_out/r4ab4/parity_w5b3.log && \
timeout -k 10 700 bash tools/ab_bench.sh base w5own nogate w5b3 w5ng > gpurun_out/r4ab4/ab.txt 2>&1 && echo AB_OK && cat gpurun_out/r4ab4/ab.txt && \
MFGP_LIB_PATH=$V/libmfgp_base.so timeout -k 10 120 python tools/flow_trace.py 5 > gpurun_out/r4ab4/trace_base.txt 2>&1 ; \
MFGP_LIB_PATH=$V/libmfgp_w5ng.so timeout -k 10 120 python tools/flow_trace.py 5 > gpurun_out/r4ab4/trace_w5ng.txt 2>&1 ; \
MFGP_LIB_PATH=$V/libmfgp_w5own.so timeout -k 10 120 python tools/flow_trace.py 5 > gpurun_out/r4ab4/trace_w5own.txt 2>&1 ; echo TRACES_DONE
