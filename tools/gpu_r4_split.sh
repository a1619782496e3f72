set -o pipefail
mkdir -p gpurun_out/r4split
timeout -k 10 60 ./tools/ubench_graph_probe > gpurun_out/r4split/graph_probe.txt 2>&1 && echo GP_OK && cat gpurun_out/r4split/graph_probe.txt && \
timeout -k 10 60 ./tools/ubench_rsplit > gpurun_out/r4split/ubench.txt 2>&1 && echo UB_OK && cat gpurun_out/r4split/ubench.txt && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4split/parity.log 2>&1 && echo PARITY_OK && tail -3 gpurun_out/r4split/parity.log && \
timeout -k 10 400 bash tools/ab_bench.sh base r1 r2 r3 r1p0 > gpurun_out/r4split/ab.txt 2>&1 && echo AB_OK && cat gpurun_out/r4split/ab.txt && \
timeout -k 10 120 python tools/flow_trace.py 5 > gpurun_out/r4split/trace_r1.txt 2>&1 && echo TRACE_OK && \
timeout -k 10 120 python tools/tp_breakdown.py hbs > gpurun_out/r4split/tp_hbs.txt 2>&1 && echo TP_OK && cat gpurun_out/r4split/tp_hbs.txt && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_svgp.py -x -q --timeout 120 --timeout-method thread -k shared_inducing > gpurun_out/r4split/svgp_shared.log 2>&1 && echo SVGP_SHARED_OK
