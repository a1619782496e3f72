#!/bin/bash
# Round-3 probes (GPU box, repo root): dependent-latency micro-benchmarks for the chain floor,
# the k_chol_flow timeline at Goku, and the Goku SingleBinSVGP KAT with its printed errors.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench_latency > gpurun_out/lat1.txt \
&& timeout -k 10 60 ./tools/ubench_lat2 > gpurun_out/lat2.txt \
&& timeout -k 10 60 ./tools/ubench_lat3 > gpurun_out/lat3.txt \
&& timeout -k 10 120 python -u tools/flow_trace.py 5 > gpurun_out/flow_trace.txt 2>&1 \
&& timeout -k 10 300 python -u -m pytest tests/test_gpu_svgp.py -k goku_singlebin_training_kat -s -x \
     --timeout 240 --timeout-method thread > gpurun_out/kat.log 2>&1
echo rc=$?
