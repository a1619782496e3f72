#!/bin/bash
# One GPU call: the -m gpu suite + a default bench line (tools/gpu_check.sh), then the k_grad
# ablation variants' phase times (tools/grad_variants.py).  Each GPU step is time-limited.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python -u tools/grad_variants.py run 24 > gpurun_out/grad_variants.txt 2>&1 && echo GV_OK && cat gpurun_out/grad_variants.txt
