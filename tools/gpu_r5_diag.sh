#!/bin/bash
# Round 5: k32_diag in one 79 KB buffer -- fp32 parity tests, then Synth A/B against the 157 KB kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/diag_f32.log 2>&1 || { tail -30 gpurun_out/diag_f32.log; exit 1; }
tail -3 gpurun_out/diag_f32.log
bash tools/synth_ab.sh prediag diag79
