#!/bin/bash
# Kernel trace of the default bench line (in-tree library): where the SVGP sub-object's time goes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/deftr
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/deftr/tree -o run -- python3 bench.py \
  > gpurun_out/deftr/tree.json 2> gpurun_out/deftr/tree.err || exit 5
echo DONE
