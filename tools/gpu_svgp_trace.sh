#!/bin/bash
# Kernel trace of the Goku SVGP step (in-tree library): per-kernel time per iteration
set -o pipefail
O=gpurun_out/${OUT:-svtr}
mkdir -p $O
export TMPDIR=/tmp
ARGS="--config goku_svgp --steps 20 --warmup 5 --no-train-predict --no-latent --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o run -- python3 bench.py $ARGS > $O/new.json 2> $O/new.err || exit 5
echo DONE
