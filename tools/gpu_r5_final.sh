#!/bin/bash
# Round 5 final pass: the SVGP profile (the only config whose kernels changed since profile_all r05b),
# then closing pass 3's checks (GPU suite, smoke, default line, two-process lines, tiny poison run)
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh gpurun_out/r05d/goku_svgp goku_svgp "--steps 50 --warmup 20" \
    "--steps 10 --warmup 10 --no-train-predict --no-latent" "--steps 50 --warmup 20 --no-train-predict --no-cpu-baseline" || exit 4
echo SVGP_PROFILE_DONE
sed -e 's#gpurun_out/r05close3#gpurun_out/r05final2#' tools/gpu_r5_close3.sh > /tmp/close_final.sh
bash /tmp/close_final.sh
