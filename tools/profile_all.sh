#!/bin/bash
# All configs of a round's profile (GPU box, repo root): Goku (BASELINE metric), Synth fp32, Goku SVGP.
set -e
R=${1:-r03}
bash tools/profile_round.sh gpurun_out/$R/goku goku "--no-extras" "--steps 20 --warmup 5 --no-cpu-baseline --no-train-predict --no-extras"
echo GOKU_DONE
bash tools/profile_round.sh gpurun_out/$R/synth synth "--steps 6 --warmup 2" "--steps 2 --warmup 1"
echo SYNTH_DONE
bash tools/profile_round.sh gpurun_out/$R/goku_svgp goku_svgp "--steps 50 --warmup 20" \
    "--steps 10 --warmup 10 --no-train-predict --no-latent" "--steps 50 --warmup 20 --no-train-predict --no-cpu-baseline"
echo SVGP_DONE
