# goku_svgp profile with single-model PMC passes (traffic per iteration) + the default bench line.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 bash tools/profile_round.sh gpurun_out/r04/goku_svgp goku_svgp "--steps 50 --warmup 20" \
    "--steps 10 --warmup 10 --no-train-predict --no-latent" "--steps 50 --warmup 20 --no-train-predict --no-cpu-baseline" > gpurun_out/r04_svgpprof.log 2>&1; echo "PROF rc=$?"
