# Kernel traces of the Goku SVGP step for the in-tree library and $VARIANT (per-kernel diff).
set -o pipefail
O=gpurun_out/${OUT:-svprof}
mkdir -p $O
export TMPDIR=/tmp
ARGS="--config goku_svgp --steps 20 --warmup 5 --no-train-predict --no-latent --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o run -- python3 bench.py $ARGS > $O/new.json 2> $O/new.err || exit 5
MFGP_LIB_PATH=$PWD/$VARIANT timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/var -o run -- python3 bench.py $ARGS > $O/var.json 2> $O/var.err || exit 6
echo DONE
