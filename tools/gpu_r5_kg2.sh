# Round 5: kernel trace + one SQ pass of the SVGP step with the MFMA-distance k_kgrad.
set -o pipefail
O=gpurun_out/${OUT:-r05t}
mkdir -p $O
export TMPDIR=/tmp
ARGS="--config goku_svgp --steps 20 --warmup 5 --no-train-predict --no-latent --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py $ARGS > $O/kt.json 2> $O/kt.err || exit 5
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_kgrad" --output-format csv -d $O/p1 -o run -- python3 bench.py --config goku_svgp --steps 4 --warmup 2 --no-train-predict --no-latent --no-cpu-baseline > $O/p1.json 2> $O/p1.err || exit 6
echo DONE
