# Round 5: kernel-trace summaries of the Goku and Goku-SVGP lines (no counters).
set -o pipefail
O=gpurun_out/${OUT:-r05p}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/goku -o run -- python3 bench.py --no-extras --no-cpu-baseline --no-train-predict --steps 100 > $O/goku_bench.json 2> $O/goku.err || exit 5
echo GOKU_DONE
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/svgp -o run -- python3 bench.py --config goku_svgp --steps 50 --warmup 20 --no-train-predict --no-latent --no-cpu-baseline > $O/svgp_bench.json 2> $O/svgp.err || exit 5
echo SVGP_DONE
find $O -name "*kernel_stats.csv"
