# Round 5: SQ counters of the SVGP k_kgrad launches (two passes of 8 SQ counters each).
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
ARGS="--config goku_svgp --steps 4 --warmup 2 --no-train-predict --no-latent --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "k_kgrad|k_bgemm2|k_svgp_cond2" --output-format csv -d $O/p1 -o run -- python3 bench.py $ARGS > $O/p1.json 2> $O/p1.err || exit 5
echo P1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "k_kgrad|k_bgemm2|k_svgp_cond2" --output-format csv -d $O/p2 -o run -- python3 bench.py $ARGS > $O/p2.json 2> $O/p2.err || exit 6
echo P2
find $O -name "*counter_collection.csv"
