# Round 5, first GPU pass: full GPU suite (flow with the Gram inside, resident sessions), the
# tiny-kernel poison run, the default bench line, an interleaved A/B against the round-4 cleanup
# build (variants/libmfgp_base.so), the two-rank (gloo, shared GPU) bench lines.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05/gpu_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r05/gpu_tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/tiny_poison.sh run > /dev/null 2>&1; prc=$?; echo "POISON rc=$prc"; tail -3 gpurun_out/tiny_poison.log
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > gpurun_out/r05/ab_new_$i.json 2>/dev/null || exit 3
  MFGP_LIB_PATH=$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_base.so timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > gpurun_out/r05/ab_base_$i.json 2>/dev/null || exit 3
  python -c "import json; a=json.load(open('gpurun_out/r05/ab_new_$i.json')); b=json.load(open('gpurun_out/r05/ab_base_$i.json')); print('AB new', a['value'], a['roofline']['phase_ms'], ' base', b['value'], b['roofline']['phase_ms'])"
done
timeout -k 10 400 python bench.py > gpurun_out/r05/bench_default.json 2> gpurun_out/r05/bench_default.err; echo "BENCH rc=$?"; head -c 600 gpurun_out/r05/bench_default.json; echo
MFGP_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r05/dist2_goku.json 2> gpurun_out/r05/dist2_goku.err; echo "DIST2 goku rc=$?"; head -c 400 gpurun_out/r05/dist2_goku.json; echo
MFGP_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config goku_svgp --steps 20 --warmup 5 --no-train-predict > gpurun_out/r05/dist2_svgp.json 2> gpurun_out/r05/dist2_svgp.err; echo "DIST2 svgp rc=$?"; head -c 400 gpurun_out/r05/dist2_svgp.json; echo
for i in 1 2; do
  MFGP_BGEMM2=1 timeout -k 10 300 python tools/bench_svgp.py --which single > gpurun_out/r05/svgp_bg2_$i.txt 2>&1 || exit 3
  MFGP_BGEMM2=0 timeout -k 10 300 python tools/bench_svgp.py --which single > gpurun_out/r05/svgp_bg1_$i.txt 2>&1 || exit 3
  echo "SVGP bgemm2:"; tail -2 gpurun_out/r05/svgp_bg2_$i.txt; echo "SVGP bgemm1:"; tail -2 gpurun_out/r05/svgp_bg1_$i.txt
done
