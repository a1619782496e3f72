# SVGP re-associated reverse pass: parity tests, bench leg; then the pending flow A/B batch.
# Continues past a failing test (rc 1) only; any other status (fault, abort, time limit) ends the script.
set -o pipefail
mkdir -p gpurun_out/r4svgp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_svgp.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r4svgp/svgp_tests.log 2>&1
rc=$?; echo "SVGP_TESTS rc=$rc"; grep -E "rel err|passed|failed|Error" gpurun_out/r4svgp/svgp_tests.log | tail -20
ok $rc || exit $rc
timeout -k 10 300 python -u bench.py --config goku_svgp --steps 100 --warmup 10 --no-train-predict > gpurun_out/r4svgp/bench_svgp.json 2> gpurun_out/r4svgp/bench_svgp.err
rc=$?; echo "BENCH_SVGP rc=$rc"; cat gpurun_out/r4svgp/bench_svgp.json
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4_ab3.sh
