# Round 4: full GPU suite, smoke, default bench line.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04/gpu_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r04/gpu_tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r04/smoke.log 2>&1; echo "SMOKE rc=$?"; tail -2 gpurun_out/r04/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r04/bench_default.json 2> gpurun_out/r04/bench_default.err; echo "BENCH rc=$?"; cat gpurun_out/r04/bench_default.json
