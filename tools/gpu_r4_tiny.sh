# One-launch small-problem LML path: parity (all schedules), smoke, HBS bench leg.
set -o pipefail
mkdir -p gpurun_out/r4tiny
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r4tiny/parity.log 2>&1
rc=$?; echo "PARITY rc=$rc"; grep -E "tiny vs|L-BFGS Forrester|hbs \{|goku \{|passed|failed|FAILED" gpurun_out/r4tiny/parity.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4tiny/smoke.log 2>&1; echo "SMOKE rc=$?"; tail -1 gpurun_out/r4tiny/smoke.log
timeout -k 10 300 python tools/tp_breakdown.py hbs > gpurun_out/r4tiny/hbs_breakdown.txt 2>&1; echo "HBS rc=$?"; cat gpurun_out/r4tiny/hbs_breakdown.txt | tail -5
