# Round 4 profiles (rocprofv3 stats + FETCH / WRITE / MFMA passes) and the re-run of the fixed tests.
set -o pipefail
timeout -k 10 900 bash tools/profile_all.sh r04 > gpurun_out/r04_prof.log 2>&1; rc=$?; echo "PROF rc=$rc"; tail -3 gpurun_out/r04_prof.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_svgp.py -v -s --timeout 300 --timeout-method thread -k "trajectory or goku_singlebin_grad" > gpurun_out/r04/retest.log 2>&1; echo "RETEST rc=$?"; grep -E "Synth 100|rel err|passed|failed" gpurun_out/r04/retest.log
