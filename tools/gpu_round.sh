set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK && bash tools/profile_round.sh gpurun_out/r01b && echo PROF_OK
