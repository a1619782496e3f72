# Round 5, GPU pass B: the in-flow Gram as a prologue phase (182 VGPRs), the fixed two-process
# SVGP test, an interleaved Goku A/B against the round-4 cleanup build, the SVGP GEMM A/B, and a
# kernel-trace profile of the Goku line.
set -o pipefail
mkdir -p gpurun_out/r05c
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_multiprocess.py tests/test_gpu_svgp.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05c/tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -4 gpurun_out/r05c/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "goku or flow or lbfgs or large or synthetic" > gpurun_out/r05c/parity.log 2>&1
rc=$?; echo "PARITY rc=$rc"; tail -3 gpurun_out/r05c/parity.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > gpurun_out/r05c/ab_new_$i.json 2>/dev/null || exit 3
  MFGP_LIB_PATH=$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_base.so timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > gpurun_out/r05c/ab_base_$i.json 2>/dev/null || exit 3
  python -c "import json; a=json.load(open('gpurun_out/r05c/ab_new_$i.json')); b=json.load(open('gpurun_out/r05c/ab_base_$i.json')); print('AB new', a['value'], a['roofline']['phase_ms'], ' base', b['value'], b['roofline']['phase_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05c/trace -o run -- python3 bench.py --no-extras --no-cpu-baseline --no-train-predict --steps 100 > gpurun_out/r05c/bench_under_rocprof.json 2> gpurun_out/r05c/trace.err
echo "PROF rc=$?"; find gpurun_out/r05c/trace -name "*kernel_stats.csv" | head -2
