# Round 5: parity subset + Goku A/B (tools/gpu_r5_c.sh without the two-process line) + chain timeline
set -o pipefail
O=gpurun_out/${OUT:-r05f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -4 $O/tests.log
[ $rc -eq 0 ] || exit 5
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > $O/ab_new_$i.json 2>/dev/null || exit 5
  MFGP_LIB_PATH=$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_base.so timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > $O/ab_base_$i.json 2>/dev/null || exit 5
  python -c "import json; a=json.load(open('$O/ab_new_$i.json')); b=json.load(open('$O/ab_base_$i.json')); print('AB new', a['value'], a['roofline']['phase_ms'], ' base', b['value'], b['roofline']['phase_ms'])"
done
timeout -k 10 120 python tools/flow_trace.py 5 > $O/trace_new.txt 2>&1; echo "trace rc=$?"; head -12 $O/trace_new.txt
