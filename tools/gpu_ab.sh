# GPU A/B: the parity suite (api surface + parity), then the Goku line interleaved, the in-tree
# libmfgp.so against $VARIANT (a build under multi_fidelity_gpflow_amd/variants/), $N rounds.
# Usage: OUT=<dir under gpurun_out> VARIANT=<lib> [N=2] [TESTS=0] bash tools/gpu_ab.sh
set -o pipefail
O=gpurun_out/${OUT:-ab}
mkdir -p $O
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -4 $O/tests.log
  [ $rc -eq 0 ] || exit 5
fi
for i in $(seq 1 ${N:-2}); do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > $O/ab_new_$i.json 2>/dev/null || exit 5
  MFGP_LIB_PATH=$PWD/$VARIANT timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > $O/ab_var_$i.json 2>/dev/null || exit 5
  python -c "import json; a=json.load(open('$O/ab_new_$i.json')); b=json.load(open('$O/ab_var_$i.json')); print('AB new', a['value'], a['roofline']['phase_ms'], ' var', b['value'], b['roofline']['phase_ms'])"
done
