# GPU A/B for the SVGP path: tests/test_gpu_svgp.py, then the single-bin Goku SVGP line interleaved,
# the in-tree libmfgp.so against $VARIANT, $N rounds.
set -o pipefail
O=gpurun_out/${OUT:-svab}
mkdir -p $O
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_svgp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -4 $O/tests.log
  [ $rc -eq 0 ] || exit 5
fi
A="--config goku_svgp --steps 50 --warmup 10 --no-train-predict --no-latent --no-cpu-baseline"
for i in $(seq 1 ${N:-2}); do
  timeout -k 10 200 python bench.py $A > $O/ab_new_$i.json 2>/dev/null || exit 5
  MFGP_LIB_PATH=$PWD/$VARIANT timeout -k 10 200 python bench.py $A > $O/ab_var_$i.json 2>/dev/null || exit 5
  python -c "import json; a=json.load(open('$O/ab_new_$i.json')); b=json.load(open('$O/ab_var_$i.json')); print('AB new', a['ms_per_step'], ' var', b['ms_per_step'])"
done
