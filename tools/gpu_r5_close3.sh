# Round 5 closing pass 2 (after the SVGP stream / Psi / pipelining changes): the GPU suite, smoke, the default bench line, the two-process (gloo,
# shared device) lines of goku and goku_svgp, and the k_gpr_tiny poison run.
set -o pipefail
O=gpurun_out/r05close3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit 6
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 7
head -c 400 $O/bench_default.json; echo
for cfg in goku goku_svgp; do
  MFGP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --config $cfg --no-cpu-baseline > $O/dist2_$cfg.out 2> $O/dist2_$cfg.err || exit 8
  grep '^{' $O/dist2_$cfg.out > $O/dist2_$cfg.json || exit 9
  echo "DIST2 $cfg ok"
done
MFGP_LIB_PATH=$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_poison.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "tiny or (test_lml_and_grad and nb32-tiny) or (test_predict_f and nb32-tiny) or test_lbfgs_forrester_kat" \
  tests/test_gpu_parity.py > $O/tiny_poison.log 2>&1
echo "POISON rc=$?"; tail -1 $O/tiny_poison.log
