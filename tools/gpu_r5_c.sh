# Round 5, GPU pass C: band tiles of rows <= 3 published by idle worker waves (FT_G), tile (0,0)
# split over diag waves 0/1; parity subset, interleaved Goku A/B against the round-4 build, the
# two-process SVGP bench line.
set -o pipefail
O=gpurun_out/${OUT:-r05d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -4 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > $O/ab_new_$i.json 2>/dev/null || exit 5
  MFGP_LIB_PATH=$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_base.so timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > $O/ab_base_$i.json 2>/dev/null || exit 5
  python -c "import json; a=json.load(open('$O/ab_new_$i.json')); b=json.load(open('$O/ab_base_$i.json')); print('AB new', a['value'], a['roofline']['phase_ms'], ' base', b['value'], b['roofline']['phase_ms'])"
done
MFGP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config goku_svgp --no-cpu-baseline > $O/dist2_goku_svgp.json 2> $O/dist2_goku_svgp.err
echo "DIST2 rc=$?"; cat $O/dist2_goku_svgp.json
