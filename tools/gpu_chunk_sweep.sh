# k_grad m-chunk sweep on the Goku line (MFGP_GRAD_CHUNK), interleaved.
set -o pipefail
O=gpurun_out/${OUT:-chunk}
mkdir -p $O
for i in 1 2; do
  for c in 18 24 30; do
    MFGP_GRAD_CHUNK=$c timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-train-predict > $O/c${c}_$i.json 2>/dev/null || exit 5
    python -c "import json; a=json.load(open('$O/c${c}_$i.json')); print('chunk $c', a['value'], a['roofline']['phase_ms']['grad'])"
  done
done
