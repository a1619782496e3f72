#!/bin/bash
# Interleaved A/B on the GPU box (repo root).  One script for every A/B of the rounds (it replaces
# the per-round ab_bench / goku_ab / svgp_ab / ab_svgp / gpu_svgp_ab / synth_ab / ab_env /
# sweep_goku_knobs scripts):
#   bash tools/ab.sh MODE OUTDIR ROUNDS ITEM [ITEM ...]
# MODE picks the workload, ITEM what differs between runs:
#   goku  LIB    Goku headline line (bench.py, 300 replayed steps)   ITEM: a libmfgp.so path
#   svgp  LIB    single-bin Goku SVGP iteration (tools/bench_svgp.py) ITEM: a libmfgp.so path
#   synth LIB    Synth fp32 line (bench.py --config synth)           ITEM: a libmfgp.so path
#   env   ENV    Goku headline line under environment settings      ITEM: "VAR=v VAR2=w" or "-"
# A LIB item may also be a variant name: multi_fidelity_gpflow_amd/variants/libmfgp_<name>.so
# (tools/build_variants.py).  Each round runs every item once; the first failing run ends the script.
set -o pipefail
export TMPDIR=/tmp
MODE=${1:?usage: ab.sh MODE OUTDIR ROUNDS ITEM...}; O=${2:?}; R=${3:?}
shift 3
mkdir -p "$O"
libpath() { [ -f "$1" ] && echo "$PWD/$1" || echo "$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_$1.so"; }
for r in $(seq 1 "$R"); do
  k=0
  for it in "$@"; do
    k=$((k + 1)); f="$O/${MODE}_${k}_$r"
    case "$MODE" in
      goku)
        MFGP_LIB_PATH=$(libpath "$it") timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline \
          --no-train-predict > "$f.json" 2> "$f.err" || exit 3
        python -c "import json; d=json.load(open('$f.json')); print('round $r [$it]', d['value'], 'evals/s', d['ms_per_step'], 'ms', d['roofline']['phase_ms'])" ;;
      env)
        envs=""; [ "$it" != "-" ] && envs="$it"
        env $envs timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --no-train-predict \
          > "$f.json" 2> "$f.err" || exit 3
        python -c "import json; d=json.load(open('$f.json')); print('round $r [$it]', d['value'], 'evals/s', d['ms_per_step'], 'ms', d['roofline']['phase_ms'])" ;;
      svgp)
        MFGP_LIB_PATH=$(libpath "$it") timeout -k 10 200 python tools/bench_svgp.py --which single --iters 40 \
          > "$f.json" 2> "$f.err" || exit 3
        python -c "import json; d=json.loads(open('$f.json').read().splitlines()[-1]); print('round $r [$it]', round(d['s_per_iter']*1e3, 4), 'ms')" ;;
      synth)
        MFGP_LIB_PATH=$(libpath "$it") timeout -k 10 200 python bench.py --config synth --steps 6 --warmup 2 \
          --no-cpu-baseline > "$f.json" 2> "$f.err" || exit 3
        python -c "import json; d=json.load(open('$f.json')); r=d['roofline']; print('round $r [$it]', d['ms_per_step'], round(r['frac'], 4), r['phase_ms'])" ;;
      *) echo "unknown mode $MODE"; exit 2 ;;
    esac
  done
done
