#!/bin/bash
# One parameterised GPU-box runner (replaces the per-round gpu_r4_* / gpu_r5_* scripts).
#   bash tools/gpu_run.sh OUTDIR STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failing step ends the script.
#   tests            the whole -m gpu suite                       -> OUTDIR/gpu_tests.log
#   pytest:ARGS      pytest on ARGS (comma-separated words)      -> OUTDIR/pytest_N.log
#   smoke            __graft_entry__.smoke()                      -> OUTDIR/smoke.log
#   bench[:ARGS]     bench.py ARGS (comma-separated)              -> OUTDIR/bench_N.json
#   dist2:CFG        two gloo ranks sharing the GPU, bench.py --gpus 2 --config CFG
#   profile:CFG      tools/profile_round.sh (trace + PMC passes)  -> OUTDIR/CFG/
#   py:SCRIPT[,ARGS] python SCRIPT ARGS                           -> OUTDIR/py_N.log
#   rccl             one rank, world-size-1 nccl group, shared-theta line -> OUTDIR/rccl_ws1_shared.json
#   svgptrace        kernel trace of 30 single-bin SVGP iterations  -> OUTDIR/svgp_single_trace/
#   cpuproto         the CPU baseline's full 1000-step protocol    -> OUTDIR/cpu_protocol.json
# (A/B runs: tools/ab.sh.)
set -o pipefail
export TMPDIR=/tmp
O=${1:?usage: gpu_run.sh OUTDIR STEP...}
shift
mkdir -p "$O"
i=0
for step in "$@"; do
  i=$((i + 1))
  name=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=$(echo "${step#*:}" | tr ',' ' ')
  t0=$(date +%s)
  case "$name" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$O/gpu_tests.log" 2>&1; rc=$?; tail -2 "$O/gpu_tests.log" ;;
    pytest)
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $arg \
        > "$O/pytest_$i.log" 2>&1; rc=$?; tail -3 "$O/pytest_$i.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 600 python bench.py $arg > "$O/bench_$i.json" 2> "$O/bench_$i.err"; rc=$?
      head -c 600 "$O/bench_$i.json"; echo ;;
    dist2)
      MFGP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --config "$arg" --no-cpu-baseline \
        > "$O/dist2_$arg.out" 2> "$O/dist2_$arg.err"; rc=$?
      grep '^{' "$O/dist2_$arg.out" > "$O/dist2_$arg.json" ;;
    profile)
      case "$arg" in
        goku) bash tools/profile_round.sh "$O/goku" goku "--no-extras" \
                "--steps 20 --warmup 5 --no-cpu-baseline --no-train-predict --no-extras" ;;
        synth) bash tools/profile_round.sh "$O/synth" synth "--steps 6 --warmup 2" "--steps 2 --warmup 1" ;;
        goku_svgp) bash tools/profile_round.sh "$O/goku_svgp" goku_svgp "--steps 50 --warmup 20" \
                "--steps 10 --warmup 10 --no-train-predict --no-latent" \
                "--steps 50 --warmup 20 --no-train-predict --no-cpu-baseline" ;;
        *) echo "unknown profile config $arg"; false ;;
      esac; rc=$? ;;
    rccl)
      MFGP_DIST_WS1=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29555 bench.py --mode shared --no-extras --no-cpu-baseline \
        --no-train-predict --steps 300 > "$O/rccl_ws1_shared.out" 2> "$O/rccl_ws1_shared.err"; rc=$?
      [ $rc -eq 0 ] && { grep '^{' "$O/rccl_ws1_shared.out" > "$O/rccl_ws1_shared.json"; rc=$?; }
      head -c 700 "$O/rccl_ws1_shared.json"; echo ;;
    svgptrace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/svgp_single_trace" -o run -- \
        python3 tools/bench_svgp.py --which single --iters 30 > "$O/svgp_single.json" 2> "$O/svgp_single.err"; rc=$?
      cat "$O/svgp_single.json" ;;
    cpuproto)
      timeout -k 10 300 python tools/cpu_protocol.py "$O/cpu_protocol.json" > "$O/cpu_protocol.log" 2>&1; rc=$?
      cat "$O/cpu_protocol.json" ;;
    py)
      timeout -k 10 600 python -u $arg > "$O/py_$i.log" 2>&1; rc=$?; tail -30 "$O/py_$i.log" ;;
    *)
      echo "unknown step $step"; rc=2 ;;
  esac
  echo "STEP $i $step rc=$rc ($(( $(date +%s) - t0 )) s)"
  [ $rc -eq 0 ] || exit $rc
done
