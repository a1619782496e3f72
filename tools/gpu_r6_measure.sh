#!/bin/bash
# Round-6 measurement pass (GPU box, repo root): the default line, the RCCL world-size-1 shared-theta
# line, the CPU baseline's full protocol, and a single-bin SVGP kernel trace.  OUT=$1
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06e}
mkdir -p "$O"
bash tools/gpu_run.sh "$O" bench || exit 3
MFGP_DIST_WS1=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29555 bench.py --mode shared --no-extras --no-cpu-baseline \
  --no-train-predict --steps 300 > "$O/rccl_ws1_shared.out" 2> "$O/rccl_ws1_shared.err" || exit 4
grep '^{' "$O/rccl_ws1_shared.out" > "$O/rccl_ws1_shared.json" || exit 5
head -c 700 "$O/rccl_ws1_shared.json"; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/svgp_single_trace" -o run -- \
  python3 tools/bench_svgp.py --which single --iters 30 > "$O/svgp_single.json" 2> "$O/svgp_single.err" || exit 6
cat "$O/svgp_single.json"
timeout -k 10 300 python tools/cpu_protocol.py "$O/cpu_protocol.json" > "$O/cpu_protocol.log" 2>&1 || exit 7
cat "$O/cpu_protocol.json"
