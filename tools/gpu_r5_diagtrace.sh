#!/bin/bash
# Round 5: kernel traces of one Synth step with each k32_diag variant (timeline of the lookahead)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dtr
for v in prediag diag79; do
  MFGP_LIB_PATH=multi_fidelity_gpflow_amd/variants/libmfgp_$v.so timeout -k 10 300 rocprofv3 --kernel-trace \
    --output-format csv -d gpurun_out/dtr/$v -o tr -- python3 bench.py --config synth --steps 2 --warmup 1 \
    --no-cpu-baseline --no-train-predict > gpurun_out/dtr/$v.json 2> gpurun_out/dtr/$v.err || exit $?
done
find gpurun_out/dtr -name "*.csv" | head
