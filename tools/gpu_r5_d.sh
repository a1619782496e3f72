# Round 5: chain timelines (tools/flow_trace.py) of the in-flow Gram build and the round-4 build.
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 120 python tools/flow_trace.py 5 > $O/trace_new.txt 2>&1; echo "new rc=$?"
MFGP_LIB_PATH=$PWD/multi_fidelity_gpflow_amd/variants/libmfgp_base.so timeout -k 10 120 python tools/flow_trace.py 5 > $O/trace_base.txt 2>&1; echo "base rc=$?"
exit 0
