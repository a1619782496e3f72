set -o pipefail
mkdir -p gpurun_out/r4tiny
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -k "tiny or lml or lbfgs or adam or non_pd or graph" > gpurun_out/r4tiny/parity2.log 2>&1; rc=$?; echo "PARITY rc=$rc"; grep -E "tiny vs|L-BFGS Forrester|hbs \{|passed|failed|FAILED" gpurun_out/r4tiny/parity2.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4tiny/prof_on -o run -- python3 tools/tp_breakdown.py hbs > gpurun_out/r4tiny/on.txt 2>&1; echo "ON rc=$?"; tail -2 gpurun_out/r4tiny/on.txt
MFGP_TINY=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4tiny/prof_off -o run -- python3 tools/tp_breakdown.py hbs > gpurun_out/r4tiny/off.txt 2>&1; echo "OFF rc=$?"; tail -2 gpurun_out/r4tiny/off.txt
for d in prof_on prof_off; do f=$(find gpurun_out/r4tiny/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; head -8 "$f" | cut -d, -f1-8; done
timeout -k 10 300 python tools/tp_breakdown.py hbs > gpurun_out/r4tiny/hbs_on.txt 2>&1; tail -2 gpurun_out/r4tiny/hbs_on.txt
