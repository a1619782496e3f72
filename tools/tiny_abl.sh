# k_gpr_tiny phase ablation (GPU box, repo root): kernel time per TINY_STOP variant.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tinyabl
for v in ${TINY_VARIANTS:-full}; do
  lib=multi_fidelity_gpflow_amd/variants/libmfgp_$v.so
  [ $v = full ] && lib=multi_fidelity_gpflow_amd/libmfgp.so
  MFGP_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tinyabl/$v -o run -- python3 tools/tiny_abl.py > gpurun_out/tinyabl/$v.log 2>&1 || exit $?
  f=$(find gpurun_out/tinyabl/$v -name "*kernel_stats.csv" | head -1)
  echo "$v $(grep k_gpr_tiny "$f" | cut -d, -f2-4)"
done
