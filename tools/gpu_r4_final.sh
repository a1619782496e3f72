# Round-4 closing measurement: the three profiles with the final library.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 1000 bash tools/profile_all.sh r04 > gpurun_out/r04_prof_final.log 2>&1; echo "PROF rc=$?"; tail -5 gpurun_out/r04_prof_final.log
