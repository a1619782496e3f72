# Round-4 closing measurement: default bench line and the three profiles with the final library.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 400 python bench.py > gpurun_out/r04/bench_default_final.json 2> gpurun_out/r04/bench_default_final.err; echo "BENCH rc=$?"
python -c "import json; d=json.load(open('gpurun_out/r04/bench_default_final.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['hbs']['train_predict_s'], d['goku_svgp']['ms_per_step'], d['synth']['ms_per_step'])"
timeout -k 10 900 bash tools/profile_all.sh r04 > gpurun_out/r04_prof_final.log 2>&1; echo "PROF rc=$?"
