# GPU pass: configs[2] stream (split-bf16, fp8) and configs[3] corpus bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 3 --clips 400 > gpurun_out/bench_config3.json 2> gpurun_out/bench_config3.err || { tail gpurun_out/bench_config3.err; exit 1; }
cat gpurun_out/bench_config3.json
timeout -k 10 300 python bench.py --config 3 --clips 400 --precision fp8 > gpurun_out/bench_config3_fp8.json 2> gpurun_out/bench_config3_fp8.err || { tail gpurun_out/bench_config3_fp8.err; exit 2; }
cat gpurun_out/bench_config3_fp8.json
timeout -k 10 300 python bench.py --config 4 --files 32 > gpurun_out/bench_config4.json 2> gpurun_out/bench_config4.err || { tail gpurun_out/bench_config4.err; exit 3; }
cat gpurun_out/bench_config4.json
