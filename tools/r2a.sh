set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py --precision f32 --cpu-seconds 5 > gpurun_out/bench_f32.log 2>&1 || { cat gpurun_out/bench_f32.log; exit 2; }
timeout -k 10 200 python bench.py --precision bf16 --cpu-seconds 0 > gpurun_out/bench_bf16.log 2>&1 || { cat gpurun_out/bench_bf16.log; exit 3; }
tail -1 gpurun_out/bench_f32.log; tail -1 gpurun_out/bench_bf16.log
