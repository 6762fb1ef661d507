# GPU pass: stream tests, then the configs[2] stream and configs[3] corpus lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_bench_configs.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_stream.log 2>&1 || { tail -30 gpurun_out/pytest_stream.log; exit 1; }
tail -2 gpurun_out/pytest_stream.log
bash tools/r2q.sh
