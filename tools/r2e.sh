set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|error|FAIL" gpurun_out/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --cpu-seconds 0 --secondary "" > gpurun_out/bench_x3.log 2>&1 || { tail -20 gpurun_out/bench_x3.log; exit 2; }
tail -1 gpurun_out/bench_x3.log | cut -c1-400
