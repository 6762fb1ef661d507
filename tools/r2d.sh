set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_config_step.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/pytest_cnn.log 2>&1; rc=$?
grep -E "bf16x3|passed|failed|Error|error" gpurun_out/pytest_cnn.log | tail -14
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 ./tools/conv_bench_x3 > gpurun_out/cb3.log 2>&1; cat gpurun_out/cb3.log
timeout -k 10 100 ./tools/conv_bench_x3 9 > gpurun_out/cb3a.log 2>&1; cat gpurun_out/cb3a.log
timeout -k 10 300 python bench.py --cpu-seconds 0 --secondary "" > gpurun_out/bench_x3.log 2>&1 || { tail -20 gpurun_out/bench_x3.log; exit 2; }
tail -1 gpurun_out/bench_x3.log
