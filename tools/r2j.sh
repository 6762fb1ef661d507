# GPU pass: parity tests, front-end harness, bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 90 ./tools/fe_bench > gpurun_out/fe_bench.log 2>&1 || { cat gpurun_out/fe_bench.log; exit 2; }
cat gpurun_out/fe_bench.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.log
