# GPU pass: what the round-end driver runs (GPU tests, smoke, default bench line)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 2; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 3; }
cat gpurun_out/bench.log
