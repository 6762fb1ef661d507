# GPU pass: parity tests, front-end variants in the harness, 1x3 tile A/B, bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 90 ./tools/fe_bench_main > gpurun_out/fe_bench.log 2>&1 || { cat gpurun_out/fe_bench.log; exit 2; }
cat gpurun_out/fe_bench.log
for r in 1 2; do for v in old s0 m0 b0 main; do echo -n "$v "; timeout -k 10 60 ./tools/fe_bench_$v 1 | grep DIAG || exit 2; done; done
timeout -k 10 600 bash tools/ab.sh 3 main tools/ab/libaa_o1x3a.so tools/ab/libaa_o1x3b.so || exit 3
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.log
