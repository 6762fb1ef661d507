#!/bin/bash
# One GPU-box pass: parity tests, PMC traffic of a bench step, the kernel-trace
# summary, then the bench line (which reads the traffic summary).
# usage (through gpurun): bash tools/gpu_round.sh r01
set -o pipefail
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out profiles/$R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 2 --cpu-seconds 0 > gpurun_out/pmc_fetch.log 2>&1 || exit 2
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 3 --warmup 2 --cpu-seconds 0 > gpurun_out/pmc_write.log 2>&1 || exit 3
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_traffic.json || exit 4
cp gpurun_out/pmc_traffic.json profiles/$R/pmc_traffic.json
# the fp8 CNN (BASELINE configs[4] precision): its own traffic summary
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc8_fetch -o run -- python3 bench.py --precision fp8 --steps 3 --warmup 2 --cpu-seconds 0 > gpurun_out/pmc8_fetch.log 2>&1 || exit 7
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc8_write -o run -- python3 bench.py --precision fp8 --steps 3 --warmup 2 --cpu-seconds 0 > gpurun_out/pmc8_write.log 2>&1 || exit 8
python tools/pmc_traffic.py gpurun_out/pmc8_fetch gpurun_out/pmc8_write gpurun_out/pmc_traffic_fp8.json fp8 || exit 9
cp gpurun_out/pmc_traffic_fp8.json profiles/$R/pmc_traffic_fp8.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- python3 bench.py --steps 25 --warmup 5 --cpu-seconds 0 > gpurun_out/stats.log 2>&1 || exit 5
python tools/prof_summary.py gpurun_out/stats > gpurun_out/kernel_stats.txt
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 6; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats8 -o run -- python3 bench.py --precision fp8 --steps 25 --warmup 5 --cpu-seconds 0 > gpurun_out/stats8.log 2>&1 || exit 10
python tools/prof_summary.py gpurun_out/stats8 > gpurun_out/kernel_stats_fp8.txt
timeout -k 10 300 python bench.py --precision fp8 > gpurun_out/bench_fp8.log 2>&1 || { cat gpurun_out/bench_fp8.log; exit 11; }
cat gpurun_out/kernel_stats.txt
tail -1 gpurun_out/bench.log
