#!/bin/bash
# One GPU-box pass: parity tests, PMC traffic of a bench step per precision,
# the kernel-trace summary of the headline, then the bench line (which reads
# the traffic summary).
# usage (through gpurun): bash tools/gpu_round.sh r02 [precision ...]
set -o pipefail
R=${1:-r02}
shift
PRECS=${@:-bf16x3 bf16 fp8}
export TMPDIR=/tmp
mkdir -p gpurun_out profiles/$R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
B="--steps 3 --warmup 2 --cpu-seconds 0 --secondary="
for P in $PRECS; do
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$P -o run -- python3 bench.py --precision $P $B > gpurun_out/pmc_fetch_$P.log 2>&1 || exit 2
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$P -o run -- python3 bench.py --precision $P $B > gpurun_out/pmc_write_$P.log 2>&1 || exit 3
  python tools/pmc_traffic.py gpurun_out/pmc_fetch_$P gpurun_out/pmc_write_$P gpurun_out/pmc_traffic_$P.json $P > /dev/null || exit 4
  cp gpurun_out/pmc_traffic_$P.json profiles/$R/pmc_traffic_$P.json
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_$P -o run -- python3 bench.py --precision $P --steps 25 --warmup 5 --cpu-seconds 0 --secondary= > gpurun_out/stats_$P.log 2>&1 || exit 5
  python tools/prof_summary.py gpurun_out/stats_$P > gpurun_out/kernel_stats_$P.txt
  cp gpurun_out/kernel_stats_$P.txt profiles/$R/bench_kernel_stats_$P.txt
  cp gpurun_out/stats_$P/*kernel_stats.csv profiles/$R/bench_kernel_stats_$P.csv 2>/dev/null || cp gpurun_out/stats_$P/*/*kernel_stats.csv profiles/$R/bench_kernel_stats_$P.csv
done
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { cat gpurun_out/bench.err; exit 6; }
cp gpurun_out/bench.log profiles/$R/bench.json
cat gpurun_out/kernel_stats_bf16x3.txt
tail -1 gpurun_out/bench.log
