# GPU pass: SQ counters of every bench kernel (headline precision), then the
# profile round (tests, PMC traffic, kernel stats, bench line)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 bash tools/pmc_sq.sh bench python3 bench.py --steps 3 --warmup 2 --cpu-seconds 0 --secondary= --no-parity > gpurun_out/pmc_sq_bench.txt 2>&1 || { tail -20 gpurun_out/pmc_sq_bench.txt; exit 1; }
bash tools/gpu_round.sh r02 bf16x3 bf16 fp8
