set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/conv_bench_x3 19 > gpurun_out/cb19.txt 2>&1 || { tail -5 gpurun_out/cb19.txt; exit 1; }
cat gpurun_out/cb19.txt
timeout -k 10 300 bash tools/pmc_sq.sh fz ./tools/conv_bench_x3 20 > gpurun_out/pmc_fz.txt 2>&1 || { tail -20 gpurun_out/pmc_fz.txt; exit 2; }
cat gpurun_out/pmc_fz.txt
