# GPU pass: SQ counters of the front-end kernel, 3x3/32->64 tile A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 bash tools/pmc_fe.sh > gpurun_out/pmc_fe.txt 2>&1 || { tail -20 gpurun_out/pmc_fe.txt; exit 1; }
grep -A25 "fe_stft_mel_4096" gpurun_out/pmc_fe.txt | head -30
timeout -k 10 600 bash tools/ab.sh 3 main tools/ab/libaa_c2a.so tools/ab/libaa_c2b.so || exit 3
