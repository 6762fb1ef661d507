# GPU pass: A/B of precomputed fragment addresses in every conv_x3 kernel
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab.sh 4 main tools/ab/libaa_aoff.so || exit 3
