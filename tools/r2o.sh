# GPU pass: A/B of VGPR-form MFMA (no AGPR accumulators) for the CNN kernels
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab.sh 4 main tools/ab/libaa_vgprf.so || exit 3
