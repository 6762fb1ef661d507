# GPU pass: A/B of global-B (no LDS weight ring) variants of the small conv layers
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/ab.sh 3 main tools/ab/libaa_r32a.so tools/ab/libaa_r32b.so tools/ab/libaa_r64a.so tools/ab/libaa_r64b.so tools/ab/libaa_r13.so || exit 3
