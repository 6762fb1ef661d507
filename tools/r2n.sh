# GPU pass: A/B of fe_db tile heights and the head's load batching
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/ab.sh 3 main tools/ab/libaa_db8.so tools/ab/libaa_db24.so tools/ab/libaa_h4.so tools/ab/libaa_h8.so || exit 3
