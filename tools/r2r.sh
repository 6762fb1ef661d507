# GPU pass: CNN parity tests, then A/B of the fused tiles 9x21 and 12x15 against 12x21
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_config_step.py tests/test_gpu_pipeline.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_cnn.log 2>&1 || { tail -30 gpurun_out/pytest_cnn.log; exit 1; }
tail -2 gpurun_out/pytest_cnn.log
timeout -k 10 1000 bash tools/ab.sh 3 main tools/ab/libaa_f9.so tools/ab/libaa_f15.so || exit 3
