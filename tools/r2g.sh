set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_keras_import.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_keras.log 2>&1; rc=$?
grep -E "max\|dlogit|PASS|FAIL|Error|error" gpurun_out/pytest_keras.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
exit $rc
