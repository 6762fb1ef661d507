set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_get_end.py tests/test_corpus.py tests/test_gpu_stream.py tests/test_gpu_cli.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|max|passed|failed" gpurun_out/pytest_new.log | tail -40
exit $rc
