#!/bin/bash
# conv_wg32 check (through gpurun): CNN parity tests on the variant build, then A/B against main
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AA_LIB=$PWD/tools/ab/libaa_wg32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_config_step.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wg32_tests.log 2>&1 || { tail -30 gpurun_out/wg32_tests.log; exit 1; }
tail -1 gpurun_out/wg32_tests.log
bash tools/ab.sh 3 main tools/ab/libaa_wg32.so
