#!/bin/bash
# conv_x3 change check (through gpurun): CNN parity tests on the working-tree
# build, then an alternating A/B against tools/ab/libaa_$1.so
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_config_step.py -x -q --timeout 200 --timeout-method thread > gpurun_out/x3_tests.log 2>&1 || { tail -30 gpurun_out/x3_tests.log; exit 1; }
tail -1 gpurun_out/x3_tests.log
bash tools/ab.sh ${ROUNDS:-3} main tools/ab/libaa_$1.so
