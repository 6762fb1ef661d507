#!/bin/bash
# signal_noise A/B (through gpurun): masks and components of the working tree
# against tools/ab/libaa_base.so (bit-identical), the signal / batch / get_end
# GPU tests, then configs[3] lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/sn_ab.py gpurun_out/sn_new.npz && AA_LIB=tools/ab/libaa_base.so timeout -k 10 120 python tools/sn_ab.py gpurun_out/sn_base.npz && python tools/sn_ab.py --compare gpurun_out/sn_new.npz gpurun_out/sn_base.npz || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_signal.py tests/test_gpu_batch.py tests/test_get_end.py tests/test_gpu_frontend.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sn_tests.log 2>&1 || { tail -30 gpurun_out/sn_tests.log; exit 2; }
tail -2 gpurun_out/sn_tests.log
for L in ${LANES:-1 3}; do
AA_BATCH_LANES=$L AA_BATCH_PROFILE=1 timeout -k 10 200 python bench.py --config 4 --files 256 --batch 32 > gpurun_out/c4_$L.json 2> gpurun_out/c4_$L.err || { tail -5 gpurun_out/c4_$L.err; exit 3; }
echo "lanes=$L $(python -c "import json;print(json.load(open('gpurun_out/c4_$L.json'))['value'])") $(grep -h 'over 256' gpurun_out/c4_$L.err)"
done
