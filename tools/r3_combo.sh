set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/sn_ab.py gpurun_out/sn_new.npz && AA_LIB=tools/ab/libaa_base.so timeout -k 10 120 python tools/sn_ab.py gpurun_out/sn_base.npz && python tools/sn_ab.py --compare gpurun_out/sn_new.npz gpurun_out/sn_base.npz || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_signal.py -x -q --timeout 150 --timeout-method thread > gpurun_out/sn_tests.log 2>&1 || { tail -30 gpurun_out/sn_tests.log; exit 2; }
tail -1 gpurun_out/sn_tests.log
bash tools/pipe_ab.sh || exit 3
SEC=serial,pool1,cold bash tools/r3_check.sh
