#!/bin/bash
# bit-identity of the front end and signal_noise against tools/ab/libaa_base.so,
# then an alternating A/B of the headline step (through gpurun)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/fe_ab.py gpurun_out/fe_new.npz && AA_LIB=tools/ab/libaa_base.so timeout -k 10 120 python tools/fe_ab.py gpurun_out/fe_base.npz && python tools/fe_ab.py --compare gpurun_out/fe_new.npz gpurun_out/fe_base.npz || exit 1
timeout -k 10 120 python tools/sn_ab.py gpurun_out/sn_new.npz && AA_LIB=tools/ab/libaa_base.so timeout -k 10 120 python tools/sn_ab.py gpurun_out/sn_base.npz && python tools/sn_ab.py --compare gpurun_out/sn_new.npz gpurun_out/sn_base.npz || exit 2
bash tools/ab.sh 3 main tools/ab/libaa_base.so
