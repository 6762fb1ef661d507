#!/bin/bash
# Front-end A/B on one GPU box: the in-tree libaa.so against tools/ablib/libaa_NAME.so
# variants (tools/ab_head.py, or tools/ab_build.py with AB_FE_DEFS): the log-mel
# must be bit-identical (tools/fe_ab.py), then a kernel trace of the serial
# bench step per library, alternating, prints the front-end kernels' times.
# usage (through gpurun): bash tools/fe_kernel_ab.sh ROUNDS NAME [NAME ...]
set -o pipefail
export TMPDIR=/tmp
R=$1; shift
mkdir -p gpurun_out
timeout -k 10 200 python tools/fe_ab.py gpurun_out/fe_main.npz > gpurun_out/fe_ab.log 2>&1 || exit 1
for N in "$@"; do
  AA_LIB=$PWD/tools/ablib/libaa_$N.so AA_LIB_AB=1 timeout -k 10 200 python tools/fe_ab.py gpurun_out/fe_$N.npz >> gpurun_out/fe_ab.log 2>&1 || exit 2
  python tools/fe_ab.py --compare gpurun_out/fe_main.npz gpurun_out/fe_$N.npz || exit 3
done
for r in $(seq 1 $R); do
  for L in main "$@"; do
    if [ $L = main ]; then unset AA_LIB; else export AA_LIB=$PWD/tools/ablib/libaa_$L.so AA_LIB_AB=1; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/st_${L}_$r -o run -- python3 bench.py --steps 25 --warmup 5 --cpu-seconds 0 --secondary= --pipeline 0 --no-parity > gpurun_out/st_${L}_$r.log 2>&1 || exit 4
    python tools/prof_summary.py /tmp/st_${L}_$r > gpurun_out/ks_${L}_$r.txt || exit 5
    echo "== $L $r"; grep -E "fe_db|fe_stft|fe_stats" gpurun_out/ks_${L}_$r.txt
  done
done
