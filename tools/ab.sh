#!/bin/bash
# In-pipeline A/B of libaa variants on one GPU box: alternating bench runs.
# usage (through gpurun): [AB_ARGS="--model effnetv2"] bash tools/ab.sh ROUNDS lib1 lib2 ...   (paths; "main" = the in-tree libaa.so)
set -o pipefail
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for L in "$@"; do
    if [ "$L" = main ]; then unset AA_LIB; else export AA_LIB=$PWD/$L AA_LIB_AB=1; fi
    timeout -k 10 120 python bench.py --steps 100 --warmup 20 --cpu-seconds 0 --secondary= --no-parity ${AB_ARGS:-} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$L" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/bench_full.json").read())  # the full record (the printed line has no stage tables)
st = d["roofline"]["stages_ms"]
print(f"{sys.argv[1]:28s} {d['value']:9.1f}  " + " ".join(f"{k.split('_')[1] if k.startswith('conv') else k[:8]}={1e3*v:6.1f}" for k, v in st.items()), flush=True)
PY
  done
done
