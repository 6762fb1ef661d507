#!/bin/bash
# host-side profile of the batched corpus path (through gpurun): one lane, the
# lane thread under cProfile, top functions by own time
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/cprof.*
AA_BATCH_LANES=1 AA_BATCH_CPROFILE=gpurun_out/cprof timeout -k 10 300 python bench.py --config 4 --files 256 > gpurun_out/c4cp.json 2> gpurun_out/c4cp.err || { tail -5 gpurun_out/c4cp.err; exit 1; }
cat gpurun_out/c4cp.json
python - <<'PY'
import glob, pstats
fs = sorted(glob.glob("gpurun_out/cprof.*"))
st = pstats.Stats(fs[-1])
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumtime").print_stats(30)
PY
