#!/bin/bash
# round-3 check (through gpurun): the default bench line, its kernel-trace
# summary, and configs[3] with 1 / 2 host processes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
cat gpurun_out/b.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bprof -o run -- python3 bench.py --steps 25 --warmup 5 --cpu-seconds 0 --secondary= > gpurun_out/bp.log 2>&1 || exit 2
python tools/prof_summary.py gpurun_out/bprof > gpurun_out/b_kernels.txt && cat gpurun_out/b_kernels.txt
for P in 1 2; do
AA_BATCH_PROFILE=1 timeout -k 10 300 python bench.py --config 4 --files 256 --procs-per-gpu $P > gpurun_out/c4p_$P.json 2> gpurun_out/c4p_$P.err || { tail -8 gpurun_out/c4p_$P.err; exit 3; }
echo "procs=$P $(tail -1 gpurun_out/c4p_$P.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'])")"
done
