#!/bin/bash
# round-3 check (through gpurun): the headline line with its secondaries, and
# the signal_noise kernel split of 60 s clips.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --cpu-seconds 0 --secondary=${SEC:-serial,pool1,cold} > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 4; }
cat gpurun_out/b.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/snprof -o run -- python3 tools/sn_bench.py 60 > gpurun_out/snp.log 2>&1 || exit 5
python tools/prof_summary.py gpurun_out/snprof > gpurun_out/sn_kernels.txt && cat gpurun_out/sn_kernels.txt
