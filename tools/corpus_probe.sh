#!/bin/bash
# configs[3] probe (through gpurun): the CLI parity test, the corpus bench with
# its per-phase host timing (AA_BATCH_PROFILE), the kernel-trace summary of the
# same run, and the headline bench line without the CPU leg.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
FILES=${1:-256}
timeout -k 10 240 python -u -m pytest tests/test_gpu_cli.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/cli.log 2>&1 || { tail -30 gpurun_out/cli.log; exit 1; }
grep -h "max|d" gpurun_out/cli.log
AA_BATCH_PROFILE=1 timeout -k 10 300 python bench.py --config 4 --files $FILES > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 2; }
cat gpurun_out/c4.json; grep -h "batch phases" gpurun_out/c4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o run -- python3 bench.py --config 4 --files $FILES > gpurun_out/c4p.log 2>&1 || exit 3
python tools/prof_summary.py gpurun_out/c4prof > gpurun_out/c4_kernels.txt && head -30 gpurun_out/c4_kernels.txt
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 4; }
cat gpurun_out/b.json
