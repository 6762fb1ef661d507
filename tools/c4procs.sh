#!/bin/bash
# configs[3] with 1..3 host processes per GPU (through gpurun)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for P in 1 2 3; do for L in 2 3; do
AA_BATCH_LANES=$L AA_BATCH_PROFILE=1 timeout -k 10 300 python bench.py --config 4 --files 256 --batch 32 --procs-per-gpu $P > gpurun_out/c4p_${P}_${L}.json 2> gpurun_out/c4p_${P}_${L}.err || { tail -8 gpurun_out/c4p_${P}_${L}.err; exit 3; }
echo "procs=$P lanes=$L $(python -c "import json;d=json.load(open('gpurun_out/c4p_${P}_${L}.json'));print(d['value'], d['n_gpus'], d['config']['documents_gathered'])")"
done; done
