#!/bin/bash
# configs[3] corpus line repeated on one box (through gpurun): value and host phases per run
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${RUNS:-3}); do
AA_BATCH_PROFILE=1 timeout -k 10 200 python bench.py --config 4 --files ${FILES:-256} --batch 32 > gpurun_out/c4r_$r.json 2> gpurun_out/c4r_$r.err || { tail -5 gpurun_out/c4r_$r.err; exit 1; }
echo "run=$r $(python -c "import json;print(json.load(open('gpurun_out/c4r_$r.json'))['value'])") $(grep -h 'over ' gpurun_out/c4r_$r.err)"
done
