#!/bin/bash
# in-pipeline A/B of bench.py modes on one box (through gpurun):
# alternating runs of the headline step without / with --pipeline 1
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do for P in ${MODES:-0 1 2}; do
timeout -k 10 120 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --secondary= --pipeline $P > gpurun_out/pipe_${P}_$r.json 2> gpurun_out/pipe.err || { tail -5 gpurun_out/pipe.err; exit 1; }
echo "pipeline=$P round=$r $(python -c "import json;d=json.load(open('gpurun_out/pipe_${P}_$r.json'));print(d['value'], d['ms_per_step'], d['max_abs_dlogit'])")"
done; done
