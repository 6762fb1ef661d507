#!/bin/bash
# configs[3] sweep (through gpurun): corpus bench lines over lanes x batch x
# files, then the kernel-trace summary of the default configuration.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for F in 256 1024; do for L in 3 4; do for B in 32 64; do
AA_BATCH_LANES=$L AA_BATCH_PROFILE=1 timeout -k 10 200 python bench.py --config 4 --files $F --batch $B > gpurun_out/c4_${F}_${L}_${B}.json 2> gpurun_out/c4_${F}_${L}_${B}.err || { tail -5 gpurun_out/c4_${F}_${L}_${B}.err; exit 2; }
echo "files=$F lanes=$L batch=$B $(python -c "import json;print(json.load(open('gpurun_out/c4_${F}_${L}_${B}.json'))['value'])") $(grep -h "over $F" gpurun_out/c4_${F}_${L}_${B}.err)"
done; done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o run -- python3 bench.py --config 4 --files 256 > gpurun_out/c4p.log 2>&1 || exit 3
python tools/prof_summary.py gpurun_out/c4prof > gpurun_out/c4_kernels.txt && head -24 gpurun_out/c4_kernels.txt
