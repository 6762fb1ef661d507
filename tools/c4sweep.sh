set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in 1 2 3 4; do for B in 16 32; do
AA_BATCH_LANES=$L AA_BATCH_PROFILE=1 timeout -k 10 200 python bench.py --config 4 --files 256 --batch $B > gpurun_out/c4_${L}_${B}.json 2> gpurun_out/c4_${L}_${B}.err || { tail -5 gpurun_out/c4_${L}_${B}.err; exit 2; }
echo "lanes=$L batch=$B $(python -c "import json;print(json.load(open('gpurun_out/c4_${L}_${B}.json'))['value'])") $(grep -h 'over 256' gpurun_out/c4_${L}_${B}.err)"
done; done
