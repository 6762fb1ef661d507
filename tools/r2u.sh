# GPU pass: configs[3] corpus line with and without the upload in the prefetch (A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do for u in 1 0; do
  AA_CORPUS_UPLOAD=$u timeout -k 10 300 python bench.py --config 4 --files 32 > gpurun_out/bench_config4_u$u.json 2> gpurun_out/bench_config4.err || { tail gpurun_out/bench_config4.err; exit 3; }
  echo "upload=$u $(grep -o '"value": [0-9.]*' gpurun_out/bench_config4_u$u.json)"
done; done
