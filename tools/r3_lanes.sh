set -o pipefail
export TMPDIR=/tmp
MODES="2 3 4" bash tools/pipe_ab.sh || exit 1
timeout -k 10 300 python bench.py --cpu-seconds 0 --secondary=serial > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 2; }
python -c "import json;d=json.load(open('gpurun_out/b.json'));r=d['roofline'];print(d['value'], r['kernel'], r['avg_ms'], r['frac'], r['overlapped_avg_ms'], d['secondary']['serial']['value'])"
