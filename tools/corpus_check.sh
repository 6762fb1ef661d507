#!/bin/bash
# corpus-path check (through gpurun): the pipeline / batch / CLI / corpus /
# signal / stream GPU tests, configs[3] lines (3 runs) and the configs[2] stream line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_batch.py tests/test_gpu_cli.py tests/test_corpus.py tests/test_gpu_signal.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > gpurun_out/corpus_tests.log 2>&1 || { tail -30 gpurun_out/corpus_tests.log; exit 1; }
tail -1 gpurun_out/corpus_tests.log
for r in 1 2 3; do
AA_BATCH_PROFILE=1 timeout -k 10 300 python bench.py --config 4 --files 256 > gpurun_out/c4_$r.json 2> gpurun_out/c4_$r.err || { tail -8 gpurun_out/c4_$r.err; exit 2; }
echo "run $r $(python -c "import json;print(json.load(open('gpurun_out/c4_$r.json'))['value'])") $(grep -h 'over 256' gpurun_out/c4_$r.err)"
done
timeout -k 10 300 python bench.py --config 3 --clips 400 > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail -8 gpurun_out/c3.err; exit 3; }
python -c "import json;print(\"config3\", json.load(open(\"gpurun_out/c3.json\"))[\"value\"])"
