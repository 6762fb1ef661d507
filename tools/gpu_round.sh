#!/bin/bash
# GPU-box passes (run through gpurun); everything lands in gpurun_out/ (copy
# the summaries DESIGN.md cites into profiles/rNN/).
#
#   bash tools/gpu_round.sh round [prec ...]  parity tests, PMC traffic of a bench
#                                             step per precision, kernel traces of the
#                                             default and serial steps, the bench
#                                             line, smoke (default mode)
#   bash tools/gpu_round.sh corpus [files]    configs[3]: CLI parity, the corpus line
#                                             with host phases (RUNS repeats, default
#                                             1), its kernel-trace summary
#   bash tools/gpu_round.sh sn                signal_noise: GPU parity tests, per-clip
#                                             time and its kernel-trace summary
#   bash tools/gpu_round.sh graph             graph executor: GPU parity tests, the
#                                             EfficientNetV2-shaped bench line and the
#                                             kernel-trace summary of its serial step
#   bash tools/gpu_round.sh ab NAME [rounds]  CNN parity tests, then alternating bench
#                                             runs of the in-tree library against
#                                             tools/ablib/libaa_NAME.so (tools/ab.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
MODE=${1:-round}
[ $# -gt 0 ] && shift
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"

case $MODE in
round)
  PRECS=${@:-bf16x3}
  timeout -k 10 900 $PT tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
  # PMC passes on the serial step (per-launch bytes do not depend on the
  # overlap; the dispatch order of one step stays that of the stage list)
  B="--steps 3 --warmup 2 --cpu-seconds 0 --secondary= --pipeline 0"
  for P in $PRECS; do
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$P -o run -- python3 bench.py --precision $P $B > gpurun_out/pmc_fetch_$P.log 2>&1 || exit 2
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$P -o run -- python3 bench.py --precision $P $B > gpurun_out/pmc_write_$P.log 2>&1 || exit 3
    python tools/pmc_traffic.py gpurun_out/pmc_fetch_$P gpurun_out/pmc_write_$P gpurun_out/pmc_traffic_$P.json $P > /dev/null || exit 4
    # kernel-trace summary of the default (overlapped) step: its durations are
    # the ones the bench line's live events see
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_$P -o run -- python3 bench.py --precision $P --steps 25 --warmup 5 --cpu-seconds 0 --secondary= > gpurun_out/stats_$P.log 2>&1 || exit 5
    python tools/prof_summary.py gpurun_out/stats_$P > gpurun_out/kernel_stats_$P.txt
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_serial_$P -o run -- python3 bench.py --precision $P --steps 25 --warmup 5 --cpu-seconds 0 --secondary= --pipeline 0 > gpurun_out/stats_serial_$P.log 2>&1 || exit 6
    python tools/prof_summary.py gpurun_out/stats_serial_$P > gpurun_out/kernel_stats_serial_$P.txt
  done
  # the bench line reads the traffic and serial-trace summaries from profiles/:
  # on the box, give it this pass's (PROFILE_DIR, e.g. profiles/r04; the local
  # copy is made from gpurun_out/ afterwards)
  if [ -n "$PROFILE_DIR" ]; then
    for P in $PRECS; do
      cp gpurun_out/pmc_traffic_$P.json "$PROFILE_DIR/" && cp gpurun_out/stats_serial_$P/run_kernel_stats.csv "$PROFILE_DIR/bench_kernel_stats_serial_$P.csv" || exit 9
    done
  fi
  timeout -k 10 500 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { cat gpurun_out/bench.err; exit 7; }
  cat gpurun_out/kernel_stats_serial_bf16x3.txt
  tail -1 gpurun_out/bench.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 8; }
  tail -2 gpurun_out/smoke.log
  ;;
corpus)
  FILES=${1:-256}
  timeout -k 10 240 $PT tests/test_gpu_cli.py tests/test_gpu_batch.py > gpurun_out/corpus_tests.log 2>&1 || { tail -30 gpurun_out/corpus_tests.log; exit 1; }
  tail -1 gpurun_out/corpus_tests.log
  for r in $(seq 1 ${RUNS:-1}); do
    AA_BATCH_PROFILE=1 timeout -k 10 300 python bench.py --config 4 --files $FILES > gpurun_out/c4_$r.json 2> gpurun_out/c4_$r.err || { tail -20 gpurun_out/c4_$r.err; exit 2; }
    echo "run=$r $(tail -1 gpurun_out/c4_$r.json)"; grep -h "batch phases" gpurun_out/c4_$r.err
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o run -- python3 bench.py --config 4 --files $FILES > gpurun_out/c4p.log 2>&1 || exit 3
  python tools/prof_summary.py gpurun_out/c4prof > gpurun_out/corpus_kernel_stats.txt && head -30 gpurun_out/corpus_kernel_stats.txt
  ;;
sn)
  timeout -k 10 600 $PT tests/test_gpu_signal.py tests/test_get_end.py > gpurun_out/sn_tests.log 2>&1 || { tail -30 gpurun_out/sn_tests.log; exit 1; }
  tail -1 gpurun_out/sn_tests.log
  timeout -k 10 200 python tools/sn_bench.py > gpurun_out/sn_bench.txt 2>&1 || { tail -20 gpurun_out/sn_bench.txt; exit 2; }
  cat gpurun_out/sn_bench.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/snprof -o run -- python3 tools/sn_bench.py > gpurun_out/snp.log 2>&1 || exit 3
  python tools/prof_summary.py gpurun_out/snprof > gpurun_out/sn_kernel_stats.txt && cat gpurun_out/sn_kernel_stats.txt
  ;;
graph)
  timeout -k 10 400 $PT tests/test_gpu_graph.py > gpurun_out/graph_tests.log 2>&1 || { tail -30 gpurun_out/graph_tests.log; exit 1; }
  tail -1 gpurun_out/graph_tests.log
  timeout -k 10 300 python bench.py --model effnetv2 --steps 20 --warmup 5 --cpu-seconds 0 --secondary=serial > gpurun_out/graph_bench.json 2> gpurun_out/graph_bench.err || { tail -20 gpurun_out/graph_bench.err; exit 2; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/graphprof -o run -- python3 bench.py --model effnetv2 --steps 20 --warmup 5 --cpu-seconds 0 --secondary= --pipeline 0 --no-parity > gpurun_out/graphp.log 2>&1 || exit 3
  python tools/prof_summary.py gpurun_out/graphprof > gpurun_out/graph_kernel_stats_serial.txt && head -30 gpurun_out/graph_kernel_stats_serial.txt
  ;;
ab)
  NAME=$1
  timeout -k 10 300 $PT tests/test_gpu_cnn.py tests/test_gpu_config_step.py > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
  bash tools/ab.sh ${2:-3} main tools/ablib/libaa_$NAME.so
  ;;
*)
  echo "unknown mode $MODE"; exit 64 ;;
esac
