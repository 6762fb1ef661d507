#!/bin/bash
# One GPU-box pass: parity tests, PMC traffic of a bench step per precision,
# the kernel-trace summary of the headline, then the bench line (which reads
# the traffic summary).  Everything lands in gpurun_out/ (copy into profiles/).
# usage (through gpurun): bash tools/gpu_round.sh [precision ...]
set -o pipefail
PRECS=${@:-bf16x3}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
# PMC passes on the serial step (per-launch bytes do not depend on the overlap;
# the dispatch order of one step stays that of the stage list)
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
# on the box, give it this pass's (PROFILE_DIR, e.g. profiles/r03; the local
# copy is made from gpurun_out/ afterwards)
if [ -n "$PROFILE_DIR" ]; then
  for P in $PRECS; do
    cp gpurun_out/pmc_traffic_$P.json "$PROFILE_DIR/" && cp gpurun_out/stats_serial_$P/run_kernel_stats.csv "$PROFILE_DIR/bench_kernel_stats_serial_$P.csv" || exit 9
  done
fi
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { cat gpurun_out/bench.err; exit 7; }
cat gpurun_out/kernel_stats_serial_bf16x3.txt
tail -1 gpurun_out/bench.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 8; }
tail -2 gpurun_out/smoke.log
