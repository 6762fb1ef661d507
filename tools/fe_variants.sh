#!/bin/bash
# Alternating runs of fe_bench variant binaries (tools/fe_bench_*), the full
# kernel only, with a hash of each variant's mel output:
#   bash tools/fe_variants.sh ROUNDS tools/fe_bench_a tools/fe_bench_b ...
set -o pipefail
R=$1; shift
for r in $(seq 1 $R); do
  for B in "$@"; do
    out=$(timeout -k 5 60 $B pmc 2>&1) || { echo "$B failed: $out"; exit 1; }
    echo "$(basename $B) $(echo "$out" | grep -E 'DIAG|hash' | tr '\n' ' ')"
  done
done
