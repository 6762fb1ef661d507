#!/bin/bash
# corpus (configs[3]) A/B over HIP hardware queues and host lanes:
#   bash tools/c4_ab.sh ROUNDS "NAME VAR=.. --bench-flag=.." ...
set -o pipefail
mkdir -p gpurun_out
run() { # name [VAR=value ...] [--bench-flag ...]
  local name=$1; shift
  local envs=() flags=()
  for a in "$@"; do case $a in --*) flags+=("$a");; *) envs+=("$a");; esac; done
  env "${envs[@]}" timeout -k 10 240 python -u bench.py --config 4 --cpu-seconds 0 --no-parity "${flags[@]}" > gpurun_out/c4ab_$name.log 2>&1 || { tail -5 gpurun_out/c4ab_$name.log; return 1; }
  python - "$name" <<'PY'
import json, sys
line = [l for l in open(f"gpurun_out/c4ab_{sys.argv[1]}.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[1]:24s} {d['value']:9.1f}", flush=True)
PY
}
R=$1; shift
for r in $(seq 1 $R); do
  for spec in "$@"; do
    run $spec || exit 1
  done
done
