#!/bin/bash
# Graph-executor A/B on one GPU box: alternating EfficientNetV2-shaped bench
# runs under environment variants (kernel-choice knobs read at run time).
# usage (through gpurun): bash tools/graph_ab.sh ROUNDS "ENV=.. ENV2=.." "..." ...   ("-": no variables)
set -o pipefail
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for V in "$@"; do
    [ "$V" = "-" ] && V=""
    env $V timeout -k 10 200 python bench.py --model effnetv2 --steps 20 --warmup 5 --cpu-seconds 0 --secondary= --no-parity > gpurun_out/gab.log 2>&1 || { tail -5 gpurun_out/gab.log; exit 1; }
    python - "${V:--}" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/gab.log").read().strip().splitlines()[-1])
d = json.load(open("gpurun_out/bench_full.json")) if "stages_ms" not in d["roofline"] else d  # (the printed line is compact)
import re
g = {}
for k, v in d["roofline"]["stages_ms"].items():
    m = re.match(r"(dwconv|matvec|conv_gx3_1x1|conv_gx3_3x3|conv_gf32|fe_)", k)
    key = m.group(1) if m else "other"
    g[key] = g.get(key, 0.0) + v
print(f"{sys.argv[1]:28s} {d['value']:9.1f} sum={1e3 * d['roofline']['stages_sum_ms']:7.1f}us  " + " ".join(f"{k}={1e3*v:.0f}" for k, v in sorted(g.items())), flush=True)
st = d["roofline"]["stages_ms"]
pick = ["conv_gx3_1x1_s1_112_672", "conv_gx3_1x1_s1_672_112+add+se", "conv_gx3_1x1_s1_192_1152", "conv_gx3_1x1_s1_1152_192+add+se",
        "conv_gx3_1x1_s1_96_384", "conv_gx3_1x1_s1_384_96+add+se", "conv_gx3_1x1_s1_672_192+se", "conv_gx3_1x1_s1_192_1280"]
print(" " * 30 + " ".join(f"{k[13:]}={1e3 * st[k]:.1f}" for k in pick if k in st), flush=True)
PY
  done
done
