"""Print register use and the innermost MFMA loop of kernels in a gfx950 .s file.

Usage: python tools/isa_loop.py FILE.s NAME_SUBSTRING [--body]
(make FILE.s with: hipcc -S --cuda-device-only --offload-arch=gfx950 -O3
 -std=c++17 -I include audio-analysis_amd/csrc/aa_cnn.hip -o FILE.s)
"""
import re
import sys
from collections import Counter


def main():
    path, key = sys.argv[1], sys.argv[2]
    body = "--body" in sys.argv
    s = open(path).read()
    names = [n for n in re.findall(r"^(_Z\S+):", s, re.M) if key in n]
    meta = {}
    for m in re.finditer(r"\.name:\s+(\S+)(.*?)(?=\n  - |\n\.end_amdgpu_metadata)", s, re.S):
        meta[m.group(1)] = m.group(2)
    for name in names:
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        lines = s[i:j].split("\n")
        md = meta.get(name, "")
        regs = {k: re.search(r"\." + k + r":\s+(\d+)", md) for k in
                ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "private_segment_fixed_size")}
        print(name)
        print("  " + " ".join(f"{k}={v.group(1)}" for k, v in regs.items() if v))
        # loops: label with 'Loop Header' ... the backward branch to it
        heads = [(n, l.split(":")[0]) for n, l in enumerate(lines) if "Loop Header" in l]
        for n0, lab in heads:
            n1 = next((n for n in range(n0 + 1, len(lines)) if re.search(r"s_cbranch\w*\s+" + re.escape(lab) + r"\b", lines[n])), None)
            if n1 is None:
                continue
            c = Counter()
            for l in lines[n0:n1 + 1]:
                t = l.strip().split(" ")[0]
                if t and not t.startswith((";", ".")):
                    c[t] += 1
            if not any(k.startswith("v_mfma") for k in c):
                continue
            tot = sum(c.values())
            print(f"  loop {lab} lines {n0}-{n1}: {tot} instr  " + ", ".join(f"{k}:{v}" for k, v in c.most_common(12)))
            if body:
                print("\n".join(lines[n0:n1 + 1]))


if __name__ == "__main__":
    main()
