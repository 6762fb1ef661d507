"""Per-basic-block instruction mix of one kernel in a hipcc -S listing.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude --cuda-device-only -S \
        audio-analysis_amd/csrc/aa_cnn.hip -o /tmp/aa_cnn.s
    python tools/isa_stats.py /tmp/aa_cnn.s <mangled-name-substring> [--dump BB]

Counts per block: VALU (v_* other than MFMA), MFMA, LDS (ds_*), VMEM
(buffer_/global_), SALU (s_* other than waitcnt/branches), waits and barriers;
the branch targets show the loop structure.
"""
import re
import sys


def kernel_lines(path, key):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if start is None and key in l and l.rstrip().endswith(key.split()[-1] if False else l.rstrip()) and re.match(r"^_Z\S*:", l) and key in l.split(":")[0]:
            start = i
            break
    if start is None:
        sys.exit(f"no kernel label containing {key!r}")
    out = []
    for l in lines[start + 1:]:
        if l.startswith("\t.section") or re.match(r"^\.Lfunc_end", l):
            break
        out.append(l)
    return lines[start].split(":")[0], out


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "bar"
    if op.startswith(("s_cbranch", "s_branch")):
        return "br"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, key = sys.argv[1], sys.argv[2]
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    name, body = kernel_lines(path, key)
    print(name)
    blocks, cur, lab = [], [], "entry"
    for l in body:
        s = l.strip()
        if not s or s.startswith((";", ".")) and not re.match(r"^\.LBB\S*:", s):
            continue
        m = re.match(r"^(\.LBB\S*):", s)
        if m:
            blocks.append((lab, cur))
            lab, cur = m.group(1), []
            continue
        cur.append(s.split(";")[0].strip())
    blocks.append((lab, cur))
    cols = ["valu", "mfma", "lds", "vmem", "salu", "wait", "bar", "br"]
    tot = dict.fromkeys(cols, 0)
    print(f"{'block':<16}" + "".join(f"{c:>6}" for c in cols) + "  branches")
    for lab, ins in blocks:
        c = dict.fromkeys(cols, 0)
        for i in ins:
            k = classify(i)
            if k in c:
                c[k] += 1
        for k in cols:
            tot[k] += c[k]
        br = [i for i in ins if classify(i) == "br"]
        print(f"{lab:<16}" + "".join(f"{c[k]:>6}" for k in cols) + "  " + " | ".join(br))
        if dump and lab == dump:
            print("\n".join("    " + i for i in ins))
    print(f"{'total':<16}" + "".join(f"{tot[k]:>6}" for k in cols))


if __name__ == "__main__":
    main()
