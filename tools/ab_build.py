"""Build variant libaa.so files that differ only in the split-bf16 tile table
(AA_X3_CFGS), for in-pipeline A/B timing on one GPU box (tools/ab.sh):
kernel times differ by +-5-25 % between boxes and with the data's toggle
rate (the MI355X runs power-limited), so tile choices are compared in the
real pipeline, alternating runs on the same box.

usage: python tools/ab_build.py NAME X3TABLE WGTABLE [NAME X3TABLE WGTABLE ...]
  X3TABLE / WGTABLE: 'X(...) X(...) ...' for AA_X3_CFGS / AA_WG_CFGS, '-' keeps
  the in-tree table, '' an empty one
writes tools/ablib/libaa_NAME.so (the other objects come from the main build)."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "audio-analysis_amd"))
from aa_amd import _build  # noqa: E402


def build(name, table, wg="-"):
    _build.build()
    out = ROOT / "tools" / "ablib"
    out.mkdir(exist_ok=True)
    cc = _build.hipcc()
    obj = out / f"aa_cnn_{name}.o"
    cmd = [cc, "-O3", "-std=c++17", "-fPIC", f"--offload-arch={_build.ARCH}", f"-I{_build.INCLUDE}",
           *([f"-DAA_X3_ALT(X)={table}"] if table != "-" else []),
           *([f"-DAA_WG_ALT(X)={wg}"] if wg != "-" else []),
           *_build.EXTRA_FLAGS.get("aa_cnn.hip", []),
           *os.environ.get("AB_DEFS", "").split(), "-c", str(_build.CSRC / "aa_cnn.hip"), "-o", str(obj)]
    subprocess.run(cmd, check=True)
    objs = [_build.PKG.parent / "build" / (s.rsplit(".", 1)[0] + ".o") for s in _build.SOURCES
            if s != "aa_cnn.hip" and not (s == "aa_frontend.hip" and os.environ.get("AB_FE_DEFS"))]
    if os.environ.get("AB_FE_DEFS"):  # a front-end variant too
        fo = out / f"aa_frontend_{name}.o"
        subprocess.run([cc, "-O3", "-std=c++17", "-fPIC", f"--offload-arch={_build.ARCH}", f"-I{_build.INCLUDE}",
                        *_build.EXTRA_FLAGS.get("aa_frontend.hip", []), *os.environ["AB_FE_DEFS"].split(), "-c",
                        str(_build.CSRC / "aa_frontend.hip"), "-o", str(fo)], check=True)
        objs.append(fo)
    lib = out / f"libaa_{name}.so"
    subprocess.run([cc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", str(obj), *map(str, objs), "-o",
                    str(lib)], check=True)
    obj.unlink()
    print(lib)


if __name__ == "__main__":
    a = sys.argv[1:]
    for i in range(0, len(a), 3):
        build(a[i], a[i + 1], a[i + 2])
