"""Build tools/ablib/libaa_NAME.so from the sources as they are at a git revision
(default HEAD), for an in-pipeline A/B of uncommitted kernel changes against
the committed ones (tools/ab.sh).  The other objects come from the main build.

usage: python tools/ab_head.py NAME [REV]"""
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "audio-analysis_amd"))
from aa_amd import _build  # noqa: E402


def main(name, rev="HEAD"):
    _build.build()
    tmp = _build.CSRC.parent / "csrc_ab"  # a sibling keeps the relative includes valid
    shutil.rmtree(tmp, ignore_errors=True)
    tmp.mkdir()
    try:
        for f in _build.CSRC.iterdir():
            rel = f.relative_to(ROOT).as_posix()
            src = subprocess.run(["git", "show", f"{rev}:{rel}"], cwd=ROOT, capture_output=True)
            (tmp / f.name).write_bytes(src.stdout if src.returncode == 0 else f.read_bytes())
        out = ROOT / "tools" / "ablib"
        out.mkdir(exist_ok=True)
        cc = _build.hipcc()
        objs = []
        for s in _build.SOURCES:
            obj = out / f"{s.rsplit('.', 1)[0]}_{name}.o"
            subprocess.run([cc, "-O3", "-std=c++17", "-fPIC", f"--offload-arch={_build.ARCH}", f"-I{_build.INCLUDE}",
                            *_build.EXTRA_FLAGS.get(s, []), "-c", str(tmp / s), "-o", str(obj)], check=True)
            objs.append(obj)
        lib = out / f"libaa_{name}.so"
        subprocess.run([cc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(lib)],
                       check=True)
        for o in objs:
            o.unlink()
        print(lib)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
