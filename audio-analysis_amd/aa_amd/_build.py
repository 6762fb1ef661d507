"""Build libaa.so in-tree with hipcc for gfx950 (no torch extension machinery:
the library is a plain C-ABI shared object loaded with ctypes)."""
from __future__ import annotations

import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG.parent / "csrc"
INCLUDE = PKG.parent.parent / "include"
LIB = PKG / "libaa.so"
SOURCES = ["aa_api.cpp", "aa_frontend.hip", "aa_cnn.hip", "aa_scan.hip", "aa_signal.hip", "aa_flac.cpp",
           "aa_vorbis.cpp", "aa_tracks.cpp", "aa_resample.hip", "aa_graph.hip"]
ARCH = os.environ.get("AA_OFFLOAD_ARCH", "gfx950")
# per-source flags: the FFT front end is written in scalar f32; SLP packing it
# into v_pk_* ops needs paired SGPR constants and register shuffles that push
# the wave-per-frame kernel past its 128-VGPR budget (spills)
# the CNN kernels keep MFMA accumulators in VGPRs: no AGPR copies
# (v_accvgpr_read) between the fused first layer's MFMAs and its activation
# split (in-pipeline A/B: step +0.5 %); and no SLP packing there either: the
# fused first conv is bound by the SIMD's vector issue (VALU issue + the 8
# cycles each MFMA holds it, profiles/r06/pmc_fused_first_conv.txt), and the
# packed v_pk_add_f32 the vectoriser formed in the activation split costs
# more issue than two scalar subtracts (fused conv 127 -> 120 us, step
# 270.8k -> 275.4k audio-s/s, profiles/r06/ab_slp.txt)
EXTRA_FLAGS = {"aa_frontend.hip": ["-fno-slp-vectorize"], "aa_signal.hip": ["-fno-slp-vectorize"],
               "aa_cnn.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-slp-vectorize"],
               # same for the graph route: the split-bf16 1x1 / expand convs are
               # VALU-issue-bound too (effnetv2 step 61.0k -> 62.5k audio-s/s,
               # profiles/r06/ab_graph_noslp.txt)
               "aa_graph.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-slp-vectorize"]}


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libaa.so)")


def _stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    # this file too: a change of the per-source flags rebuilds
    deps = [CSRC / s for s in SOURCES] + list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h")) + [Path(__file__)]
    return any(p.stat().st_mtime > t for p in deps)


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not _stale():
        return LIB
    cc = hipcc()
    objdir = PKG.parent / "build"
    objdir.mkdir(exist_ok=True)
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INCLUDE}",
             "-Wall", "-Wno-unused-function"]

    def compile_one(src: str) -> Path:
        obj = objdir / (src.rsplit(".", 1)[0] + ".o")
        cmd = [cc, *flags, *EXTRA_FLAGS.get(src, []), "-c", str(CSRC / src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1, 16)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
