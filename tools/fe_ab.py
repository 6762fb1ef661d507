"""Front end of the working-tree library against another build (AA_LIB, e.g.
tools/ablib/libaa_base.so from tools/ab_head.py): the log-mel of the bench's
64 windows (htk / hop 640 and Slaney / hop 281 plans, power 2 and 1) must be
bit-identical.

usage: python tools/fe_ab.py OUT.npz ; python tools/fe_ab.py --compare A.npz B.npz"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "audio-analysis_amd")]

import numpy as np


def run(out):
    import torch
    import bench
    from aa_amd.frontend import FeSettings, FrontEnd
    dev = torch.device("cuda")
    res = {}
    pcm, rows, _ = bench.make_batch(0, bench.fe_settings())
    for name, s in {"htk640_p2": bench.fe_settings(),
                    "htk640_p1": FeSettings(htk=True, hop_length=640, n_fft=4096, n_mels=160, break_freq=1750, power=1),
                    "htk640_p15": FeSettings(htk=True, hop_length=640, n_fft=4096, n_mels=160, break_freq=1750, power=1.5),
                    "slaney281": FeSettings(htk=False, hop_length=281, n_fft=4096, n_mels=160)}.items():
        fe = FrontEnd(s, dev)
        lm = fe.run(torch.from_numpy(pcm).to(dev), torch.from_numpy(rows).to(dev))
        res[name] = lm.cpu().numpy()
    np.savez(out, **res)
    print(f"{out}: {', '.join(res)}")


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if not np.array_equal(A[k], B[k])]
    for k in bad:
        print(f"{k}: max |d| {np.abs(A[k] - B[k]).max():.3e}, {np.mean(A[k] != B[k]) * 100:.4f} % differ")
    print(f"{len(A.files) - len(bad)} of {len(A.files)} log-mel tensors bit-identical")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    run(sys.argv[1])
