"""Diagnostic: the fused first-layer pair (conv_wgf vs conv_x3, AA_WGF=1/0)
through aa_model on calibrated networks against the oracle: model1 and a
two-conv chain (3x3 1->32, 3x3 32->32 + pool 3, GlobalMaxPool2D), whose
"logits" are the pooled maxima of the pair's own output.

    python tools/wgf_model_check.py        (GPU box; runs each AA_WGF in a child)
"""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (str(ROOT), str(ROOT / "audio-analysis_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def child(tmp):
    import numpy as np
    import torch
    from aa_amd.model import Model
    from oracle import cnn_oracle
    from tools.make_models import calibration_input, make_chain, make_model
    tmp = Path(tmp)
    for name in ("chain", "model1"):
        p = tmp / name / "audioModel.safetensors"
        if not p.exists():
            if name == "chain":
                make_chain(tmp / name, [(32, (3, 3), None), (32, (3, 3), (3, 3))])
            else:
                make_model(tmp / name, "model1", seed=1)
        x = calibration_input(6, 160, 226, True, np.random.default_rng(232))
        m = Model(p, x.shape[1:], precision="bf16x3")
        lg, _ = m.forward(torch.from_numpy(x).cuda())
        torch.cuda.synchronize()
        lg = lg.cpu().numpy()
        ref, _ = cnn_oracle.forward(p, x)
        d = np.abs(lg - ref)
        print(f"AA_WGF={os.environ.get('AA_WGF', '1')} {name}: max|d| {d.max():.3e} (ref {ref.min():.2f}..{ref.max():.2f}); "
              f"worst logits by window {d.max(axis=1).round(4).tolist()}", flush=True)


def dump(out):
    """The chain's BN-folded pair and the check input as raw f32 for tools/wgf_check (WGF_DATA)."""
    import numpy as np
    from oracle import cnn_oracle
    from tools.make_models import calibration_input, make_chain
    out = Path(out)
    p = make_chain(out / "chain", [(32, (3, 3), None), (32, (3, 3), (3, 3))])
    arch, t = cnn_oracle.load_arch(p)
    folded = []
    for i, ly in enumerate(arch):
        if ly["type"] != "conv2d":
            continue
        w = np.asarray(t[ly["name"] + ".kernel"], np.float64)  # [kh][kw][cin][cout]
        b = np.asarray(t[ly["name"] + ".bias"], np.float64) if ly.get("use_bias") else np.zeros(w.shape[-1])
        bn = arch[i + 1]
        s = np.asarray(t[bn["name"] + ".gamma"], np.float64) / np.sqrt(np.asarray(t[bn["name"] + ".moving_variance"], np.float64) + float(bn.get("eps", 1e-3)))
        b = (b - np.asarray(t[bn["name"] + ".moving_mean"], np.float64)) * s + np.asarray(t[bn["name"] + ".beta"], np.float64)
        folded.append((w * s, b))
    (w1, b1), (w2, b2) = folded
    x = calibration_input(6, 160, 226, True, np.random.default_rng(232))
    np.ascontiguousarray(x[..., 0], np.float32).tofile(out / "x.bin")
    np.ascontiguousarray(w1.reshape(9, 32).T, np.float32).tofile(out / "w1.bin")  # [cout][tap]
    b1.astype(np.float32).tofile(out / "b1.bin")
    np.ascontiguousarray(w2.reshape(9, 32, 32), np.float32).tofile(out / "k2.bin")  # [tap][cin][cout]
    b2.astype(np.float32).tofile(out / "b2.bin")
    print("folded |w1| max", np.abs(w1).max(), "|b1| max", np.abs(b1).max(), "|w2| max", np.abs(w2).max(), "|b2| max", np.abs(b2).max())


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--dump":
        dump(sys.argv[2])
    elif len(sys.argv) > 1:
        child(sys.argv[1])
    else:
        tmp = tempfile.mkdtemp()
        for v in ("0", "1"):
            env = dict(os.environ, AA_WGF=v)
            subprocess.run([sys.executable, __file__, tmp], env=env, check=True)
