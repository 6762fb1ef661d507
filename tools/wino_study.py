"""Numerics study: Winograd F(m, 3) along W for model1's 9x3 conv in split-bf16.

conv_wg runs the 9x3 layer as F(2, 3) along W (2/3 of the direct MFMA work).
F(3, 3) would take 5/9 (and its output triples are exactly the 3x3 pool's
column windows), F(4, 3) 1/2 -- at the price of larger transform
coefficients.  This study emulates the split-bf16 arithmetic of the GPU on the
CPU (operands rounded to bf16 hi + lo, products hi.hi + lo.hi + hi.lo summed
exactly, outputs rounded to f32; BatchNorm folded into the weights as the
planner does) for model1 on the bench's 64 windows, with every conv direct
and with the 9x3 conv through F(2|3|4, 3), and reports max |delta logit|
against float64.

    python tools/wino_study.py [--windows 64]
"""
from __future__ import annotations

import argparse
import sys
import tempfile
from fractions import Fraction
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (str(ROOT), str(ROOT / "audio-analysis_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np
import torch
import torch.nn.functional as F


def toom_cook(m, r=3, points=None):
    """(A^T [m][a], G [a][r], B^T [a][a]) of F(m, r), a = m + r - 1, with the
    given finite points plus infinity, as exact fractions, solved from the
    correlation identity y_i = sum_k g_k d_{i+k}."""
    a = m + r - 1
    pts = [Fraction(p) for p in points][:a - 1]
    AT = [[pts[j] ** i for j in range(a - 1)] + [Fraction(1 if i == m - 1 else 0)] for i in range(m)]
    G = []
    for j in range(a - 1):
        f = Fraction(1)
        for l in range(a - 1):
            if l != j:
                f *= pts[j] - pts[l]
        G.append([pts[j] ** k / f for k in range(r)])
    G.append([Fraction(1 if k == r - 1 else 0) for k in range(r)])
    # B^T column t: solve sum_e AT[i][e] G[e][k] b_e = [i + k == t] for all i, k
    import numpy as np
    M = np.array([[float(AT[i][e] * G[e][k]) for e in range(a)] for i in range(m) for k in range(r)])
    BT = np.zeros((a, a))
    for t in range(a):
        rhs = np.array([1.0 if i + k == t else 0.0 for i in range(m) for k in range(r)])
        sol, res, *_ = np.linalg.lstsq(M, rhs, rcond=None)
        assert np.allclose(M @ sol, rhs, atol=1e-9), (m, t)
        BT[:, t] = sol
    BT = np.array([[float(Fraction(v).limit_denominator(1000)) for v in row] for row in BT])
    return (np.array([[float(v) for v in row] for row in AT]), np.array([[float(v) for v in row] for row in G]), BT)


def split(x):
    """bf16 hi + lo of an f32 tensor (round to nearest even), as f64."""
    x = x.float()
    hi = x.to(torch.bfloat16).float()
    lo = (x - hi).to(torch.bfloat16).float()
    return hi.double(), lo.double()


def conv_split(x, w, b):
    """Direct valid conv, split-bf16 products summed exactly, f32 out."""
    xh, xl = split(x)
    wh, wl = split(w)
    y = F.conv2d(xh, wh) + F.conv2d(xh, wl) + F.conv2d(xl, wh)
    return (y + b[None, :, None, None]).float().double()


def conv_wino(x, w, b, m, pts, presplit=False):
    """The kh x 3 valid conv through F(m, 3) along W: input transform in f32,
    weight transform in f64, both split, products exact, output transform in
    f32 (outputs past the last whole group computed on zero columns and cut)."""
    AT, G, BT = toom_cook(m, 3, pts)
    a = m + 2
    N, C, H, W = x.shape
    O, _, kh, kw = w.shape
    Wo = W - 2
    J = -(-Wo // m)
    xp = F.pad(x, (0, J * m + 2 - W))
    # d[:, :, :, j, t] = x[:, :, :, m j + t]
    d = torch.stack([xp[..., m * j:m * j + a] for j in range(J)], dim=3).float()
    if presplit:  # the transform as an MFMA on the bf16 hi + lo of d (products exact, f32 sums)
        dh, dl = split(d)
        U = (torch.einsum("et,nchjt->nechj", torch.from_numpy(BT), dh) +
             torch.einsum("et,nchjt->nechj", torch.from_numpy(BT), dl)).float()
    if not presplit:
        U = torch.einsum("et,nchjt->nechj", torch.from_numpy(BT).float(), d)  # f32 transform
    V = torch.einsum("et,ockt->eock", torch.from_numpy(G), w)  # f64
    M = []
    for e in range(a):
        uh, ul = split(U[:, e])
        vh, vl = split(V[e][..., None])
        M.append((F.conv2d(uh, vh) + F.conv2d(uh, vl) + F.conv2d(ul, vh)).float())  # [N, O, H - kh + 1, J]
    M = torch.stack(M, 0)
    Y = torch.einsum("ie,enohj->nohji", torch.from_numpy(AT).float(), M)  # f32
    y = Y.reshape(N, O, H - kh + 1, J * m)[..., :Wo]
    return (y + b[None, :, None, None].float()).double()


def forward(arch, tensors, x, wino=None):
    """model1 in float64 (wino None and no split) or split-bf16 emulation."""
    t = lambda k: torch.from_numpy(np.asarray(tensors[k])).double()
    h = torch.from_numpy(x).double().permute(0, 3, 1, 2)
    emu = wino is not False
    i = 0
    logits = None
    while i < len(arch):
        ly = arch[i]
        kind = ly["type"]
        if kind == "conv2d":
            w = t(ly["name"] + ".kernel").permute(3, 2, 0, 1)
            b = t(ly["name"] + ".bias") if ly.get("use_bias") else torch.zeros(w.shape[0], dtype=torch.float64)
            if i + 1 < len(arch) and arch[i + 1]["type"] == "batchnorm":  # folded as the planner does
                bn = arch[i + 1]["name"]
                s = t(bn + ".gamma") / torch.sqrt(t(bn + ".moving_variance") + float(arch[i + 1].get("eps", 1e-3)))
                b = (b - t(bn + ".moving_mean")) * s + t(bn + ".beta")
                w = w * s[:, None, None, None]
                i += 1
            if not emu:
                h = F.conv2d(h, w) + b[None, :, None, None]
            elif wino and len(wino) > 2 and wino[2] and tuple(w.shape[2:]) == (9, 3):  # the shipped F(6,3) 9x3
                h = conv_wino(h, w, b, 6, [0, 1, -1, 2, -2, 0.5, -0.5])
            elif wino and (tuple(w.shape[2:]) == (9, 3) or (len(wino) > 2 and wino[2] and tuple(w.shape[1:]) == (32, 3, 3))):
                h = conv_wino(h, w, b, *wino[:2], presplit=len(wino) > 3 and wino[3] and tuple(w.shape[2:]) == (3, 3))
            else:
                h = conv_split(h, w, b)
        elif kind == "leakyrelu":
            h = F.leaky_relu(h, float(ly.get("alpha", 0.3)))
            if emu:
                h = h.float().double()
        elif kind == "maxpool2d":
            h = F.max_pool2d(h, ly["pool"], ly["pool"])
        elif kind == "globalmaxpool2d":
            h = torch.amax(h, dim=(2, 3))
            logits = h
        i += 1
    return logits.numpy()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=64)
    ap.add_argument("--calib", action="store_true", help="the GPU tests' dB-like inputs (make_models.calibration_input)")
    ap.add_argument("--first", action="store_true", help="Winograd variants on the 3x3/32 pooled conv (with F(6,3) 9x3)")
    args = ap.parse_args(argv)
    import bench
    from oracle import cnn_oracle, fe_oracle
    from tools.make_models import make_model
    fe_s = bench.fe_settings()
    cfg = bench.fe_config(fe_s)
    pcm, _, views = bench.make_batch(0, fe_s)
    x = np.stack([fe_oracle.window_logmel(bench.window_samples(pcm, v, cfg["win_len"]), cfg)
                  for v in views[:args.windows]]).astype(np.float32)
    if args.calib:
        from tools.make_models import calibration_input
        x = calibration_input(6, 160, 226, True, np.random.default_rng(226 + 6))
    print(f"input {x.shape} mean {x.mean():.2f} std {x.std():.2f}")
    torch.set_num_threads(8)
    p = make_model(Path(tempfile.mkdtemp()) / "model1", "model1", seed=1)
    arch, tensors = cnn_oracle.load_arch(p)
    ref = forward(arch, tensors, x, wino=False)
    print(f"logits {ref.min():.3f} .. {ref.max():.3f}")
    variants = [("F(6,3) 9x3 + 3x3/32 presplit", (6, [0, 1, -1, 2, -2, 0.5, -0.5], True, True)),
                       ("F(6,3) 9x3 + 3x3/32", (6, [0, 1, -1, 2, -2, 0.5, -0.5], True)),
                       ("F(6,3) 9x3 only", (6, [0, 1, -1, 2, -2, 0.5, -0.5])),
                       ("direct split-bf16", None), ("F(2,3) {0,1,-1}", (2, [0, 1, -1])),
                       ("F(3,3) {0,1,-1,2}", (3, [0, 1, -1, 2])), ("F(3,3) {0,1,-1,1/2}", (3, [0, 1, -1, 0.5])),
                       ("F(4,3) {0,1,-1,2,-2}", (4, [0, 1, -1, 2, -2])),
                       ("F(4,3) {0,1,-1,1/2,-1/2}", (4, [0, 1, -1, 0.5, -0.5]))]
    if args.first:
        variants = [("direct split-bf16", None)] + [
            (f"3x3/32 F({m},3) {pts}", (m, pts, True, True)) for m, pts in
            [(2, [0, 1, -1]), (3, [0, 1, -1, 0.5]), (3, [0, 1, -1, 2]), (4, [0, 1, -1, 0.5, -0.5]), (4, [0, 1, -1, 2, -2]),
             (6, [0, 1, -1, 2, -2, 0.5, -0.5])]]
    for name, wino in variants:
        lg = forward(arch, tensors, x, wino=wino)
        print(f"{name:28s} max|dlogit| {np.abs(lg - ref).max():.3e}  mean {np.abs(lg - ref).mean():.3e}", flush=True)


if __name__ == "__main__":
    main()
