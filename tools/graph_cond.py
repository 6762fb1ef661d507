"""Conditioning probe of the effnetv2 bench network.

The first ``bench.py --model effnetv2`` run failed its own gate with
max|dlogit| = 2.0e3 on a network whose BatchNorm statistics came from the
synthetic dB-like calibration input (make_graph without ``calib``, seed 5,
T = 513, 3 channels).  This probe takes that network and the bench's own 64
windows and separates the three possible sources of such a delta:

* the input: GPU front end vs oracle front end (<= 1e-3 dB) pushed through the
  network (oracle float64 on both log-mels);
* the network's own conditioning: oracle float32 vs oracle float64 on the same
  input, and oracle float64 under a relative input perturbation of 2^-17 (the
  size of a split-bf16 operand's representation error);
* the GPU kernels: GPU f32 and GPU split-bf16 vs oracle float64 on the SAME
  log-mel (the oracle's), per block output (arch prefixes ending at each
  block, compared relative to the block output's scale) and at the logits.

A kernel bug shows as a GPU error far above the oracle-f32 / perturbation
errors at the same point; conditioning shows as all of them growing together
(profiles/r05/graph_cond_*.json: the uncalibrated network's own float32
evaluation is 387 logits away from float64).  tests/test_gpu_graph.py uses
the same functions.

    python tools/graph_cond.py [--windows 64] [--calibrated] [--prefix]
"""
from __future__ import annotations

import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (str(ROOT), str(ROOT / "audio-analysis_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np
import torch


def rel_err(a, b):
    """max |a - b| / max |b|."""
    return float(np.abs(a - b).max()) / max(float(np.abs(b).max()), 1e-30)


def bench_network(out_dir, calibrated):
    """The effnetv2 network of bench.py (calibrated on another seed's log-mels)
    or the uncalibrated one its first run failed on."""
    import bench
    from oracle import fe_oracle
    from tools.make_models import make_graph
    fe_s = bench.fe_settings("effnetv2")
    calib = None
    if calibrated:
        cfg = bench.fe_config(fe_s)
        cal_pcm, _, cal_views = bench.make_batch(1000, fe_s)
        calib = np.stack([fe_oracle.window_logmel(bench.window_samples(cal_pcm, v, cfg["win_len"]), cfg)
                          for v in cal_views[::len(cal_views) // 3][:3]])
    return make_graph(Path(out_dir) / "effnetv2", "effnetv2", in_channels=3, T=fe_s.n_frames, seed=5, calib=calib)


def bench_logmels(n_windows=64):
    """(oracle log-mels [W][160][513][3] f32, pcm, window rows, selected indices)
    of the bench's first batch (rank 0), ``n_windows`` spread over its 64."""
    import bench
    from oracle import fe_oracle
    fe_s = bench.fe_settings("effnetv2")
    cfg = bench.fe_config(fe_s)
    pcm, rows, views = bench.make_batch(0, fe_s)
    sel = np.linspace(0, len(views) - 1, n_windows).round().astype(int)
    x = np.stack([fe_oracle.window_logmel(bench.window_samples(pcm, views[i], cfg["win_len"]), cfg)
                  for i in sel]).astype(np.float32)
    return x, pcm, rows, sel


def block_ends(arch):
    """Indices of the last layer of the stem, of every block and of the head."""
    ends = []
    for i, ly in enumerate(arch):
        nxt = arch[i + 1]["name"] if i + 1 < len(arch) else ""
        if ly["type"] in ("dense", "globalavgpool2d"):
            continue
        if nxt.split("_")[0] != ly["name"].split("_")[0]:
            ends.append(i)
    return ends


def prefix_model(out_dir, arch, tensors, i, meta):
    """arch[:i + 1] as its own model file (the graph's output = that layer's
    NHWC activations per window)."""
    from safetensors.numpy import save_file
    sub = arch[:i + 1]
    names = {ly["name"] for ly in sub}
    used = {k: np.ascontiguousarray(v) for k, v in tensors.items() if k.rsplit(".", 1)[0] in names}
    d = Path(out_dir) / f"prefix_{i}"
    d.mkdir(parents=True, exist_ok=True)
    save_file(used, str(d / "audioModel.safetensors"), metadata={"arch": json.dumps(sub)})
    (d / "metadata.txt").write_text(json.dumps(meta))
    return d / "audioModel.safetensors"


def prefix_errors(mpath, x, dev, tmp, ends=None):
    """Per block end: relative errors (to the float64 oracle, scaled by the
    block output's max) of the float32 oracle, GPU f32 and GPU split-bf16."""
    from aa_amd.model import Model
    from oracle import cnn_oracle
    arch, tensors = cnn_oracle.load_arch(mpath)
    meta = json.loads((Path(mpath).parent / "metadata.txt").read_text())
    cap64, cap32 = {}, {}
    cnn_oracle._forward_graph(arch, tensors, torch.from_numpy(x).double().permute(0, 3, 1, 2), torch.float64,
                              capture=cap64)
    cnn_oracle._forward_graph(arch, tensors, torch.from_numpy(x).float().permute(0, 3, 1, 2), torch.float32,
                              capture=cap32)
    P = x.shape[0]
    rows = []
    for i in (ends if ends is not None else block_ends(arch)):
        name = arch[i]["name"]
        p = prefix_model(tmp, arch, tensors, i, meta)
        r64 = cap64[name].permute(0, 2, 3, 1).reshape(P, -1).numpy()
        r32 = cap32[name].permute(0, 2, 3, 1).reshape(P, -1).numpy()
        row = {"block_end": name, "scale": float(np.abs(r64).max()), "oracle_f32": rel_err(r32, r64)}
        for prec in ("f32", "bf16x3"):
            m = Model(p, x.shape[1:], precision=prec, device=dev, meta=meta)
            out = m.forward(torch.from_numpy(x).to(dev))[0].cpu().numpy()
            row[f"gpu_{prec}"] = rel_err(out, r64)
            del m
        rows.append(row)
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=64)
    ap.add_argument("--prefix-windows", type=int, default=4)
    ap.add_argument("--calibrated", action="store_true", help="the bench's calibrated network instead")
    ap.add_argument("--prefix", action="store_true", help="per-block comparisons through arch prefixes")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)

    import bench
    from aa_amd.frontend import FrontEnd
    from aa_amd.model import Model
    from oracle import cnn_oracle

    tmp = Path(tempfile.mkdtemp(prefix="aa_cond_"))
    t0 = time.time()
    mpath = bench_network(tmp, args.calibrated)
    print(f"network built ({'calibrated' if args.calibrated else 'uncalibrated'}) in {time.time() - t0:.1f} s",
          flush=True)
    x_ora, pcm, rows, sel = bench_logmels(args.windows)
    dev = torch.device("cuda:0")
    fe = FrontEnd(bench.fe_settings("effnetv2"), dev)
    x_gpu = fe.run(torch.from_numpy(pcm).to(dev), torch.from_numpy(rows).to(dev)).cpu().numpy()[sel]
    res = {"network": "calibrated" if args.calibrated else "uncalibrated", "windows": args.windows,
           "logmel_max_abs_db": float(np.abs(x_gpu - x_ora).max())}
    arch, tensors = cnn_oracle.load_arch(mpath)
    f64 = lambda x: cnn_oracle.forward(arch, x, dtype=torch.float64, tensors=tensors)[0]
    ref = f64(x_ora)
    res["logit_range"] = [float(ref.min()), float(ref.max())]
    rng = np.random.default_rng(0)
    pert = x_ora.astype(np.float64) * (1 + 2.0 ** -17 * rng.choice([-1.0, 1.0], x_ora.shape))
    res["oracle_f64_gpu_logmel"] = float(np.abs(f64(x_gpu) - ref).max())
    res["oracle_f64_perturbed_2^-17"] = float(np.abs(f64(pert) - ref).max())
    res["oracle_f32"] = float(np.abs(cnn_oracle.forward(arch, x_ora, tensors=tensors)[0] - ref).max())
    for prec in ("f32", "bf16x3"):
        m = Model(mpath, x_ora.shape[1:], precision=prec, device=dev)
        lg = m.forward(torch.from_numpy(x_ora).to(dev))[0].cpu().numpy()
        res[f"gpu_{prec}_oracle_logmel"] = float(np.abs(lg - ref).max())
        lg2 = m.forward(torch.from_numpy(x_gpu).to(dev))[0].cpu().numpy()
        res[f"gpu_{prec}_gpu_logmel"] = float(np.abs(lg2 - ref).max())
        del m
    print(json.dumps(res, indent=1), flush=True)
    if args.prefix:
        res["prefix"] = prefix_errors(mpath, x_ora[:args.prefix_windows], dev, tmp)
        for row in res["prefix"]:
            print(f"{row['block_end']:28s} scale {row['scale']:10.3e}  rel err: oracle f32 {row['oracle_f32']:.2e}  "
                  f"gpu f32 {row['gpu_f32']:.2e}  gpu bf16x3 {row['gpu_bf16x3']:.2e}", flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
