"""fp8 CNN on the GPU against both CPU emulations (oracle.cnn_oracle.
forward_fp8_emulated with mfma=True: the fp8 MFMAs' grouped truncating sums;
mfma=False: torch's f32 conv), whole networks and the per-kernel chains:
max / mean |delta logit| and the share of bit-equal logits (through gpurun)."""
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "audio-analysis_amd")]

import numpy as np
import torch

from oracle import cnn_oracle
from tools.make_models import calibration_input, make_chain, make_ensemble, make_model


def run(path, x):
    from aa_amd.model import Model
    m = Model(path, x.shape[1:], precision="fp8")
    lg, _ = m.forward(torch.from_numpy(x).cuda())
    torch.cuda.synchronize()
    return lg.cpu().numpy()


def main():
    root = Path(tempfile.mkdtemp())
    make_ensemble(root)
    m = lambda k: root / k / "audioModel.safetensors"
    cases = [("model1 T226", m("model1"), calibration_input(3, 160, 226, True, np.random.default_rng(3)), True),
             ("model2 T226", m("model2"), calibration_input(2, 160, 226, True, np.random.default_rng(7)), True),
             ("mag T226", make_model(root / "mag", "magmodel", seed=11, mag=2), calibration_input(2, 160, 226, False, np.random.default_rng(6)), True)]
    chains = {"3x3_64_k128": [(32, (3, 3), None), (64, (3, 3), None), (64, (3, 3), None)],
              "9x3_64_k128": [(32, (3, 3), None), (64, (3, 3), None), (128, (9, 3), (3, 3))],
              "1x3_128_k128": [(32, (3, 3), None), (128, (3, 3), None), (256, (1, 3), None)]}
    for k, spec in chains.items():
        cases.append((k, make_chain(root / k, spec, seed=5), calibration_input(3, 160, 226, True, np.random.default_rng(8)), False))
    for name, path, x, first_bf16 in cases:
        lg = run(path, x)
        for mfma in (False, True):
            t = time.time()
            el, _ = cnn_oracle.forward_fp8_emulated(path, x, first_bf16=first_bf16, mfma=mfma)
            d = np.abs(lg - el)
            print(f"{name:14s} mfma={int(mfma)}: max {d.max():.4f} mean {d.mean():.5f} bit-equal {100 * (lg == el).mean():.1f} % "
                  f"({time.time() - t:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
