"""CPU checks of the fp8 emulation the GPU fp8 test compares against
(oracle.cnn_oracle.forward_fp8_emulated)."""
import numpy as np
import torch

from oracle import cnn_oracle
from tools.make_models import calibration_input


def test_e4m3fn_known_values():
    x = torch.tensor([0.0, 1.0, 1.0625, 1.1875, 448.0, 500.0, -1e4, 2.0 ** -9, 2.0 ** -10, 0.3])
    got = cnn_oracle._fp8(x).tolist()
    # 1.0625 is halfway between 1 and 1.125: ties to even -> 1.0; 1.1875 -> 1.25;
    # beyond 448 saturates; 2^-9 is the smallest subnormal, 2^-10 ties to 0
    assert got[:9] == [0.0, 1.0, 1.0, 1.25, 448.0, 448.0, -448.0, 2.0 ** -9, 0.0]
    assert abs(got[9] - 0.3) <= 0.3 * 2 ** -4


def test_fp8_emulation_close_to_f32(model_root):
    path = model_root / "model1" / "audioModel.safetensors"
    x = calibration_input(2, 160, 226, True, np.random.default_rng(3))
    el, ep = cnn_oracle.forward_fp8_emulated(path, x)
    fl, _ = cnn_oracle.forward_fp8_emulated(path, x, mfma=False)
    assert np.abs(el - fl).max() < 0.5  # the MFMA sums vs torch's f32 conv: truncation-sized
    rl, rp = cnn_oracle.forward(path, x)
    assert np.isfinite(el).all()
    # e4m3 activations: a 3-bit mantissa through six layers
    assert np.abs(el - rl).max() < 1.5
    assert np.abs(ep - rp).max() < 0.3
