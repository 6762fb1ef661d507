"""Host issue time of the bench step (two streams) against its wall time:
whether the Python/ctypes launches keep ahead of the GPU (through gpurun:
`python tools/issue_probe.py`)."""
import sys, time, tempfile
from pathlib import Path
sys.path[:0] = ["/root/repo", "/root/repo/audio-analysis_amd"]
import torch, bench
from tools.make_models import make_model
dev = torch.device("cuda")
tmp = tempfile.mkdtemp()
mp = make_model(Path(tmp) / "model1", "model1", seed=1)
first = bench.make_batch(0, bench.fe_settings())
st = bench.Step(dev, 0, mp, "bf16x3", pairs=bench.HEAD_PAIRS, first=first, pipeline=2)
for _ in range(20): st()
torch.cuda.synchronize()
for n in (50, 200):
    t0 = time.perf_counter()
    for _ in range(n): st()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"n={n}: issue {1e3*(t1-t0)/n:.3f} ms/step, total {1e3*(t2-t0)/n:.3f} ms/step")
