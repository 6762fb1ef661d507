import cProfile, pstats, sys, tempfile, time
from pathlib import Path
sys.path.insert(0, "audio-analysis_amd"); sys.path.insert(0, ".")
import torch
from aa_amd import corpus
from tools import synth
from tools.make_models import make_model
root = Path(tempfile.mkdtemp())
model = make_model(root / "model1", "model1", seed=1)
files = []
for i in range(16):
    p = root / f"c{i}.wav"; synth.write_wav(p, synth.clip(5000 + i)); files.append(p)
corpus.run([files[0]], [str(model)])
torch.cuda.synchronize()
pr = cProfile.Profile(); pr.enable()
t0 = time.perf_counter(); corpus.run(files, [str(model)]); torch.cuda.synchronize(); dt = time.perf_counter() - t0
pr.disable()
print("per file ms", 1e3 * dt / len(files))
pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
