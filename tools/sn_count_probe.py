import sys, time
sys.path[:0] = ["/root/repo", "/root/repo/audio-analysis_amd"]
import numpy as np, torch
from tools import synth
from aa_amd.signals import SignalDetector
from aa_amd.identify_tracks import Signal, get_tracks_from_signals
dev = torch.device("cuda", 0)
det = SignalDetector(48000, 281, dev)
cs = []
sigs_all = []
for i in range(16):
    x = synth.clip(5000 + i)
    stats = det.components(torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(dev))
    cs.append(len(stats))
    sigs_all.append([Signal(*t) for t in det.to_tuples(stats)])
print("components per clip:", cs)
t0 = time.perf_counter()
nt = 0
for rep in range(20):
    for sg in sigs_all:
        nt += len(get_tracks_from_signals([s.copy() for s in sg], 60.0))
t1 = time.perf_counter()
print(f"get_tracks_from_signals: {1e3 * (t1 - t0) / (20 * len(sigs_all)):.3f} ms per clip, {nt / (20 * len(sigs_all)):.1f} tracks")
