import sys, numpy as np, torch
sys.path[:0] = ['.', 'audio-analysis_amd']
from tests.test_gpu_signal import _clip
from aa_amd.signals import SignalDetector
from oracle.fe_oracle import stft_mag
det = SignalDetector(48000, 281, torch.device('cuda'))
for n, seed in [(60*48000, 30), (7*48000+12345, 32)]:
    x = _clip(n/48000, seed)
    g = det.spectrogram(torch.from_numpy(x).cuda()).cpu().numpy()
    w = stft_mag(x, 4096, 281)
    d = g.view(np.uint32) != w.view(np.uint32)
    bins, frames = np.nonzero(d)
    print('n', n, 'diffs', d.sum(), 'frames', np.unique(frames)[:20], 'nframes', len(np.unique(frames)), 'of', w.shape[1])
    print(' bins', np.unique(bins)[:20], len(np.unique(bins)))
    if d.sum():
        i = np.argmax(np.abs(g - w) / np.maximum(w, 1e-30))
        b, f = np.unravel_index(i, w.shape)
        print(' worst', b, f, g[b, f], w[b, f], 'ulps', int(g.view(np.int32)[b,f]) - int(w.view(np.int32)[b,f]))
        ul = (g.view(np.int32)[d].astype(np.int64) - w.view(np.int32)[d].astype(np.int64))
        print(' ulp hist', np.unique(np.clip(ul, -5, 5), return_counts=True))
        # per-frame count for the first few frames with diffs
        uf, cnt = np.unique(frames, return_counts=True)
        print(' per-frame counts', list(zip(uf[:10], cnt[:10])))
# timing: the STFT alone (aa_sn_spectrogram: no median, no max) vs inside aa_sn_run
x = torch.from_numpy(_clip(60.0, 30)).cuda()
for _ in range(3):
    det.spectrogram(x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    det.spectrogram(x)
e1.record(); torch.cuda.synchronize()
print('aa_sn_spectrogram (stft64, no median) ms per 60 s clip', e0.elapsed_time(e1) / 20)
det.set_timing(True)
for _ in range(10):
    det.components(x)
torch.cuda.synchronize(); det.set_timing(False)
for i in range(det.n_stages()):
    ms, c = det.stage_time(i)
    print(det.stage_info(i)[0], 'ms per launch', ms / max(c, 1), c)
# A/B of the two row-median kernels (plan option read at creation)
import os
for mode in ("lds", "reg"):
    os.environ["AA_SN_SELECT"] = mode
    d2 = SignalDetector(48000, 281, torch.device('cuda'))
    st = d2.components(x)
    d2.set_timing(True)
    for _ in range(10):
        d2.components(x)
    torch.cuda.synchronize(); d2.set_timing(False)
    ms, c = d2.stage_time(2)
    print('select', mode, 'ms per launch', ms / max(c, 1), 'components', len(st))
