import os, sys, torch
sys.path[:0] = ['.', 'audio-analysis_amd']
from tests.test_gpu_signal import _clip
from aa_amd.signals import SignalDetector
x = torch.from_numpy(_clip(60.0, 30)).cuda()
for sel, diag in [("row", 0), ("reg", 0), ("reg", 1), ("reg", 3)]:
    os.environ["AA_SN_SELECT"] = sel; os.environ["AA_SN_DIAG"] = str(diag)
    d = SignalDetector(48000, 281, torch.device('cuda'))
    d.components(x)
    d.set_timing(True)
    for _ in range(10):
        d.components(x)
    torch.cuda.synchronize(); d.set_timing(False)
    ms, c = d.stage_time(2)
    print(sel, diag, 'select ms', round(ms / c, 4))
