"""The bench's non-default configurations run end to end on the GPU and
print one contract-shaped JSON line (BASELINE configs[2] stream: --config 3;
configs[3] corpus of WAV files through the analyse path: --config 4;
configs[4] fp16 log-mel + fp8: --precision fp8 --logmel f16)."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _bench(*args):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, timeout=240,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "ms_per_step", "config", "dtype"):
        assert k in line
    assert line["value"] > 0
    return line


def test_bench_config4_corpus(gpu):
    line = _bench("--config", "4", "--files", "3")
    assert line["config"]["documents_gathered"] == 3


def test_bench_config3_stream(gpu):
    line = _bench("--config", "3", "--clips", "24")
    assert line["config"]["records_gathered"] == 24


def test_bench_configs4_fp16_logmel_fp8(gpu):
    line = _bench("--precision", "fp8", "--logmel", "f16", "--steps", "5", "--warmup", "2", "--secondary=",
                  "--cpu-seconds", "0")
    assert line["dtype"] == "fp8 (fp16 log-mel)"
    assert "roofline" in line and line["roofline"]["achieved"] > 0


@pytest.mark.parametrize("pipeline", ["0", "1", "2"])
def test_bench_step_modes_hold_the_gate(gpu, pipeline):
    """The headline step back to back (0), with the next batch's front end
    overlapped (1) and with two batches in flight on two streams (2, the
    default): each asserts the 1e-3 logit gate on its own 64 windows (a step
    on clip pair 0 after the timed loop, against the CPU oracle)."""
    line = _bench("--pipeline", pipeline, "--steps", "6", "--warmup", "2", "--secondary=", "--cpu-seconds", "0")
    assert line["parity_gate"]["pass"]
    assert line["max_abs_dlogit"]["bf16x3"] <= 1e-3
    assert line["steps"] == 6
