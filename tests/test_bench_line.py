"""bench.py's printed line stays parseable by the driver (<= 8,000 characters).

Round 5's line grew to 28.9 KB (per-stage tables of every secondary) and the
driver, which keeps ~8 KB of stdout, could not parse it.  These tests build the
line from a recorded full run (profiles/r05/bench.json, the 28.9 KB record) and
check its length and the fields the contract needs."""
import json
from pathlib import Path

import pytest

import bench

ROOT = Path(__file__).resolve().parents[1]
RECORD = ROOT / "profiles" / "r05" / "bench.json"


@pytest.fixture(scope="module")
def record():
    return json.loads(RECORD.read_text())


def test_recorded_run_compacts_under_limit(record):
    assert len(json.dumps(record)) > bench.LINE_LIMIT  # the record that broke r05's line
    text = bench.compact_line(record, "gpurun_out/bench_full.json")
    assert len(text) <= 8000
    line = json.loads(text)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "parity_gate",
              "max_abs_dlogit"):
        assert k in line, k
    r = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "whole_step"):
        assert k in r, k
    assert not any(k.startswith("stages") for k in r)
    assert line["value"] == record["value"]
    assert line["cpu_baseline"] == record["cpu_baseline"]


def test_secondaries_are_scalars(record):
    line = json.loads(bench.compact_line(record))
    sec = line["secondary"]
    assert set(sec) == set(record["secondary"])
    for name, s in sec.items():
        assert set(s) <= set(bench._SEC_KEYS) | {"kernel", "warm_same_run", "files_per_rank", "clips_per_rank"}
        assert isinstance(s["value"], float), name
        for v in s.values():
            assert not isinstance(v, (dict, list)), (name, v)
    assert sec["effnetv2"]["gate"] is True
    assert sec["f32"]["gate"] is True and "gate" not in sec["bf16"]


def test_oversized_line_raises(record):
    big = dict(record)
    big["data"] = "x" * 9000
    with pytest.raises(ValueError):
        bench.compact_line(big)


def test_worst_case_sizes_fit(record):
    """Every default secondary with long kernel names and the widest numbers
    still fits (the headline never depends on trimming luck)."""
    rec = json.loads(json.dumps(record))
    for name in bench.parse([]).secondary.split(","):
        rec["secondary"].setdefault(name, {"value": 1.0})
        rec["secondary"][name].update(value=123456789.123, ms_per_step=12345.6789, dtype="fp8 (fp16 log-mel)",
                                      max_abs_dlogit=0.12345678901234567,
                                      roofline={"frac": 0.12345678, "kernel": "k" * 200})
    assert len(bench.compact_line(rec, "gpurun_out/bench_full.json")) <= 8000
