"""Corpus runner (aa_amd.corpus): files sharded over ranks, examine() per
file, per-file JSON documents all-gathered, rank 0 writes the reference's
outputs.  CPU: two gloo ranks with a deterministic stand-in for examine()
must reproduce the single-process results byte for byte.  GPU: real
classifications of synthetic recordings (model1+model2 through libaa.so) by
two ranks sharing cuda:0 over gloo against one process."""
import json
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from aa_amd import corpus

FILES = [f"rec{i:02d}.wav" for i in range(7)]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def fake_examine(path, models, analyse_tracks=False):
    i = int(os.path.basename(path)[3:5])
    rng = np.random.default_rng(i)
    n = int(rng.integers(0, 4))
    return {"species_identify": [{"start_s": float(rng.random()), "predictions": [
        {"what": "morepork", "confidence": int(rng.integers(0, 100))}] * k} for k in range(n)],
        "non_bird_tags": ["noise"], "models": list(models), "tracks": analyse_tracks}


def bad_examine(path, models, analyse_tracks=False):
    if path.endswith("rec03.wav"):
        raise ValueError("Could not load rec03.wav")  # e.g. an unsupported codec
    return fake_examine(path, models, analyse_tracks)


def _strip(res):
    return json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "processing_time_seconds"}
                       for k, v in res.items()}, sort_keys=True)


def _cpu_worker(rank, world, port, q, examine=fake_examine):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _strip(corpus.run(FILES, ["m1", "m2"], True, examine_fn=examine, rank=rank,
                                       world=world))))
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return outs


def test_corpus_single_process_order():
    res = corpus.run(FILES, ["m1"], False, examine_fn=fake_examine)
    assert list(res) == list(range(len(FILES)))


@pytest.mark.parametrize("world", [2, 3])
def test_corpus_gloo_matches_single_process(world):
    single = _strip(corpus.run(FILES, ["m1", "m2"], True, examine_fn=fake_examine))
    outs = _spawn(_cpu_worker, world)
    for r in range(world):
        assert outs[r] == single  # every rank holds every file's document, byte for byte


def test_corpus_failed_file_does_not_stall_the_gather(tmp_path):
    """A file whose examine() raises (the reference's process would log and
    exit 1 for that file alone) is marked failed; the all-gather still
    completes on every rank, the other files keep their results, and no
    sidecar is written for the failed one."""
    single = json.loads(_strip(corpus.run(FILES, ["m1", "m2"], True, examine_fn=bad_examine)))
    assert corpus.FAILED in single["3"] and len(single) == len(FILES)
    outs = _spawn(_cpu_worker, 2, bad_examine)
    assert outs[0] == outs[1] == json.dumps(single, sort_keys=True)
    files = [str(tmp_path / f) for f in FILES]
    res = corpus.run(files, ["m1"], True, examine_fn=bad_examine)
    corpus.write_results(files, res)
    written = sorted(p.name for p in tmp_path.glob("*.txt"))
    assert written == [f"rec{i:02d}.txt" for i in range(7) if i != 3]


def _gpu_worker(rank, world, port, q, files, models):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _strip(corpus.run(files, models, False, rank=rank, world=world))))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_corpus_gpu_two_ranks_match_one(gpu, model_root, tmp_path):
    from tools import synth
    files = []
    for i in range(4):
        p = tmp_path / f"rec{i:02d}.wav"
        synth.write_wav(p, synth.clip(100 + i, seconds=12.0))
        files.append(str(p))
    models = [str(model_root / m / "audioModel.keras") for m in ("model1", "model2")]
    single = _strip(corpus.run(files, models, False))
    assert "species_identify" in single
    outs = _spawn(_gpu_worker, 2, files, models)
    assert outs[0] == single and outs[1] == single


def test_lanes_follow_hardware_queues(monkeypatch):
    """Batch lanes by GPU_MAX_HW_QUEUES (two queues per lane: compute + copy
    streams), AA_BATCH_LANES overriding; raise_hw_queues only ever raises."""
    from aa_amd import corpus
    monkeypatch.delenv("AA_BATCH_LANES", raising=False)
    for q, lanes in (("4", 3), ("7", 3), ("8", 5), ("12", 5), ("16", 8), ("32", 8), ("junk", 3)):
        monkeypatch.setenv("GPU_MAX_HW_QUEUES", q)
        assert corpus.default_lanes() == lanes, q
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    assert corpus.default_lanes() == 3  # HIP's default 4
    monkeypatch.setenv("AA_BATCH_LANES", "6")
    assert corpus.default_lanes() == 6
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    corpus.raise_hw_queues()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "16"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "24")
    corpus.raise_hw_queues()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "24"
