"""The collectives of the sharded corpus path over RCCL on
the GPU: a one-rank "nccl" process group (127.0.0.1) in the test process, so
the device-side all-gathers of aa_amd.shard.gather_records and
aa_amd.corpus.gather_documents run through RCCL (the CPU suite covers two and
three ranks over gloo: tests/test_shard.py, tests/test_corpus.py).  One rank
per GPU is RCCL's rule, and the box has one GPU, so the multi-rank exchange
itself is not exercised here; what is: communicator set-up on the device,
uint8 / int64 / float32 all-gathers on cuda tensors, and the corpus run's
documents through that gather equal to the same run without a process group."""
import json
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_group():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        yield dev
    finally:
        dist.destroy_process_group()


def test_gather_records_over_rccl(rccl_group):
    from aa_amd import shard
    dev = rccl_group
    rng = np.random.default_rng(3)
    # rows (file_idx, track_idx, n_labels, scores...) out of order, plus a
    # padding row (-1) that the gather drops
    rows = [(4, 1), (0, 2), (4, 0), (0, 0), (2, 5)]
    rec = torch.full((len(rows) + 1, 3 + 6), -1.0, dtype=torch.float32)
    for k, (f, t) in enumerate(rows):
        rec[k, 0], rec[k, 1], rec[k, 2] = f, t, 6
        rec[k, 3:] = torch.from_numpy(rng.random(6, dtype=np.float32))
    out = shard.gather_records(rec.to(dev))
    assert out.device.type == "cuda"
    got = out.cpu()
    want = rec[:-1][torch.argsort(rec[:-1, 0].double() * 1e6 + rec[:-1, 1].double())]
    assert torch.equal(got, want)


def test_gather_documents_over_rccl(rccl_group):
    from aa_amd import corpus
    docs = {7: {"species_identify": [{"label": "morepork", "confidence": 0.5}]}, 1: {"end_s": 12.5},
            3: {corpus.FAILED: "ValueError: x"}}
    got = corpus.gather_documents(docs, device=rccl_group)
    assert json.dumps(got, sort_keys=True) == json.dumps(dict(sorted(docs.items())), sort_keys=True)
    assert list(got) == [1, 3, 7]
    # a rank that classified nothing contributes an empty payload
    assert corpus.gather_documents({}, device=rccl_group) == {}


def test_corpus_run_through_rccl_gather(rccl_group, tmp_path):
    """corpus.run with the documents gathered over RCCL (world 1) equals the
    same files without a process group (the batched path, aa_amd.batch)."""
    from aa_amd import corpus
    from tools import synth
    from tools.make_models import make_model
    model = make_model(tmp_path / "model1", "model1", seed=1)
    files = []
    for i, secs in enumerate((60.0, 17.0, 3.5)):
        p = tmp_path / f"clip{i}.wav"
        synth.write_wav(p, synth.clip(7000 + i, seconds=secs))
        files.append(p)
    over_rccl = corpus.run(files, [str(model)], rank=0, world=1, device=rccl_group, batch=4)
    # the same documents with the gather skipped (the local dict, sorted)
    from aa_amd.batch import BatchAnalyser
    ba = BatchAnalyser([str(model)], False, device=rccl_group, batch=4, lanes=1)
    local = dict(sorted(ba.run([(i, str(f)) for i, f in enumerate(files)]).items()))

    def strip(d):
        return json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "processing_time_seconds"}
                           for k, v in d.items()}, sort_keys=True)

    assert list(over_rccl) == [0, 1, 2]
    assert strip(over_rccl) == strip(local)
