"""Multi-process coverage of the sharded path on CPU: two
ranks over gloo (127.0.0.1), each classifies "its" files (here: synthetic
per-track scores), then the per-file result gather; every rank must end with
the same records a single process would have produced, in file order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aa_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scores(file_idx, n_tracks, L):
    rng = np.random.default_rng(file_idx)
    return rng.random((n_tracks, L), dtype=np.float32)


FILES = [f"clip{i:03d}.wav" for i in range(7)]
TRACKS = [1, 3, 0, 2, 1, 4, 2]  # file 2 has no tracks: a rank may own no rows
L = 5


def _reference():
    return {i: {t: _scores(i, n, L)[t] for t in range(n)} for i, n in enumerate(TRACKS) if n}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blocks = []
        for i, _ in shard.shard(FILES, rank, world):
            n = TRACKS[i]
            blocks.append(shard.pack_records(i, np.arange(n), _scores(i, n, L), width=8))
        rec = torch.from_numpy(np.concatenate(blocks) if blocks else np.zeros((0, 11), np.float32))
        got = shard.unpack_records(shard.gather_records(rec))
        q.put((rank, {f: {t: v.tolist() for t, v in d.items()} for f, d in got.items()}))
    finally:
        dist.destroy_process_group()


def test_shard_split():
    parts = [shard.shard(FILES, r, 3) for r in range(3)]
    assert sorted(i for p in parts for i, _ in p) == list(range(len(FILES)))
    assert [i for i, _ in parts[1]] == [1, 4]
    with pytest.raises(ValueError):
        shard.shard(FILES, 2, 2)


def test_gather_single_process():
    rec = torch.from_numpy(np.concatenate([
        shard.pack_records(3, [1, 0], _scores(3, 2, L)[::-1], width=8),
        shard.pack_records(1, [0], _scores(1, 1, L), width=8)]))
    got = shard.unpack_records(shard.gather_records(rec))
    assert list(got) == [1, 3]
    np.testing.assert_array_equal(got[3][0], _scores(3, 2, L)[0])


@pytest.mark.parametrize("world", [2])
def test_gather_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _reference()
    for r in range(world):
        got = outs[r]
        assert sorted(got) == sorted(ref)
        for f, d in ref.items():
            for t, v in d.items():
                np.testing.assert_array_equal(np.float32(got[f][t]), v)
