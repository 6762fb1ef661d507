"""Corpus runner: many recordings over the GPUs of one node.

The reference analyses one recording per process: an orchestrator runs
``docker run ... analyse.py FILE`` per file (README.md:28), each writing
``FILE.txt["analysis_result"]`` (src/analyse.py:434-470).  Here one process
per GPU (``torchrun`` or ``--gpus N``) takes files ``i % world == rank``
(shard.shard), runs the same ``examine()`` on each (classify() on its GPU),
and the per-file result documents -- JSON, variable length -- are all-gathered
once at the end (RCCL over xGMI with the nccl backend, gloo on CPU), so rank 0
holds every file's result in file order and writes the reference's sidecars
(or one JSON list on stdout).  Results do not depend on the world size: each
file is classified by exactly the code a single process would run.

    python -m aa_amd.corpus FILE... [--bird-model PATH]* [--analyse-tracks B] [-o] [--gpus N]
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

from . import shard


def gather_documents(local: dict, device=None, group=None) -> dict:
    """All-gather {file_idx: JSON-serialisable document} across ranks as
    UTF-8 bytes (padded to the longest rank; one collective for the sizes, one
    for the payload).  Without an initialised process group, returns ``local``."""
    if not dist.is_initialized():
        return dict(sorted(local.items()))
    dev = torch.device(device) if device is not None else torch.device("cpu")
    payload = json.dumps(sorted(local.items()), sort_keys=True).encode()
    n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    world = dist.get_world_size(group)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = max(int(s.item()) for s in sizes)
    buf = torch.zeros(m, dtype=torch.uint8, device=dev)
    if payload:
        buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = {}
    for p, s in zip(parts, sizes):
        for k, v in json.loads(bytes(p[:int(s.item())].cpu().numpy()).decode()):
            out[int(k)] = v
    return dict(sorted(out.items()))


# host lanes (threads, each with its own compute + copy HIP streams) of the
# batched path, by the process's hardware queues: a lane needs two queues of
# its own, or its streams share a queue with another lane's and run back to
# back.  Measured on one box each, two or three rounds (configs[3] secondary,
# audio-s/s): 4 queues / 3 lanes 114-124k; 8 / 5 114-149k; 8 / 6 130-131k;
# 16 / 8 131-149k; 24 / 12 132-148k; 32 / 16 107-131k (the host threads then
# contend for the GIL) -- profiles/r05/corpus_lanes.txt,
# profiles/r06/corpus_queues_lanes.txt.  corpus.main and bench.py raise
# GPU_MAX_HW_QUEUES to 16 before the first GPU call; a library user who did
# not keeps the lanes measured for HIP's default 4.
LANES_BY_QUEUES = ((16, 8), (8, 5), (0, 3))


def default_lanes() -> int:
    """AA_BATCH_LANES if set, else the lane count for the process's
    hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4 when unset)."""
    env = os.environ.get("AA_BATCH_LANES")
    if env:
        return int(env)
    try:
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        queues = 4
    return next(lanes for q, lanes in LANES_BY_QUEUES if queues >= q)


def raise_hw_queues(n: int = 16):
    """GPU_MAX_HW_QUEUES to at least n (HIP reads it once, at initialisation:
    call before the process's first GPU call)."""
    try:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)
    except ValueError:
        cur = 0
    if cur < n:
        os.environ["GPU_MAX_HW_QUEUES"] = str(n)


def run(files, bird_models, analyse_tracks=False, examine_fn=None, rank=0, world=1, device=None, batch=16):
    """Classify this rank's share of ``files``; returns {file_idx: summary}
    of ALL files on every rank (after the gather).  ``summary`` is what
    analyse.examine returns plus ``processing_time_seconds`` (src/analyse.py:451-453).
    With a GPU and the real examine, files go ``batch`` at a time through
    aa_amd.batch (the same documents, byte for byte); ``batch=0`` or a
    custom ``examine_fn`` runs them one by one."""
    mine = shard.shard(list(files), rank, world)
    if examine_fn is None and batch and torch.cuda.is_available():
        from .batch import BatchAnalyser
        ba = BatchAnalyser(bird_models, analyse_tracks, device=torch.device("cuda", torch.cuda.current_device()),
                           batch=batch, lanes=default_lanes())
        return gather_documents(ba.run([(i, str(f)) for i, f in mine]), device=device)
    if examine_fn is None:
        from .analyse import examine as examine_fn
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from . import identify_tracks as it
    local = {}

    def decode(f):
        try:
            return it.load_recording(str(f))
        except Exception:  # left to examine(), which reports it the reference's way
            return None

    # the next file is read and decoded on a host thread while this one is
    # classified (numpy releases the GIL in the bulk conversion)
    with ThreadPoolExecutor(max_workers=1) as pool:
        nxt = pool.submit(decode, mine[0][1]) if mine else None
        for k, (i, f) in enumerate(mine):
            pre = nxt.result()
            nxt = pool.submit(decode, mine[k + 1][1]) if k + 1 < len(mine) else None
            if pre is not None:
                it._PREFETCHED[(str(f), 48000)] = pre
            # short tracks draw random window offsets from the global RandomState
            # (src/identify_tracks.py:132, :167; the reference leaves it unseeded,
            # one process per file): seeding it per file makes every file's result
            # independent of which rank ran it and what ran before
            np.random.seed(i)
            t0 = time.time()
            try:
                summary = examine_fn(str(f), bird_models, analyse_tracks=analyse_tracks)
                summary["processing_time_seconds"] = round(time.time() - t0, 1)
            except Exception as e:
                # the reference's per-file process logs and exits 1 without a
                # sidecar (src/analyse.py:482-487); here the failure stays with
                # its file and the collective below still runs on every rank
                logging.error("Terminated with error", exc_info=True)
                summary = {FAILED: f"{type(e).__name__}: {e}"}
            finally:
                it._PREFETCHED.pop((str(f), 48000), None)
            local[i] = summary
    return gather_documents(local, device=device)


FAILED = "__failed__"  # marks a file whose examine() raised: no sidecar is written for it


def failed(result) -> bool:
    return FAILED in result


def write_results(files, results, to_stdout=False):
    """Rank 0: the reference's outputs per file -- FILE.txt["analysis_result"]
    merged into an existing sidecar (src/analyse.py:454-468) -- or, with -o,
    one JSON list of {"file", "analysis_result"} on stdout."""
    if to_stdout:
        print(json.dumps([{"file": str(files[i]), "analysis_result": r} for i, r in results.items()
                          if not failed(r)], sort_keys=True, indent=4))
        return
    from .analyse import write_metadata
    for i, r in results.items():
        if failed(r):
            logging.error("%s: not analysed (%s)", files[i], r[FAILED])
            continue
        write_metadata(files[i], r)


def _worker(local_rank, world, args, port):
    if port is not None:
        os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rank = int(os.environ.get("RANK", "0"))
    dev = None
    if torch.cuda.is_available():
        # one GPU per rank; more ranks than GPUs share them round-robin
        dev = torch.device("cuda", local_rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
    if world > 1:
        backend = args.backend or ("nccl" if dev is not None else "gloo")
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
    try:
        gdev = dev if (world > 1 and dist.get_backend() == "nccl") else None
        res = run(args.files, args.bird_model, args.analyse_tracks, rank=rank, world=world, device=gdev)
        if rank == 0:
            write_results(args.files, res, to_stdout=bool(args.meta_to_stdout))
    finally:
        if world > 1:
            dist.destroy_process_group()


def parse_args(argv=None):
    from .analyse import none_or_str, str2bool
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("files", nargs="+", help="audio files")
    ap.add_argument("--bird-model", type=none_or_str, action="append", help="Path to bird model")
    ap.add_argument("--analyse-tracks", type=str2bool, default=False)
    ap.add_argument("-o", "--meta-to-stdout", action="count")
    ap.add_argument("--gpus", type=int, default=1, help="ranks to spawn when not under torchrun")
    ap.add_argument("--backend", default=None, help="process-group backend (default nccl on GPU)")
    args = ap.parse_args(argv)
    if not args.bird_model:
        args.bird_model = ["/models/pre-model/audioModel.keras", "/models/bird-model-v2m/audioModel.keras"]
    return args


def main(argv=None):
    from .analyse import init_logging
    # hardware queues for the batch lanes' compute + copy streams (HIP's
    # default 4 puts some of them on one queue; read once, before the first
    # GPU call of the process: bench.py does the same)
    raise_hw_queues()
    args = parse_args(argv)
    init_logging()
    if "WORLD_SIZE" in os.environ:
        _worker(int(os.environ.get("LOCAL_RANK", "0")), int(os.environ["WORLD_SIZE"]), args, None)
    elif args.gpus > 1:
        import socket
        import torch.multiprocessing as mp
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        mp.spawn(_worker, args=(args.gpus, args, port), nprocs=args.gpus, join=True)
    else:
        _worker(0, 1, args, None)


if __name__ == "__main__":
    try:
        main()
    except Exception:
        logging.error("Terminated with error", exc_info=True)
        sys.exit(1)
