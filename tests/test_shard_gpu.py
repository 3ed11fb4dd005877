"""GPU: the multi-rank path through libgdscan.  Two ranks (gloo collectives, both ranks
on cuda:0 -- the pool's boxes have one GPU) scan their shards of a small genome with the
HIP kernels (FET, and CSS with permutations) and all-gather the (score, stddev | p)
tracks into genome order (gdscan.shard.gather_tracks, the bench's one collective); the
gathered tracks must equal one process's scan of the whole genome bit for bit: windows
draw from per-chromosome, per-window seeds, so results do not depend on the shard
layout."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = [9000, 4000, 7000, 3000, 6000]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _scan_all(which, chroms, idx):
    from gdscan import css, fet
    out = []
    for c in idx:
        av, bv, ap, bp, regend = chroms[c]
        if which == "fet":
            a, b = fet.scan(av, bv, ap, bp, regend, seed=100 + c)
        else:
            a, b = css.scan(av, bv, ap, bp, regend, treshold=10, runs=200, seed=200 + c)
        out.append(np.stack([a, b], 1))
    return np.concatenate(out) if out else np.zeros((0, 2))


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    import conftest  # noqa: F401  (package path)
    import torch
    import torch.distributed as dist
    from gdscan import synth
    from gdscan.shard import gather_tracks, plan_shards
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    chroms = [synth.chromosome(60 + c, n, 10, 10) for c, n in enumerate(SIZES)]
    wins = [x[4] // 500 for x in chroms]
    shards = plan_shards(SIZES, world)
    ok = {}
    for which in ("fet", "css"):
        local = torch.from_numpy(_scan_all(which, chroms, shards[rank]))
        track = gather_tracks(local, shards, wins).numpy()
        if rank == 0:
            ref = _scan_all(which, chroms, range(len(SIZES)))
            ok[which] = bool(np.array_equal(track, ref, equal_nan=True)) and bool((ref[:, 0] != 0).sum() > 100)
    if rank == 0:
        q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_scan_shards_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) == {"fet": True, "css": True}
