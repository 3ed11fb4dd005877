"""CPU: chromosome sharding and the track gather over torch.distributed (gloo,
world_size 2).  Each rank scans its shard with the CPU oracle standing in for the
device scan; the gathered track must equal the single-process genome scan."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def test_plan_shards_balances_and_covers():
    from gdscan.shard import plan_shards
    counts = [500, 480, 300, 300, 120, 90, 60, 10]
    for world in (1, 2, 3, 8):
        shards = plan_shards(counts, world)
        assert sorted(c for s in shards for c in s) == list(range(len(counts)))
        loads = [sum(counts[c] for c in s) for s in shards]
        assert max(loads) - min(loads) <= max(counts)
    assert plan_shards(counts, 2) == plan_shards(counts, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent
    sys.path.insert(0, str(root))
    import ctypes
    import torch
    import torch.distributed as dist
    from conftest import ORACLE_LIB, DP, IP, oracle_fet_scan
    from gdscan import synth
    from gdscan.shard import gather_tracks, plan_shards
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = ctypes.CDLL(str(ORACLE_LIB))
    C = ctypes
    orc.orc_fet_scan.argtypes = [DP, DP, IP, IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                 C.c_uint64, C.c_int, DP, DP]
    sizes = [9000, 4000, 7000, 3000, 6000]
    chroms = [synth.chromosome(40 + c, n, 6, 6) for c, n in enumerate(sizes)]
    wins = [x[4] // 500 for x in chroms]
    shards = plan_shards(sizes, world)
    parts = []
    for c in shards[rank]:
        av, bv, ap, bp, regend = chroms[c]
        s, d = oracle_fet_scan(orc, av, bv, ap, bp, regend, seed=100 + c)
        parts.append(np.stack([s, d], 1))
    local = torch.from_numpy(np.concatenate(parts) if parts else np.zeros((0, 2)))
    track = gather_tracks(local, shards, wins).numpy()
    if rank == 0:
        ref = []
        for c, (av, bv, ap, bp, regend) in enumerate(chroms):
            s, d = oracle_fet_scan(orc, av, bv, ap, bp, regend, seed=100 + c)
            ref.append(np.stack([s, d], 1))
        q.put(bool(np.array_equal(track, np.concatenate(ref))))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_tracks_gloo_world2(oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


def test_choose_backend():
    """RCCL with device tensors when every rank has its own GPU; gloo on host tensors when
    ranks must share devices (RCCL refuses two ranks on one GPU) or gloo is asked for."""
    from gdscan.shard import choose_backend
    assert choose_backend(8, 8) == ("nccl", True)
    assert choose_backend(1, 1) == ("nccl", True)
    assert choose_backend(2, 1) == ("gloo", False)
    assert choose_backend(4, 8, "gloo") == ("gloo", False)
    assert choose_backend(1, 0) == ("nccl", True)  # one rank, GPU count unknown before init


class _Store:
    def __init__(self):
        self.v = {}

    def add(self, key, n):
        self.v[key] = self.v.get(key, 0) + n
        return self.v[key]


def test_queue_pull_pipelined_prefetches_next_ticket():
    """The input moves with the ticket: ticket t + 1 is prepared before t is worked on,
    never more than `slots` inputs are alive, and a slot is reused only after its scan."""
    from gdscan.shard import queue_pull_pipelined
    events, live = [], {}

    def prepare(c, slot):
        assert slot not in live, "slot overwritten while its ticket is still unscanned"
        live[slot] = c
        events.append(("prep", c, slot))

    def work(c, slot):
        assert live.pop(slot) == c
        events.append(("work", c, slot))

    done = queue_pull_pipelined(_Store(), "k", 5, prepare, work)
    assert done == [0, 1, 2, 3, 4]
    assert events[:3] == [("prep", 0, 0), ("prep", 1, 1), ("work", 0, 0)]
    assert [e for e in events if e[0] == "work"] == [("work", c, c % 2) for c in range(5)]
    assert queue_pull_pipelined(_Store(), "k", 0, prepare, work) == []


def _worker_to0(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from gdscan.shard import gather_tracks, gather_tracks_to
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wins = [5, 0, 7, 3, 4]
    shards = [[0, 3], [1, 2, 4]]
    offs = np.concatenate([[0], np.cumsum(wins)])
    local = torch.cat([torch.stack([torch.arange(offs[c], offs[c + 1], dtype=torch.float64),
                                    -torch.arange(offs[c], offs[c + 1], dtype=torch.float64)], 1)
                       for c in shards[rank]])
    t0 = gather_tracks_to(local, shards, wins, dst=0)
    ta = gather_tracks(local, shards, wins)
    want = torch.arange(offs[-1], dtype=torch.float64)
    if rank == 0:
        q.put(bool(torch.equal(t0[:, 0], want) and torch.equal(t0[:, 1], -want) and torch.equal(t0, ta)))
    else:
        q.put(t0 is None)
    dist.barrier()
    dist.destroy_process_group()


def test_gather_tracks_to_rank0_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_to0, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True and q.get(timeout=10) is True


def test_plan_window_shards_covers_and_balances():
    from gdscan.shard import plan_window_shards
    for wins, world in (([100], 4), ([100, 10, 300], 3), ([5, 5], 8), ([0, 50], 2), ([4997], 8)):
        plan = plan_window_shards(wins, world)
        got = {c: [] for c in range(len(wins))}
        for pieces in plan:
            for c, w0, w1 in pieces:
                assert 0 <= w0 < w1 <= wins[c]
                got[c] += list(range(w0, w1))
        for c, w in enumerate(wins):
            assert sorted(got[c]) == list(range(w))
        loads = [sum(w1 - w0 for _, w0, w1 in p) for p in plan]
        assert max(loads) - min(loads) <= 1 + sum(wins) // (8 * world) or max(wins) < world
    # a weighted split follows the weights, not the window count
    import numpy as np
    plan = plan_window_shards([100], 2, weights=[np.r_[np.full(50, 3.0), np.ones(50)]])
    assert plan[0] == [(0, 0, 33)] and plan[1] == [(0, 33, 100)]


def test_window_shard_slice_and_regularity():
    import numpy as np
    from gdscan import synth
    from gdscan.shard import is_row_regular, window_shard_slice
    av, bv, ap, bp, regend = synth.chromosome(45, 3000, 5, 7)
    assert is_row_regular(ap, bp)
    rowpos = ap[::5]
    a_lo, a_hi, b_lo, b_hi = window_shard_slice(rowpos, 5, 7, 40, 90, 2500, 500)
    assert a_lo % 5 == 0 and b_lo // 7 == a_lo // 5 and b_hi // 7 == a_hi // 5
    assert ap[a_lo] >= 40 * 500 and (a_lo == 0 or ap[a_lo - 1] < 40 * 500)
    assert ap[a_hi - 1] <= 89 * 500 + 2500 and (a_hi == len(ap) or ap[a_hi] > 89 * 500 + 2500)
    bad = bp.copy()
    bad[7 * 100] += 1  # one B individual off its row's position
    assert not is_row_regular(ap, bad)
    assert not is_row_regular(ap, bp[:-2])


def _range_worker(rank, world, port, q):
    """Each rank scans its window-range pieces with the oracle on the pieces' slices (the
    chromosome's regend and seed, positions as they are): the windows of the range see
    exactly the rows the whole-chromosome scan gives them, with the same per-window seeds."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent
    sys.path.insert(0, str(root))
    import ctypes
    import torch
    import torch.distributed as dist
    from conftest import ORACLE_LIB, DP, IP, oracle_css_scan, oracle_fet_scan
    from gdscan import lib, synth
    from gdscan.shard import gather_window_tracks, plan_window_shards, window_shard_slice
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = ctypes.CDLL(str(ORACLE_LIB))
    C = ctypes
    orc.orc_fet_scan.argtypes = [DP, DP, IP, IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                 C.c_uint64, C.c_int, DP, DP]
    orc.orc_css_scan.argtypes = [DP, DP, IP, IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_uint64, C.c_int, DP, DP]
    a, b = 6, 5
    # one long chromosome (the case whole-chromosome shards leave on one rank) and a short one
    chroms = [synth.chromosome(47, 14000, a, b), synth.chromosome(48, 3000, a, b)]
    wins = [lib.gd_window_count(x[4], 2500, 500, 0) for x in chroms]
    plan = plan_window_shards(wins, world)
    ok = True
    for kind in ("fet", "css"):
        parts = []
        for c, w0, w1 in plan[rank]:
            av, bv, ap, bp, regend = chroms[c]
            a_lo, a_hi, b_lo, b_hi = window_shard_slice(ap[::a], a, b, w0, w1, 2500, 500)
            sl = (av[a_lo:a_hi], bv[b_lo:b_hi], ap[a_lo:a_hi], bp[b_lo:b_hi], regend)
            if kind == "fet":
                s, d = oracle_fet_scan(orc, *sl, seed=300 + c)
            else:
                s, d = oracle_css_scan(orc, *sl, runs=40, seed=300 + c)
            parts.append(np.stack([s[w0:w1], d[w0:w1]], 1))
        local = torch.from_numpy(np.concatenate(parts) if parts else np.zeros((0, 2)))
        counts = [sum(w1 - w0 for _, w0, w1 in p) for p in plan]
        track = gather_window_tracks(local, counts).numpy()
        if rank == 0:
            ref = []
            for c, (av, bv, ap, bp, regend) in enumerate(chroms):
                if kind == "fet":
                    s, d = oracle_fet_scan(orc, av, bv, ap, bp, regend, seed=300 + c)
                else:
                    s, d = oracle_css_scan(orc, av, bv, ap, bp, regend, runs=40, seed=300 + c)
                ref.append(np.stack([s[:wins[c]], d[:wins[c]]], 1))
            ok &= bool(np.array_equal(track, np.concatenate(ref)))
            ok &= bool((track[:, 0] != 0).sum() > 100)
    if rank == 0:
        q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_window_range_shards_gloo(oracle, world):
    """SURVEY 8(e) / VERDICT r05 item 4: one chromosome split into window ranges across
    `world` ranks (gloo); the gathered FET and CSS tracks equal the one-process scan bit
    for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_range_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True
