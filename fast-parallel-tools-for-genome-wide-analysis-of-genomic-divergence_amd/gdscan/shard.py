"""Multi-GPU sharding of a genome-wide scan.

Windows depend only on the SNPs they cover, so a genome shards without any data-path
exchange: by whole chromosomes (plan_shards), or -- when there are fewer or very
unequal chromosomes than GPUs, or one chromosome per call -- by contiguous window
ranges whose SNP span carries the (wsize - wstep) halo (plan_window_shards, the
reference's 100-window task with its get_positions span, threadfisher.c:106-116,
191-239; threadcss.c:114-124, 226-276).  Each rank (one process per GPU) scans its
own shards.  The only collective is the optional gather of the finished
per-window tracks (score, stddev|p: 16 B per window), as equal-padded slices of one
all-gather (every rank gets the track) or of one gather to a single rank (RCCL over
xGMI on GPUs, gloo in the CPU tests).
"""
from __future__ import annotations

import numpy as np


def plan_shards(snp_counts, world):
    """Assign chromosomes to ranks, balancing SNPs (longest-processing-time greedy).

    Deterministic: ties go to the lowest rank.  Returns one sorted list of
    chromosome indices per rank."""
    order = sorted(range(len(snp_counts)), key=lambda c: (-int(snp_counts[c]), c))
    load = [0] * world
    out = [[] for _ in range(world)]
    for c in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(c)
        load[r] += int(snp_counts[c])
    return [sorted(x) for x in out]


def plan_window_shards(wins, world, weights=None):
    """Split the genome's window sets into `world` contiguous ranges of near-equal weight.

    wins[c]: windows chromosome c computes (gd_window_count of its regend); weights[c]
    (optional): per-window cost array of chromosome c (default 1 per window, the CSS
    shape; SNP rows per window for FET).  Rank r gets the genome windows between two cut
    points, as (c, w0, w1) pieces in genome order -- whole chromosomes inside the range,
    window ranges at its ends -- so every rank has work even with one chromosome, and a
    chromosome is split only where a cut falls.  Deterministic; empty pieces dropped."""
    wins = [int(w) for w in wins]
    if weights is None:
        weights = [np.ones(w) for w in wins]
    cum = [np.concatenate([[0.0], np.cumsum(np.asarray(weights[c], dtype=np.float64)[:wins[c]])])
           for c in range(len(wins))]
    base = np.concatenate([[0.0], np.cumsum([cw[-1] for cw in cum])])
    total = base[-1]
    out = [[] for _ in range(world)]
    for c in range(len(wins)):
        if wins[c] <= 0:
            continue
        # window w of chromosome c belongs to the rank whose share holds its weight's midpoint
        mid = base[c] + 0.5 * (cum[c][:-1] + cum[c][1:])
        rank = np.minimum((mid * world / total).astype(np.int64), world - 1) if total > 0 else \
            np.zeros(wins[c], dtype=np.int64)
        cuts = np.flatnonzero(np.diff(rank)) + 1
        starts = np.concatenate([[0], cuts])
        ends = np.concatenate([cuts, [wins[c]]])
        for w0, w1 in zip(starts, ends):
            out[int(rank[w0])].append((c, int(w0), int(w1)))
    return out


def window_shard_slice(rowpos, asize, bsize, w0, w1, wsize, wstep):
    """Element ranges (a_lo, a_hi, b_lo, b_hi) of the A and B arrays a window-range shard
    [w0, w1) reads: the rows from the first at position >= w0 wstep to the last at position
    <= (w1 - 1) wstep + wsize (windows are inclusive intervals, comparative.c:59-65), i.e.
    the range's own rows plus the (wsize - wstep) halo of its last window.  rowpos: the
    chromosome's row positions (whole rows, A and B rows at the same positions -- the
    form is_row_regular checks)."""
    r0 = int(np.searchsorted(rowpos, w0 * wstep, side="left"))
    r1 = int(np.searchsorted(rowpos, (w1 - 1) * wstep + wsize, side="right"))
    return r0 * asize, r1 * asize, r0 * bsize, r1 * bsize


def is_row_regular(apos, bpos):
    """True when the tracks are whole rows that a window-range shard may cut between: every
    A row holds asize equal positions (asize = get_population_size, comparative.c:25-34),
    every B row bsize, and the A and B rows sit at the same positions.  Anything else (the
    reference's A-driven slicing of misaligned tracks, Q4) shards by whole chromosomes."""
    apos, bpos = np.asarray(apos), np.asarray(bpos)
    if apos.size == 0 or bpos.size == 0:
        return False
    a = int(np.argmax(apos != apos[0])) if (apos != apos[0]).any() else apos.size
    b = int(np.argmax(bpos != bpos[0])) if (bpos != bpos[0]).any() else bpos.size
    if apos.size % a or bpos.size % b or apos.size // a != bpos.size // b:
        return False
    ar, br = apos.reshape(-1, a), bpos.reshape(-1, b)
    return bool((ar == ar[:, :1]).all() and (br == br[:, :1]).all() and np.array_equal(ar[:, 0], br[:, 0])
                and (np.diff(ar[:, 0]) >= 0).all())


def population_size(pos):
    """get_population_size (comparative.c:25-34): the leading run of pos[0]."""
    pos = np.asarray(pos)
    diff = np.flatnonzero(pos != pos[0])
    return int(diff[0]) if diff.size else int(pos.size)


def scan_window_pieces(kind, pieces, chroms, seeds, wsize=2500, wstep=500, perc=0.95, treshold=10, runs=0,
                       serial=False, exact=False):
    """Scan window-range pieces (plan_window_shards output for one rank, or any (c, w0, w1)
    list) of host-resident chromosomes in ONE device batch: each piece becomes a gd_chrom
    with w_first = w0, w_count = w1 - w0 over its rows' slice (window_shard_slice), the
    chromosome's regend and seeds[c].  kind "fet" -> (score, stddev), "css" -> (score, p).
    Returns the [sum(w1 - w0), 2] track of the pieces in order, equal bit for bit to the
    same windows of whole-chromosome scans.  Tracks must be row-regular (is_row_regular)."""
    from ._lib import GD_WINDOWS_SERIAL, GD_WINDOWS_THREADED, Chrom, check, lib
    import ctypes as C
    sl = []
    for c, w0, w1 in pieces:
        av, bv, ap, bp, regend = chroms[c]
        a, b = population_size(ap), population_size(bp)
        a_lo, a_hi, b_lo, b_hi = window_shard_slice(np.asarray(ap)[::a], a, b, w0, w1, wsize, wstep)
        sl.append((c, w0, w1, a_lo, a_hi, b_lo, b_hi))
    n = sum(w1 - w0 for _, w0, w1, *_ in sl)
    out0, out1 = np.zeros(max(n, 1)), np.zeros(max(n, 1))
    if not sl:
        return np.zeros((0, 2))
    av = np.ascontiguousarray(np.concatenate([chroms[c][0][a_lo:a_hi] for c, _, _, a_lo, a_hi, _, _ in sl]), np.float64)
    bv = np.ascontiguousarray(np.concatenate([chroms[c][1][b_lo:b_hi] for c, _, _, _, _, b_lo, b_hi in sl]), np.float64)
    ap = np.ascontiguousarray(np.concatenate([chroms[c][2][a_lo:a_hi] for c, _, _, a_lo, a_hi, _, _ in sl]), np.int32)
    bp = np.ascontiguousarray(np.concatenate([chroms[c][3][b_lo:b_hi] for c, _, _, _, _, b_lo, b_hi in sl]), np.int32)
    desc = (Chrom * len(sl))()
    ao = bo = wo = 0
    for k, (c, w0, w1, a_lo, a_hi, b_lo, b_hi) in enumerate(sl):
        d = desc[k]
        d.a_off, d.b_off, d.alen, d.blen = ao, bo, a_hi - a_lo, b_hi - b_lo
        d.regend, d.w_first, d.w_count, d.w_out, d.seed = int(chroms[c][4]), w0, w1 - w0, wo, int(seeds[c])
        ao, bo, wo = ao + (a_hi - a_lo), bo + (b_hi - b_lo), wo + (w1 - w0)
    DP, IP = C.POINTER(C.c_double), C.POINTER(C.c_int)
    ptrs = (av.ctypes.data_as(DP), bv.ctypes.data_as(DP), ap.ctypes.data_as(IP), bp.ctypes.data_as(IP))
    ws = GD_WINDOWS_SERIAL if serial else GD_WINDOWS_THREADED
    if kind == "fet":
        check(lib.gd_fet_scan_host_batch_ex(desc, len(sl), *ptrs, int(wsize), int(wstep), float(perc),
                                            1 if exact else 0, ws, out0.ctypes.data_as(DP), out1.ctypes.data_as(DP)))
    else:
        check(lib.gd_css_scan_host_batch(desc, len(sl), *ptrs, int(wsize), int(wstep), int(treshold), int(runs), ws,
                                         out0.ctypes.data_as(DP), out1.ctypes.data_as(DP)))
    return np.stack([out0[:n], out1[:n]], 1)


def gather_window_tracks(local, counts, group=None):
    """All-gather every rank's window-range track (rank r's pieces in genome order,
    counts[r] windows) into the genome-ordered concatenation of the ranks' ranges."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    width = local.shape[1] if local.dim() == 2 else 1
    pad = max(int(n) for n in counts) if counts else 0
    buf = torch.zeros((pad, width), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local.reshape(-1, width)
    out = torch.empty((world * pad, width), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    return torch.cat([out[r * pad: r * pad + int(counts[r])] for r in range(world)], 0)


def gather_tracks(local, shards, windows_per_chrom, group=None):
    """All-gather every rank's concatenated per-window track into genome order.

    local: tensor [n_local_windows, k] -- this rank's chromosomes, in shard order.
    shards: plan_shards() output; windows_per_chrom: windows of every chromosome.
    Returns the [total_windows, k] track on every rank (CPU or device tensor,
    matching `local`)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    counts = [sum(int(windows_per_chrom[c]) for c in s) for s in shards]
    width = local.shape[1] if local.dim() == 2 else 1
    pad = max(counts) if counts else 0
    buf = torch.zeros((pad, width), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local.reshape(-1, width)
    out = torch.empty((world * pad, width), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    # one gather into genome order: row offs[c] + k of the track is row r * pad + pos_c + k
    # of the all-gathered buffer (pos_c: chromosome c's start inside rank r's slice)
    src = _genome_index(shards, windows_per_chrom, pad)
    return out.index_select(0, torch.from_numpy(src).to(out.device))


def _genome_index(shards, windows_per_chrom, pad):
    """Row of the rank-major padded buffer holding each window of the genome-ordered track."""
    offs = np.concatenate([[0], np.cumsum([int(w) for w in windows_per_chrom])])
    src = np.empty(int(offs[-1]), dtype=np.int64)
    for r, s in enumerate(shards):
        pos = 0
        for c in s:
            n = int(windows_per_chrom[c])
            src[offs[c]:offs[c] + n] = np.arange(r * pad + pos, r * pad + pos + n)
            pos += n
    return src


def gather_tracks_to(local, shards, windows_per_chrom, dst=0, group=None):
    """Gather every rank's concatenated track to rank `dst` only, in genome order.

    The same equal-padded slices as gather_tracks, but one gather instead of an
    all-gather: world x fewer bytes on the links (only dst receives).  Returns the
    [total_windows, k] track on dst and None on the other ranks."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [sum(int(windows_per_chrom[c]) for c in s) for s in shards]
    width = local.shape[1] if local.dim() == 2 else 1
    pad = max(counts) if counts else 0
    buf = torch.zeros((pad, width), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local.reshape(-1, width)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, parts, dst=dst, group=group)
    if rank != dst:
        return None
    out = torch.cat(parts, 0)
    src = _genome_index(shards, windows_per_chrom, pad)
    return out.index_select(0, torch.from_numpy(src).to(out.device))


def default_store():
    """The key-value store of the default process group (c10d TCPStore under torchrun)."""
    import torch.distributed as dist
    return dist.distributed_c10d._get_default_store()


def queue_pull(store, key, n_items, work):
    """Dynamic chromosome queue across ranks: the reference's mutex-guarded task counter
    (threadcss.c:226-232, threadfisher.c:191-201) lifted to one process per GPU.  Each rank
    takes the next ticket from the store's atomic counter `key` and runs work(ticket) until
    all n_items are taken, so ranks whose chromosomes cost more (C5's early-exit
    permutations) simply pull fewer.  Returns the tickets this rank ran, in order."""
    done = []
    while True:
        k = int(store.add(key, 1)) - 1
        if k >= n_items:
            return done
        work(k)
        done.append(k)


def queue_pull_pipelined(store, key, n_items, prepare, work, slots=2):
    """queue_pull with the input moving with the ticket: a rank materialises only the
    chromosomes it pulls, into `slots` rotating buffers.  prepare(ticket, slot) starts
    producing a ticket's input (generation or H2D, asynchronous on its own stream);
    work(ticket, slot) scans it and returns when the scan no longer reads the slot.
    While ticket t scans, the next ticket is already pulled and being prepared, so the
    input of t + 1 overlaps the scan of t; per-rank input memory is `slots`
    chromosomes at any world size.  Returns the tickets this rank ran, in order."""
    def take():
        k = int(store.add(key, 1)) - 1
        return k if k < n_items else None

    done = []
    cur, slot = take(), 0
    if cur is None:
        return done
    prepare(cur, slot)
    while cur is not None:
        nxt = take()
        if nxt is not None:
            prepare(nxt, (slot + 1) % slots)
        work(cur, slot)
        done.append(cur)
        cur, slot = nxt, (slot + 1) % slots
    return done


def choose_backend(world, ndev, requested="nccl"):
    """Collective backend and tensor placement for `world` ranks on a box with `ndev`
    GPUs: RCCL ("nccl") with device tensors when every rank has its own GPU, gloo with
    host tensors when ranks must share devices (RCCL refuses two ranks on one GPU) or
    when gloo is asked for.  Returns (backend, tensors_on_device)."""
    if requested == "gloo" or world > max(1, ndev):
        return "gloo", False
    return requested, True


def gather_lists(items, group=None):
    """All-gather one variable-length list of ints per rank (tiny; CPU tensors over the
    default group's backend are not needed: uses all_gather_object)."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, [int(x) for x in items], group=group)
    return out
