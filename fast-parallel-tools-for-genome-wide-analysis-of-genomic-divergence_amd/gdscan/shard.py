"""Multi-GPU sharding of a genome-wide scan.

Windows depend only on the SNPs they cover, so a genome shards by whole
chromosomes: each rank (one process per GPU) scans its own chromosomes with no
data-path exchange.  The only collective is the optional gather of the finished
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
