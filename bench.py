#!/usr/bin/env python3
"""Benchmark: genome-wide FET window scan on MI355X (BASELINE.json configs[1]).

One step = one device-resident FET scan (per-SNP Fisher exact test, window
95th-percentile score, 100-replicate bootstrap stddev) over this rank's batch of
synthetic chromosomes: 20 chromosomes x 500k SNPs, 20+20 individuals, 2.5 kb
windows / 500 bp step  (10M SNPs, ~1M windows per GPU).  Inputs are generated on
the device before timing; weak scaling: every rank scans its own 20 chromosomes
(chromosome ids rank*20 .. rank*20+19), no data-path collective.

Prints ONE JSON line (rank 0).  `roofline` prices the whole scan's algorithmic
HBM bytes B = 12*(alen+blen) + 16*W (f64 value + i32 position per
genotype, two f64 outputs per window) against its kernel time, and also lists each
stage's kernel time.  `traffic` is the measured HBM bytes per scan from the committed
rocprofv3 PMC summary (profiles/r02_fet_traffic.json, FETCH_SIZE doubled per the
gfx950 correction + WRITE_SIZE), or null when absent.  The scan is bound by VALU issue
(the bootstrap's draws), not HBM: `roofline.valu` prices the PMC-counted VALU
wave-instructions per scan (profiles/r02_fet_valu.json) over this run's scan time
against the 614 G wave-instructions/s issue peak.  `cpu_baseline` times the
reference's own Pthreads threadcompute() (oracle/_ref, compiled from the reference
sources) on a bounded sample of the same workload, or the oracle port when that
binary is absent.

A second object, `css`, measures the CSS scan (BASELINE.json configs[2]: 1M windows,
20+20, classical MDS, runs=0) on the same resident chromosomes, priced against the
FP64 roofline with SURVEY.md 8(d)'s solver-neutral (4/3) m^3 + 10 m^2 flops per
window, with the CPU oracle port timed on a sample beside it (the reference CSS
needs GSL, absent from the image, so no reference binary exists).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd"
sys.path.insert(0, str(PKG))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E spec
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec; ubench: ~31-37 T FMA/s
PROFILE_ROUND = "r02"
TRAFFIC_FILE = ROOT / "profiles" / f"{PROFILE_ROUND}_fet_traffic.json"
VALU_FILE = ROOT / "profiles" / f"{PROFILE_ROUND}_fet_valu.json"
CSS_VALU_FILE = ROOT / "profiles" / f"{PROFILE_ROUND}_css_valu.json"
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 4 cycles per SIMD
# at the 2.4 GHz max clock (MI355X_MICROARCH.md) = 614.4 G wave-instructions/s
VALU_PEAK_GINSTS = 256 * 4 * 2.4 / 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nchrom", type=int, default=20)
    ap.add_argument("--nsnp", type=int, default=500_000)
    ap.add_argument("--asize", type=int, default=20)
    ap.add_argument("--bsize", type=int, default=20)
    ap.add_argument("--wsize", type=int, default=2500)
    ap.add_argument("--wstep", type=int, default=500)
    ap.add_argument("--perc", type=float, default=0.95)
    ap.add_argument("--cpu-chroms", type=int, default=20, help="chromosomes in the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-css", action="store_true", help="skip the CSS leg")
    ap.add_argument("--no-extra", action="store_true", help="skip the region-filter and packed-track legs")
    ap.add_argument("--css-steps", type=int, default=3)
    ap.add_argument("--css-cpu-snps", type=int, default=150_000, help="SNPs in the CSS CPU-baseline sample")
    return ap.parse_args()


def css_cpu_baseline(args):
    """The CSS oracle port (1 thread) on a prefix of chromosome 0 of the same workload."""
    from gdscan import synth
    orc = ROOT / "oracle" / "_build" / "liboracle.so"
    DP = np.ctypeslib.ndpointer(np.float64, flags="C")
    IP = np.ctypeslib.ndpointer(np.int32, flags="C")
    C = ctypes
    lib = C.CDLL(str(orc))
    fn = lib.orc_css_scan
    fn.argtypes = [DP, DP, IP, IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                   C.c_int, DP, DP]
    av, bv, ap_, bp, regend = synth.chromosome(0, args.css_cpu_snps, args.asize, args.bsize)
    n = regend // args.wstep
    s, p = np.zeros(n), np.zeros(n)
    t0 = time.perf_counter()
    fn(av, bv, ap_, bp, regend, args.wsize, args.wstep, len(av), len(bv), 10, 0, 1, 0, s, p)
    dt = time.perf_counter() - t0
    from gdscan import fet
    w = fet.window_count(regend, args.wsize, args.wstep)
    return {"value": w / dt, "unit": "windows/s", "cores": 1, "kind": "port",
            "sample": f"chromosome 0 prefix, {args.css_cpu_snps} SNPs ({args.asize}+{args.bsize}), {w} windows "
                      f"in {dt:.2f} s, 1 thread (cyclic-Jacobi restatement; the reference CSS needs GSL, "
                      f"absent here)"}


def css_shape_run(args, lib, _lib, synth, Chrom, check, dev, stream, ctx, rank, nchrom, pop, treshold, runs):
    """One timed CSS scan of `nchrom` synthetic chromosomes with pop+pop individuals."""
    import torch
    nsnp = args.nsnp
    alen = nsnp * pop
    av = torch.empty(nchrom * alen, dtype=torch.float64, device=dev)
    bv = torch.empty(nchrom * alen, dtype=torch.float64, device=dev)
    ap = torch.empty(nchrom * alen, dtype=torch.int32, device=dev)
    bp = torch.empty(nchrom * alen, dtype=torch.int32, device=dev)
    qtab = torch.from_numpy(synth.freq_table()).to(dev)
    for c in range(nchrom):
        check(lib.gd_synth_device(1000 + rank * nchrom + c, nsnp, pop, pop, synth.MASTER_SEED, qtab.data_ptr(),
                                  av.data_ptr() + c * alen * 8, bv.data_ptr() + c * alen * 8,
                                  ap.data_ptr() + c * alen * 4, bp.data_ptr() + c * alen * 4, stream))
    torch.cuda.synchronize()
    last = ap.view(nchrom, alen)[:, -1].cpu().numpy().astype(np.int64)
    chroms = (Chrom * nchrom)()
    w_out = windows = 0
    for c in range(nchrom):
        regend = int(last[c]) + 1
        chroms[c].a_off = chroms[c].b_off = c * alen
        chroms[c].alen = chroms[c].blen = alen
        chroms[c].regend = regend
        chroms[c].w_out = w_out
        chroms[c].seed = synth.MASTER_SEED + 1000 + c
        w_out += regend // args.wstep
        windows += lib.gd_window_count(regend, args.wsize, args.wstep, _lib.GD_WINDOWS_THREADED)
    sc = torch.zeros(w_out, dtype=torch.float64, device=dev)
    pv = torch.zeros_like(sc)

    def step():
        check(lib.gd_css_scan_device(ctx, chroms, nchrom, av.data_ptr(), bv.data_ptr(), ap.data_ptr(), bp.data_ptr(),
                                     args.wsize, args.wstep, treshold, runs, _lib.GD_WINDOWS_THREADED,
                                     sc.data_ptr(), pv.data_ptr(), stream))

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stage = _lib.last_stage_ms()  # the timed step's HIP events: [1] planes + MDS, [2] permutations
    pm = pv.cpu().numpy()
    computed = sc.cpu().numpy() != 0
    out = {"value": windows / dt, "unit": "windows/s (one GPU)", "ms": dt * 1e3, "windows": windows,
           "config": f"{nchrom} chromosomes x {nsnp} SNPs, {pop}+{pop}, mcT={treshold}, mcR={runs}",
           "mean_p": float(pm[computed].mean()) if computed.any() else None,
           "stage_ms": {"planes_mds": stage[1], "permutations": stage[2]}}
    if runs > 0 and computed.any():
        # permutations run per window, from p = (hits + 1) / (run + 1): an early exit (hits =
        # mcT) leaves p > mcT / (mcR + 1), a full run p <= mcT / (mcR + 1)
        p = pm[computed]
        early = p * (runs + 1) > treshold + 0.5
        nrun = np.where(early, np.rint((treshold + 1) / p) - 1, runs)
        perms = float(nrun.sum())
        # (a*b + a + b) FP64 adds per permutation actually run
        ach = perms * (pop * pop + 2 * pop) / (stage[2] * 1e-3) / 1e12
        out["permutations"] = {
            "total": perms, "mean_per_window": float(nrun.mean()),
            "histogram": {"<=10": int((nrun <= 10).sum()), "11-100": int(((nrun > 10) & (nrun <= 100)).sum()),
                          f"101-{runs - 1}": int(((nrun > 100) & (nrun < runs)).sum()),
                          str(runs): int((nrun >= runs).sum())},
            "per_s": perms / (stage[2] * 1e-3),
            # the adds run as FP32 pre-filter gathers (FP64 only near ties); the kernel is bound
            # by LDS gathers and their latency, the FLOP figure is the survey's normalisation
            "roofline": {"bound": "LDS / latency", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": ach / FP64_PEAK_TFLOPS, "kernel": "k_css_perm (HIP events)",
                         "kernel_ms": stage[2]}}
    return out


def cpu_baseline(args):
    """Reference threadcompute() (64 pthreads) on a sample of the same workload."""
    from gdscan import synth

    ref = ROOT / "oracle" / "_ref" / "libref_fisher.so"
    orc = ROOT / "oracle" / "_build" / "liboracle.so"
    DP = np.ctypeslib.ndpointer(np.float64, flags="C")
    IP = np.ctypeslib.ndpointer(np.int32, flags="C")
    C = ctypes
    if ref.exists():
        lib = C.CDLL(str(ref))
        fn = lib.threadcompute
        fn.argtypes = [DP, DP, IP, IP] + [C.c_int] * 6 + [C.c_double, DP, DP]
        kind, cores = "reference", 64
    else:
        lib = C.CDLL(str(orc))
        fn = lib.orc_fet_scan
        fn.argtypes = [DP, DP, IP, IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_uint64,
                       C.c_int, DP, DP]
        kind, cores = "port", 1
    total_w = 0
    total_t = 0.0
    for c in range(args.cpu_chroms):
        av, bv, ap_, bp, regend = synth.chromosome(c, args.nsnp, args.asize, args.bsize)
        n = regend // args.wstep
        s = np.zeros(n)
        d = np.zeros(n)
        # the reference prints progress on C stdout: silence it around the call
        sys.stdout.flush()
        saved = os.dup(1)
        devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)
        try:
            t0 = time.perf_counter()
            if kind == "reference":
                fn(av, bv, ap_, bp, 0, regend, args.wsize, args.wstep, len(av), len(bv), args.perc, s, d)
            else:
                fn(av, bv, ap_, bp, regend, args.wsize, args.wstep, len(av), len(bv), args.perc, 1, 0, s, d)
            total_t += time.perf_counter() - t0
        finally:
            os.dup2(saved, 1)
            os.close(saved)
            os.close(devnull)
        from gdscan import fet
        total_w += fet.window_count(regend, args.wsize, args.wstep)
    return {
        "value": total_w / total_t,
        "unit": "windows/s",
        "cores": cores,
        "kind": kind,
        "sample": f"{args.cpu_chroms} of the {args.nchrom} chromosomes ({args.nsnp} SNPs, "
                  f"{args.asize}+{args.bsize}), {total_w} windows in {total_t:.2f} s"
                  + (" with the reference's 64 pthreads" if kind == "reference" else ", 1 thread"),
    }


def regions_run(args, scores, stddev, chroms, nch, rank, world, dev):
    """FilterFisherScores on the FET track just computed, kept in HBM:
    the tabular track (windows with score != 0), its limit (cmedian + scoreatpercentile)
    and the merged segments.  Timed end to end per call (host sync included)."""
    import torch
    from gdscan._lib import GD_SELECT_GE
    from gdscan.regions import fet_region_limit, merge_regions
    wcount = [chroms[c].regend // args.wstep for c in range(nch)]
    seq_all = torch.repeat_interleave(torch.arange(nch, dtype=torch.int32, device=dev),
                                      torch.tensor(wcount, device=dev))
    start_all = torch.cat([torch.arange(w, dtype=torch.int64, device=dev) * args.wstep for w in wcount])
    keep = scores != 0
    sc, sd, seq, start = scores[keep], stddev[keep], seq_all[keep], start_all[keep]
    ends = torch.tensor([chroms[c].regend - 1 for c in range(nch)], dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run():
        lim = fet_region_limit(sc, sd, 0.999, 75.0, stream=stream)
        return lim, merge_regions(sc, seq, start, GD_SELECT_GE, lim[0], 100000, ends, stream=stream)

    run()
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        lim, (first, end, ns) = run()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    res = {"what": "FilterFisherScores (limit + merge) on the device-resident FET track, 1 call",
           "windows": int(sc.numel()), "ms": ms, "windows_per_s": sc.numel() / (ms * 1e-3),
           "limit": lim[0], "selected": ns, "regions": int(len(first))}
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import regions_oracle as ro
        h_sc, h_sd = sc.cpu().numpy(), sd.cpu().numpy()
        h_seq, h_start = seq.cpu().numpy(), start.cpu().numpy()
        names = [str(k) for k in range(nch)]
        c0 = time.perf_counter()
        want = ro.filter_limit(h_sc, h_sd, 0.999, 75.0)
        regs = ro.merge_regions([names[k] for k in h_seq], h_start, h_sc >= want[0], 100000,
                                lambda s: chroms[int(s)].regend - 1)
        cpu_ms = (time.perf_counter() - c0) * 1e3
        res["cpu_baseline"] = {"value": sc.numel() / (cpu_ms * 1e-3), "unit": "windows/s", "cores": 1,
                               "kind": "port", "sample": f"the whole track ({sc.numel()} windows), numpy + "
                               "Python loop restatement (oracle/regions_oracle.py)"}
        res["parity"] = bool(want[0] == lim[0] and [(int(f), int(e)) for f, e in zip(first, end)] == regs)
    return res


def packed_run(args, lib, _lib, check, ctx, stream, dev, avals, bvals, apos, bpos, chroms, nch, scores, stddev):
    """The same FET scan from packed genotype tracks: the device-
    resident tracks packed on the device (2-bit codes, one position per row), then scanned
    with gd_fet_scan_packed_device; outputs must equal the reference-layout scan's bit for
    bit.  Reported beside the headline, never as `value` (a different input format)."""
    import torch
    from gdscan._lib import PChrom
    a, b, nsnp = args.asize, args.bsize, args.nsnp
    wa, wb = (a + 31) // 32, (b + 31) // 32
    ac = torch.zeros(nch * nsnp * wa, dtype=torch.int64, device=dev)
    bc = torch.zeros(nch * nsnp * wb, dtype=torch.int64, device=dev)
    rp = torch.zeros(nch * nsnp, dtype=torch.int32, device=dev)
    pcs = (PChrom * nch)()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(nch):
        check(lib.gd_pack_chrom_device(avals.data_ptr() + c * nsnp * a * 8, bvals.data_ptr() + c * nsnp * b * 8,
                                       apos.data_ptr() + c * nsnp * a * 4, bpos.data_ptr() + c * nsnp * b * 4, a, b,
                                       nsnp, ac.data_ptr() + c * nsnp * wa * 8, bc.data_ptr() + c * nsnp * wb * 8,
                                       rp.data_ptr() + c * nsnp * 4, stream))
        q = pcs[c]
        q.row_off, q.a_word, q.b_word = c * nsnp, c * nsnp * wa, c * nsnp * wb
        q.nrows, q.asize, q.bsize, q.regend = nsnp, a, b, chroms[c].regend
        q.w_out, q.seed = chroms[c].w_out, chroms[c].seed
    torch.cuda.synchronize()
    pack_ms = (time.perf_counter() - t0) * 1e3
    ps, pd = torch.zeros_like(scores), torch.zeros_like(stddev)

    def step():
        check(lib.gd_fet_scan_packed_device(ctx, pcs, nch, ac.data_ptr(), bc.data_ptr(), rp.data_ptr(), args.wsize,
                                            args.wstep, args.perc, lib.gd_get_fet_mode(), _lib.GD_WINDOWS_THREADED,
                                            ps.data_ptr(), pd.data_ptr(), stream))

    step()
    torch.cuda.synchronize()
    n = max(1, args.steps // 2)
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / n
    windows = sum(lib.gd_window_count(chroms[c].regend, args.wsize, args.wstep, _lib.GD_WINDOWS_THREADED)
                  for c in range(nch))
    ref_bytes = 12 * nch * nsnp * (a + b)
    packed_bytes = 8 * nch * nsnp * (wa + wb) + 4 * nch * nsnp
    return {"what": "FET scan from packed genotype tracks (2-bit codes, one position per row), device-resident",
            "ms_per_step": ms, "windows_per_s": windows / (ms * 1e-3), "steps": n, "pack_ms": pack_ms,
            "input_bytes": packed_bytes, "reference_layout_bytes": ref_bytes,
            "parity": bool(torch.equal(ps, scores) and torch.equal(pd, stddev))}, (ac, bc, rp, pcs)


def host_run(args, lib, _lib, check, avals, bvals, apos, bpos, chroms, nch, scores, stddev, codes):
    """The boundary as the reference's callers use it: inputs in (pageable) host memory,
    outputs back in host memory, PCIe transfers inside the timed call
    (gd_fet_scan_host_batch: f64 value + i32 position per genotype; gd_fet_scan_packed_host:
    2-bit codes + one position per row).  A sample of the rank's chromosomes; reported
    beside the headline, never as `value`."""
    import numpy as np
    import torch
    from gdscan._lib import Chrom
    a, b, nsnp = args.asize, args.bsize, args.nsnp
    nh = min(nch, 4)
    na, nb = nh * nsnp * a, nh * nsnp * b
    av, bv = avals[:na].cpu().numpy(), bvals[:nb].cpu().numpy()
    ap, bp = apos[:na].cpu().numpy(), bpos[:nb].cpu().numpy()
    hc = (Chrom * nh)()
    nw = 0
    for c in range(nh):
        hc[c] = chroms[c]
        nw = max(nw, chroms[c].w_out + chroms[c].regend // args.wstep)
    windows = sum(lib.gd_window_count(chroms[c].regend, args.wsize, args.wstep, _lib.GD_WINDOWS_THREADED)
                  for c in range(nh))
    ref_s, ref_d = scores[:nw].cpu().numpy(), stddev[:nw].cpu().numpy()
    ac, bc, rp, pcs = codes
    wa, wb = (a + 31) // 32, (b + 31) // 32
    hac = ac[:nh * nsnp * wa].cpu().numpy()
    hbc = bc[:nh * nsnp * wb].cpu().numpy()
    hrp = rp[:nh * nsnp].cpu().numpy()

    def timed(call, reps=3):
        best = None
        for _ in range(reps + 1):  # the first call sizes the context's staging buffers
            s_, d_ = np.zeros(nw), np.zeros(nw)
            t0 = time.perf_counter()
            call(s_, d_)
            dt = time.perf_counter() - t0
            best = dt if best is None or dt < best else best
        return best, s_, d_

    import ctypes as C
    pd_ = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))
    pi_ = lambda x: x.ctypes.data_as(C.POINTER(C.c_int))
    pv_ = lambda x: x.ctypes.data
    t_ref, s1, d1 = timed(lambda s_, d_: check(lib.gd_fet_scan_host_batch(
        hc, nh, pd_(av), pd_(bv), pi_(ap), pi_(bp), args.wsize, args.wstep, args.perc, _lib.GD_WINDOWS_THREADED,
        pd_(s_), pd_(d_))))
    t_pk, s2, d2 = timed(lambda s_, d_: check(lib.gd_fet_scan_packed_host(
        pcs, nh, pv_(hac), pv_(hbc), pv_(hrp), args.wsize, args.wstep, args.perc, lib.gd_get_fet_mode(),
        _lib.GD_WINDOWS_THREADED, pd_(s_), pd_(d_))))
    ref_bytes = 12 * (na + nb) + 16 * nw
    pk_bytes = 8 * nh * nsnp * (wa + wb) + 4 * nh * nsnp + 16 * nw
    return {"what": "FET scan called with host buffers (PCIe transfers inside the call), best of 3",
            "sample": f"{nh} chromosomes x {nsnp} SNPs ({a}+{b}), {windows} windows",
            "reference_layout": {"ms": t_ref * 1e3, "windows_per_s": windows / t_ref,
                                 "host_bytes": ref_bytes, "GB_per_s": ref_bytes / t_ref / 1e9},
            "packed": {"ms": t_pk * 1e3, "windows_per_s": windows / t_pk,
                       "host_bytes": pk_bytes, "GB_per_s": pk_bytes / t_pk / 1e9},
            "parity": bool(np.array_equal(s1, ref_s) and np.array_equal(d1, ref_d)
                           and np.array_equal(s2, ref_s) and np.array_equal(d2, ref_d))}


def main():
    args = parse()
    import torch

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist_mod
        dist_mod.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = dist_mod

    from gdscan import _lib, synth
    from gdscan._lib import Chrom, check, lib

    dev = torch.device("cuda", local)
    a, b, nsnp, nch = args.asize, args.bsize, args.nsnp, args.nchrom
    alen, blen = nsnp * a, nsnp * b
    avals = torch.empty(nch * alen, dtype=torch.float64, device=dev)
    bvals = torch.empty(nch * blen, dtype=torch.float64, device=dev)
    apos = torch.empty(nch * alen, dtype=torch.int32, device=dev)
    bpos = torch.empty(nch * blen, dtype=torch.int32, device=dev)
    qtab = torch.from_numpy(synth.freq_table()).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for c in range(nch):
        gc = rank * nch + c
        check(lib.gd_synth_device(gc, nsnp, a, b, synth.MASTER_SEED, qtab.data_ptr(),
                                  avals.data_ptr() + c * alen * 8, bvals.data_ptr() + c * blen * 8,
                                  apos.data_ptr() + c * alen * 4, bpos.data_ptr() + c * blen * 4, stream))
    torch.cuda.synchronize()
    # regend of each chromosome = last position + 1
    last = apos.view(nch, alen)[:, -1].cpu().numpy().astype(np.int64)
    chroms = (Chrom * nch)()
    w_out = 0
    windows = 0
    for c in range(nch):
        regend = int(last[c]) + 1
        chroms[c].a_off = c * alen
        chroms[c].b_off = c * blen
        chroms[c].alen = alen
        chroms[c].blen = blen
        chroms[c].regend = regend
        chroms[c].w_out = w_out
        chroms[c].seed = synth.MASTER_SEED + rank * nch + c
        w_out += regend // args.wstep
        windows += lib.gd_window_count(regend, args.wsize, args.wstep, _lib.GD_WINDOWS_THREADED)
    scores = torch.zeros(w_out, dtype=torch.float64, device=dev)
    stddev = torch.zeros(w_out, dtype=torch.float64, device=dev)
    ctx = lib.gd_ctx_create(local)
    assert ctx, "gd_ctx_create failed"

    def step():
        check(lib.gd_fet_scan_device(ctx, chroms, nch, avals.data_ptr(), bvals.data_ptr(), apos.data_ptr(),
                                     bpos.data_ptr(), args.wsize, args.wstep, args.perc,
                                     _lib.GD_WINDOWS_THREADED, scores.data_ptr(), stddev.data_ptr(), stream))

    for _ in range(args.warmup):
        step()
    stage = np.zeros(_lib.GD_NSTAGES)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        stage += np.array(_lib.last_stage_ms())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stage /= args.steps
    ms_per_step = elapsed * 1e3 / args.steps
    gather_ms = None
    if dist:
        # the one collective of the path: all ranks' (score, stddev) tracks gathered in
        # genome order; measured once, outside the timed steps
        from gdscan.shard import gather_tracks
        wt = torch.zeros(world * nch, dtype=torch.int64, device=dev)
        wt[rank * nch:(rank + 1) * nch] = torch.tensor([chroms[c].regend // args.wstep for c in range(nch)])
        dist.all_reduce(wt)  # every rank learns every chromosome's window count
        shards = [list(range(r * nch, (r + 1) * nch)) for r in range(world)]
        local = torch.stack([scores, stddev], 1)
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        gather_tracks(local, shards, wt.tolist())
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3
    total_windows = windows * world
    value = total_windows * args.steps / elapsed

    kernel_ms = float(stage[_lib.GD_NSTAGES - 1])  # first kernel -> last kernel of the scan
    alg_bytes = 12.0 * (nch * (alen + blen)) + 16.0 * windows
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    out = {
        "metric": "FET genomic windows/sec (10M SNPs, 20+20 indiv, 2.5 kb windows; per-GPU batch)",
        "value": value,
        "unit": "windows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded generator, SURVEY.md 8(d)), generated on device",
        "config": {
            "workload": "FET genome-wide, configs[1]: 20 chromosomes x 500k SNPs per GPU, 20+20 individuals, "
                        "wsize 2500, wstep 500, perc 0.95, 100 bootstrap replicates",
            "chromosomes_per_gpu": nch, "snps_per_gpu": nch * nsnp, "windows_per_gpu": windows,
            "asize": a, "bsize": b, "parallelism": f"window-sharded x{world} (whole chromosomes per rank)",
            "track_gather_ms": gather_ms,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": None,
            "kernel": "whole scan pipeline (k_popsize, k_bounds, k_snp_fet, k_fet_window_fast; k_fet_lut_* "
                      "when the score table is cold), HIP events on the scan's streams per step",
            "alg_bytes_per_step": alg_bytes,
            "stage_ms": {"hbm_passes_done": stage[0], "fast_windows_done": stage[1],
                         "general_path": stage[2], "scan_total": stage[3]},
        },
    }
    if TRAFFIC_FILE.exists():
        tr = json.loads(TRAFFIC_FILE.read_text())
        if tr.get("config") == [nch, nsnp, a, b]:
            out["roofline"]["traffic"] = tr["bytes_per_scan"]
            out["roofline"]["traffic_source"] = f"{TRAFFIC_FILE.relative_to(ROOT)} ({tr['method']})"
    if VALU_FILE.exists():
        # the binding resource of the scan: VALU issue (the bootstrap's nrand48 draws),
        # not HBM -- wave-instructions per scan (PMC SQ_INSTS_VALU, committed profile)
        # over this run's scan time, against the VALU issue peak
        vr = json.loads(VALU_FILE.read_text())
        if vr.get("config") == [nch, nsnp, a, b]:
            ginst = vr["valu_wave_insts_per_scan"] / (stage[3] * 1e-3) / 1e9
            out["roofline"]["valu"] = {
                "bound": "valu-issue", "achieved": ginst, "peak": VALU_PEAK_GINSTS, "unit": "G wave-insts/s",
                "frac": ginst / VALU_PEAK_GINSTS, "insts_per_scan": vr["valu_wave_insts_per_scan"],
                "source": f"{VALU_FILE.relative_to(ROOT)} ({vr['method']})"}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args)

    if not args.no_extra:
        out["regions"] = regions_run(args, scores, stddev, chroms, nch, rank, world, dev)
        out["packed"], codes = packed_run(args, lib, _lib, check, ctx, stream, dev, avals, bvals, apos, bpos, chroms,
                                          nch, scores, stddev)
        if rank == 0 and world == 1:
            out["host_path"] = host_run(args, lib, _lib, check, avals, bvals, apos, bpos, chroms, nch, scores, stddev,
                                        codes)
        del codes

    if not args.no_css:
        pv = torch.zeros_like(scores)

        def css_step():
            check(lib.gd_css_scan_device(ctx, chroms, nch, avals.data_ptr(), bvals.data_ptr(), apos.data_ptr(),
                                         bpos.data_ptr(), args.wsize, args.wstep, 10, 0, _lib.GD_WINDOWS_THREADED,
                                         scores.data_ptr(), pv.data_ptr(), stream))

        css_step()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kms = 0.0
        for _ in range(args.css_steps):
            css_step()
            kms += _lib.last_stage_ms()[1]  # the CSS window kernel (bit planes -> scores)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        css_elapsed = time.perf_counter() - t0
        if dist:
            t = torch.tensor([css_elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            css_elapsed = float(t.item())
        kms /= args.css_steps
        m = a + b
        flops = (4.0 / 3.0 * m ** 3 + 10.0 * m * m) * windows
        ach = flops / (kms * 1e-3) / 1e12
        out["css"] = {
            "metric": "CSS genomic windows/sec (classical MDS, runs=0; per-GPU batch)",
            "value": windows * world * args.css_steps / css_elapsed,
            "unit": "windows/s",
            "ms_per_step": css_elapsed * 1e3 / args.css_steps,
            "steps": args.css_steps,
            "config": {"workload": f"CSS, configs[2] shape: {nch} chromosomes x {nsnp} SNPs per GPU, {a}+{b} "
                                   f"individuals, wsize {args.wsize}, wstep {args.wstep}, mcR=0",
                       "windows_per_gpu": windows},
            "roofline": {"bound": "fp64-valu", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": ach / FP64_PEAK_TFLOPS, "traffic": None,
                         "kernel": "k_css_pack + k_css_mds (HIP events)", "kernel_ms": kms,
                         "alg_flops_per_window": flops / windows},
        }
        if CSS_VALU_FILE.exists():
            # what binds the MDS kernel: VALU issue -- per-window serial phases (Householder
            # steps, Sturm bisection, inverse iteration, back-transformation) on a wave whose
            # lanes hold the matrix rows (40 of 64 busy at m = 40)
            cv = json.loads(CSS_VALU_FILE.read_text())
            if cv.get("config") == [nch, nsnp, a, b]:
                gi = cv["valu_wave_insts_per_scan"] / (kms * 1e-3) / 1e9
                out["css"]["roofline"]["valu"] = {
                    "bound": "valu-issue", "achieved": gi, "peak": VALU_PEAK_GINSTS, "unit": "G wave-insts/s",
                    "frac": gi / VALU_PEAK_GINSTS, "insts_per_window": cv["valu_wave_insts_per_scan"] / windows,
                    "source": f"{CSS_VALU_FILE.relative_to(ROOT)} ({cv['method']})"}
        if rank == 0 and world == 1 and not args.no_cpu:
            out["css"]["cpu_baseline"] = css_cpu_baseline(args)
        # the per-GPU shapes of configs[3] (40+40, runs=0) and configs[4] (40+40, mcT=10,
        # mcR=1000) on a few chromosomes of their own: windows/s per GPU
        del avals, bvals, apos, bpos
        out["css"]["c4_shape"] = css_shape_run(args, lib, _lib, synth, Chrom, check, dev, stream, ctx, rank,
                                               nchrom=4, pop=40, treshold=10, runs=0)
        out["css"]["c5_shape"] = css_shape_run(args, lib, _lib, synth, Chrom, check, dev, stream, ctx, rank,
                                               nchrom=1, pop=40, treshold=10, runs=1000)
    lib.gd_ctx_destroy(ctx)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
