#!/usr/bin/env python3
"""Benchmark: genome-wide FET and CSS window scans on MI355X (BASELINE.json configs).

Headline (`value`): one step = one device-resident FET scan (per-SNP Fisher exact test,
window 95th-percentile score, 100-replicate bootstrap stddev) over this rank's batch of
synthetic chromosomes: configs[1], 20 chromosomes x 500k SNPs, 20+20 individuals, 2.5 kb
windows / 500 bp step (10M SNPs, ~1M windows per GPU).  Inputs are generated on the device
before timing; weak scaling: rank r scans chromosome ids 20r .. 20r+19, no data-path
collective; `value` = all ranks' windows / the max-over-ranks time.

Launch: `python bench.py --gpus N`.  With N > 1 and no torch.distributed environment the
script starts `torch.distributed.run` with N ranks (127.0.0.1) as a child process before
anything touches the GPU, and exits with its code.  `--backend gloo --dry-run` runs the
distributed plumbing (launcher, shard plans, the chromosome queue, the track gather) on
the CPU with no GPU work (tests/test_bench_launch.py).

Beside the headline (objects in the same JSON line):
  roofline      the FET scan's algorithmic HBM bytes B = 12 (alen + blen) + 16 W per step
                 over its kernel time (HIP events), measured traffic from
                the committed PMC profile, and the VALU-issue figure that actually binds it
  cpu_baseline  the reference's own threadcompute() (oracle/_ref, compiled from the
                reference sources; 64 pthreads on the host's cores) on all 20 chromosomes,
                plus `parity`: its scores against the GPU scores of the same windows
  css           configs[2] (C3: the same 20 chromosomes, 20+20, classical MDS, runs=0), and
  css.c4        configs[3] per-GPU share: 25 chromosomes x 500k SNPs per GPU at 40+40, runs=0,
                sharded over ranks by plan_shards, (score, p) track all-gathered and timed
  css.c5        configs[4] per-GPU share: the same at mcT=10, mcR=1000, chromosomes pulled
                from a shared queue (store counter) since the early-exit permutations make
                their cost data-dependent; permutation histogram and per-rank imbalance
  Each CSS leg carries an FP64 roofline (SURVEY.md 8(d) flops), the VALU figure from the
  committed PMC profile of the kernels it dispatches, and (N=1, rank 0) a cpu_baseline:
  the oracle port threaded over the host's cores (the reference CSS needs GSL, absent).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "fast-parallel-tools-for-genome-wide-analysis-of-genomic-divergence_amd"
sys.path.insert(0, str(PKG))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E spec
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec
# The one VALU ceiling every figure here uses: one wave64 instruction per SIMD per 2 cycles at the
# 2.4 GHz peak clock, 1024 SIMDs -- the rate of the fastest instruction class (the 2-cycle ops of
# tools/ubench_valu.hip: v_lshrrev_b32, v_add_f32, v_max_u16 ... 880-994 G/s at the held ~2.1 GHz).
# Multiplies, FP64 and VOP3 three-source ops are 4-cycle: a kernel made of them tops out at 0.5.
VALU_PEAK_GINSTS = 1024 * 2.4 / 2
PROFILE_ROUND = "r06"
PROF = ROOT / "profiles"
TRAFFIC_FILE = PROF / f"{PROFILE_ROUND}_fet_traffic.json"
VALU_FILE = PROF / f"{PROFILE_ROUND}_fet_valu.json"
CSS_VALU_FILE = PROF / f"{PROFILE_ROUND}_css_valu.json"
UBENCH_FILE = PROF / f"{PROFILE_ROUND}_ubench_valu.json"
CSS_PHASE_FILE = PROF / f"{PROFILE_ROUND}_css_phases.json"


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
    ap.add_argument("--cpu-chroms", type=int, default=20, help="chromosomes in the FET CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-css", action="store_true", help="skip the CSS legs")
    ap.add_argument("--no-c45", action="store_true", help="skip the C4/C5 CSS legs")
    ap.add_argument("--no-extra", action="store_true", help="skip the region-filter and packed-track legs")
    ap.add_argument("--css-steps", type=int, default=5, help="C3 timed steps (median reported)")
    ap.add_argument("--c45-chroms", type=int, default=25, help="C4/C5 chromosomes per GPU (configs[3]/[4]: 200/8)")
    ap.add_argument("--c45-steps", type=int, default=5, help="C4/C5 timed steps (median reported)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target wall time of each CSS CPU sample")
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--dry-run", action="store_true", help="distributed plumbing only, no GPU work (CPU tests)")
    ap.add_argument("--trace-hang", type=float, default=0.0,
                    help="dump every thread's Python stack to stderr every SECONDS (diagnostics)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise torch.distributed even at one rank (exercises the RCCL gathers on one GPU)")
    return ap.parse_args()


def maybe_launch(args):
    """--gpus N > 1 without a launcher: run torch.distributed.run as a child (no GPU call
    has happened yet in this process) and return its exit code; None when already a rank."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + sys.argv[1:]
    return subprocess.call(cmd)


def host_cpus():
    """(usable cores, nproc, CPU model): the affinity set, capped by a cgroup CPU quota and by
    OMP_NUM_THREADS when the box sets it (the GPU box's CPU share; nproc shows the machine)."""
    usable = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            usable = min(usable, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        usable = min(usable, int(os.environ["OMP_NUM_THREADS"]))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, os.cpu_count(), model


# ----------------------------------------------------------------------------- CPU baselines
def silenced(fn):
    """Run fn() with C stdout sent to /dev/null (the reference prints progress)."""
    sys.stdout.flush()
    saved = os.dup(1)
    devnull = os.open(os.devnull, os.O_WRONLY)
    os.dup2(devnull, 1)
    try:
        return fn()
    finally:
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)


def fet_cpu_baseline(args, scores_dev, chroms):
    """The reference's threadcompute() (64 pthreads) on the same chromosomes; its scores
    (seed-independent) are compared with the GPU scores of the same windows."""
    from gdscan import fet, synth
    ref = ROOT / "oracle" / "_ref" / "libref_fisher.so"
    orc = ROOT / "oracle" / "_build" / "liboracle.so"
    DP = np.ctypeslib.ndpointer(np.float64, flags="C")
    IP = np.ctypeslib.ndpointer(np.int32, flags="C")
    C = ctypes
    if ref.exists():
        lib = C.CDLL(str(ref))
        fn = lib.threadcompute
        fn.argtypes = [DP, DP, IP, IP] + [C.c_int] * 6 + [C.c_double, DP, DP]
        kind = "reference"
    else:
        lib = C.CDLL(str(orc))
        fn = lib.orc_fet_scan
        fn.argtypes = [DP, DP, IP, IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_uint64,
                       C.c_int, DP, DP]
        kind = "port"
    usable, nproc, model = host_cpus()
    gpu = scores_dev.cpu().numpy()
    total_w = 0
    total_t = 0.0
    nwin = exact = 0
    max_rel = 0.0
    ncpu = min(args.cpu_chroms, len(chroms))
    for c in range(ncpu):
        av, bv, ap_, bp, regend = synth.chromosome(c, args.nsnp, args.asize, args.bsize)
        n = regend // args.wstep
        s, d = np.zeros(n), np.zeros(n)

        def call():
            t0 = time.perf_counter()
            if kind == "reference":
                fn(av, bv, ap_, bp, 0, regend, args.wsize, args.wstep, len(av), len(bv), args.perc, s, d)
            else:
                fn(av, bv, ap_, bp, regend, args.wsize, args.wstep, len(av), len(bv), args.perc, 1, 0, s, d)
            return time.perf_counter() - t0

        total_t += silenced(call)
        total_w += fet.window_count(regend, args.wsize, args.wstep)
        g = gpu[chroms[c].w_out:chroms[c].w_out + n]
        comp = (s != 0) | (g != 0)
        nwin += int(comp.sum())
        exact += int((s[comp] == g[comp]).sum())
        rel = np.abs(s[comp] - g[comp]) / np.maximum(np.abs(s[comp]), 1e-300)
        max_rel = max(max_rel, float(rel.max()) if rel.size else 0.0)
    threads = 64 if kind == "reference" else 1
    return {
        "value": total_w / total_t, "unit": "windows/s", "cores": min(threads, usable), "kind": kind,
        "parity_windows": nwin, "parity_bit_exact_frac": exact / max(nwin, 1), "parity_max_rel": max_rel,
        "threads": threads, "cpu_model": model,
        "sample": f"{ncpu}/{args.nchrom} chromosomes, {total_w} windows in {total_t:.2f} s"
                  + (f", reference threadcompute, 64 pthreads on {min(64, usable)} cores" if kind == "reference"
                     else ", oracle, 1 thread"),
        "what": f"{kind} {'threadcompute (oracle/_ref, built from the reference sources)' if kind == 'reference' else 'orc_fet_scan'}"
                "; parity = its scores vs the GPU scores of the same windows (seed-independent; the reference's "
                "stddev is time-seeded)",
    }


def css_cpu_baseline(args, pop, treshold, runs):
    """The CSS oracle port (the reference CSS needs GSL, absent here) threaded over the host's
    usable cores: one chromosome prefix per thread (ctypes releases the GIL), each sized from
    a short calibration so the sample takes about --cpu-seconds of wall time."""
    from concurrent.futures import ThreadPoolExecutor
    from gdscan import fet, synth
    usable, nproc, model = host_cpus()
    threads = max(1, min(usable, 64))
    orc = ROOT / "oracle" / "_build" / "liboracle.so"
    DP = np.ctypeslib.ndpointer(np.float64, flags="C")
    IP = np.ctypeslib.ndpointer(np.int32, flags="C")
    C = ctypes
    lib = C.CDLL(str(orc))
    fn = lib.orc_css_scan
    fn.argtypes = [DP, DP, IP, IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                   C.c_int, DP, DP]

    def data(c, nsnp):
        av, bv, ap_, bp, regend = synth.chromosome(5000 + c, nsnp, pop, pop)
        n = regend // args.wstep
        return av, bv, ap_, bp, regend, np.zeros(n), np.zeros(n)

    def run(c, d):
        av, bv, ap_, bp, regend, s, p = d
        t0 = time.perf_counter()
        fn(av, bv, ap_, bp, regend, args.wsize, args.wstep, len(av), len(bv), treshold, runs, 1 + c, 0, s, p)
        return time.perf_counter() - t0, fet.window_count(regend, args.wsize, args.wstep)

    # calibration: one thread, a prefix long enough for the threaded window set (>= 103 steps)
    dt, w = run(0, data(0, 6_000))
    per_w = dt / max(w, 1)
    # ~10 new SNPs per 500-bp window step (mean gap 50 bp): SNPs for --cpu-seconds per thread
    nsnp = int(min(500_000, max(6_000, 10.0 * args.cpu_seconds / max(per_w, 1e-9))))
    inputs = [data(c, nsnp) for c in range(threads)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(lambda c: run(c, inputs[c]), range(threads)))
    wall = time.perf_counter() - t0
    win = sum(r[1] for r in res)
    return {"value": win / wall, "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": f"{threads} x {nsnp}-SNP prefixes, {win} windows in {wall:.2f} s"}


# ----------------------------------------------------------------------------- FET extras
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
    res = {"windows": int(sc.numel()), "ms": ms, "windows_per_s": sc.numel() / (ms * 1e-3),
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
                               "kind": "port", "sample": "whole track, oracle/regions_oracle.py"}
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
    return {"ms_per_step": ms, "windows_per_s": windows / (ms * 1e-3), "steps": n, "pack_ms": pack_ms,
            "input_bytes": packed_bytes, "reference_layout_bytes": ref_bytes,
            "parity": bool(torch.equal(ps, scores) and torch.equal(pd, stddev))}, (ac, bc, rp, pcs)


def host_run(args, lib, _lib, check, avals, bvals, apos, bpos, chroms, nch, scores, stddev, codes):
    """The boundary as the reference's callers use it: inputs in (pageable) host memory,
    outputs back in host memory, PCIe transfers inside the timed call
    (gd_fet_scan_host_batch: f64 value + i32 position per genotype; gd_fet_scan_packed_host:
    2-bit codes + one position per row).  A sample of the rank's chromosomes; reported
    beside the headline, never as `value`."""
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

    C = ctypes
    pd_ = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))
    pi_ = lambda x: x.ctypes.data_as(C.POINTER(C.c_int))
    pv_ = lambda x: x.ctypes.data
    ref_call = lambda s_, d_: check(lib.gd_fet_scan_host_batch(
        hc, nh, pd_(av), pd_(bv), pi_(ap), pi_(bp), args.wsize, args.wstep, args.perc, _lib.GD_WINDOWS_THREADED,
        pd_(s_), pd_(d_)))
    t_ref, s1, d1 = timed(ref_call)  # packed on host threads inside the call (gd_api.hip host_packed)
    os.environ["GD_HOST_NOPACK"] = "1"
    try:
        t_raw, s3, d3 = timed(ref_call)  # the reference layout across PCIe (12 B per genotype)
    finally:
        os.environ.pop("GD_HOST_NOPACK", None)
    t_pk, s2, d2 = timed(lambda s_, d_: check(lib.gd_fet_scan_packed_host(
        pcs, nh, pv_(hac), pv_(hbc), pv_(hrp), args.wsize, args.wstep, args.perc, lib.gd_get_fet_mode(),
        _lib.GD_WINDOWS_THREADED, pd_(s_), pd_(d_))))
    ref_bytes = 12 * (na + nb) + 16 * nw
    pk_bytes = 8 * nh * nsnp * (wa + wb) + 4 * nh * nsnp + 16 * nw
    usable, _, _ = host_cpus()
    return {"sample": f"{nh} x {nsnp} SNPs, {windows} windows, host buffers, best of 3",
            "reference_layout": {"ms": t_ref * 1e3, "windows_per_s": windows / t_ref,
                                 "host_bytes": ref_bytes, "GB_per_s": ref_bytes / t_ref / 1e9,
                                 "how": f"packed on {min(usable, 16)} host threads inside the call, 2 bits per "
                                        "genotype + 4 B per row across PCIe"},
            "reference_layout_unpacked": {"ms": t_raw * 1e3, "windows_per_s": windows / t_raw,
                                          "GB_per_s": ref_bytes / t_raw / 1e9, "how": "GD_HOST_NOPACK=1"},
            "packed": {"ms": t_pk * 1e3, "windows_per_s": windows / t_pk,
                       "host_bytes": pk_bytes, "GB_per_s": pk_bytes / t_pk / 1e9},
            "parity": bool(np.array_equal(s1, ref_s) and np.array_equal(d1, ref_d)
                           and np.array_equal(s2, ref_s) and np.array_equal(d2, ref_d)
                           and np.array_equal(s3, ref_s) and np.array_equal(d3, ref_d))}


def c1_run(args):
    """configs[0] (FET, one synthetic chromosome: 50k SNPs, 10+10, 2.5 kb windows; the
    reference's Pthreads CPU path): the reference's own threadcompute (oracle/_ref, 64
    pthreads) and the drop-in call HyperBrowser makes, gdscan.fet.fisher_exact_tester
    (FisherExactScoreStat.py:51-58 -> fisher_cython_parallel.pyx:14-15), on the same host
    arrays -- per call: host packing, PCIe both ways, the scan -- plus one C2-sized chromosome
    (500k SNPs, 20+20) through the same call.  Scores compared bit for bit (seed-independent;
    the reference's stddev is time-seeded)."""
    from gdscan import fet, synth
    ref = ROOT / "oracle" / "_ref" / "libref_fisher.so"
    DP = np.ctypeslib.ndpointer(np.float64, flags="C")
    IP = np.ctypeslib.ndpointer(np.int32, flags="C")
    rfn = None
    if ref.exists():
        rl = ctypes.CDLL(str(ref))
        rfn = rl.threadcompute
        rfn.argtypes = [DP, DP, IP, IP] + [ctypes.c_int] * 6 + [ctypes.c_double, DP, DP]
    out = {}
    for key, (chrom, nsnp, a, b) in (("c1_50k_10x10", (0, 50_000, 10, 10)), ("chrom_500k_20x20", (1, 500_000, 20, 20))):
        av, bv, ap, bp, regend = synth.chromosome(chrom, nsnp, a, b)
        n = regend // args.wstep
        win = fet.window_count(regend, args.wsize, args.wstep)

        def best(fn, reps):
            t = None
            for _ in range(reps):
                s_, d_ = np.zeros(n), np.zeros(n)
                t0 = time.perf_counter()
                fn(s_, d_)
                dt = time.perf_counter() - t0
                t = dt if t is None or dt < t else t
            return t, s_, d_

        drop = lambda s_, d_: fet.fisher_exact_tester(av, bv, ap, bp, 0, regend, args.wsize, args.wstep, len(av),
                                                      len(bv), args.perc, s_, d_)
        best(drop, 1)  # context, pinned buffers
        t_gpu, sg, dg = best(drop, 5)
        os.environ["GD_HOST_NOPACK"] = "1"
        try:
            t_raw, _, _ = best(drop, 3)
        finally:
            os.environ.pop("GD_HOST_NOPACK", None)
        o = {"snps": nsnp, "individuals": f"{a}+{b}", "windows": win,
             "dropin": {"ms": t_gpu * 1e3, "windows_per_s": win / t_gpu,
                        "call": "gdscan.fet.fisher_exact_tester (host arrays in and out, packed on host threads)"},
             "dropin_unpacked": {"ms": t_raw * 1e3, "windows_per_s": win / t_raw, "how": "GD_HOST_NOPACK=1"}}
        if rfn is not None:
            t_ref, sr, _ = best(lambda s_, d_: silenced(lambda: rfn(av, bv, ap, bp, 0, regend, args.wsize, args.wstep,
                                                                    len(av), len(bv), args.perc, s_, d_)), 2)
            comp = (sr != 0) | (sg != 0)
            o["reference"] = {"ms": t_ref * 1e3, "windows_per_s": win / t_ref, "kind": "reference",
                              "call": "threadcompute (oracle/_ref, built from the reference sources), 64 pthreads",
                              "cores": min(64, host_cpus()[0])}
            o["parity_windows"] = int(comp.sum())
            o["parity_bit_exact"] = bool(np.array_equal(sr[comp], sg[comp]))
            o["speedup_vs_reference"] = t_ref / t_gpu
        out[key] = o
    return out


# ----------------------------------------------------------------------------- CSS legs
class Env:
    """What every leg needs: the library, this rank's device, stream, context, process group."""

    def __init__(self, args, rank, world, local, dist):
        import torch
        from gdscan import _lib, synth
        from gdscan._lib import Chrom, check, lib
        self.args, self.rank, self.world, self.dist = args, rank, world, dist
        if args.dry_run:
            lib = DryLib(lib)
        self.torch, self._lib, self.synth, self.Chrom, self.check, self.lib = torch, _lib, synth, Chrom, check, lib
        self.dev = torch.device("cpu") if args.dry_run else torch.device("cuda", local)
        # gloo (ranks sharing a GPU, or --backend gloo) reduces host tensors; RCCL device ones
        self.cdev = torch.device("cpu") if (dist and dist.get_backend() == "gloo") or args.dry_run else self.dev
        self.stream = torch.cuda.current_stream(self.dev).cuda_stream
        self.ctx = lib.gd_ctx_create(local)
        assert self.ctx, "gd_ctx_create failed"

    def max_over_ranks(self, x):
        if not self.dist:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sync(self):
        self.torch.cuda.synchronize()
        if self.dist:
            self.dist.barrier()
        self.torch.cuda.synchronize()


def css_valu(shape_key, windows, kernel_ms):
    """VALU figures of a CSS leg from the committed PMC profile: wave-instructions per
    window of the kernels the leg dispatches over this run's kernel time (G/s), and the
    SIMDs' VALU busy fraction of the dominant kernel as the counters saw it."""
    if not CSS_VALU_FILE.exists():
        return {}
    doc = json.loads(CSS_VALU_FILE.read_text()).get(shape_key)
    if not doc or kernel_ms <= 0:
        return {}
    gi = doc["valu_wave_insts_per_window"] * windows / (kernel_ms * 1e-3) / 1e9
    return {"valu": {"achieved_ginsts": gi, "peak_ginsts": VALU_PEAK_GINSTS, "frac": gi / VALU_PEAK_GINSTS,
                     "insts_per_window": doc["valu_wave_insts_per_window"]}}


def dist_build(shape_key, m, kernel_ms, windows):
    """SURVEY.md 8(d)'s CSS distance-build figure: 4 m^2 npos integer ops per window
    (compare_all, css.c:277-327) over the time the bit planes (k_css_pack) plus the
    popcount distance build take -- the build's share of the MDS kernel from the
    committed GD_CSS_PROFILE phase profile, k_css_pack's share of the stage from the
    kernel trace.  The build runs on the VALU (64-bit AND + popcount over the bit planes,
    64 SNP products per instruction), not on the matrix cores, so no MFMA peak is quoted
    for it: the figure is its share of the window time and its integer-op rate."""
    if not CSS_PHASE_FILE.exists():
        return None
    doc = json.loads(CSS_PHASE_FILE.read_text()).get(shape_key)
    if not doc or kernel_ms <= 0:
        return None
    share = doc["pack_share"] + (1.0 - doc["pack_share"]) * doc["d_share"]
    ms = kernel_ms * share
    ops = 4.0 * m * m * doc["npos_mean"]
    return {"unit": "VALU popcount (bit-plane AND + popcount, no MFMA)", "int_ops_per_window": ops,
            "share_of_window_time": share, "ms": ms,
            "int_tops_valu": ops * windows / (ms * 1e-3) / 1e12 if ms > 0 else None,
            "pack_share": doc["pack_share"], "d_share_of_mds": doc["d_share"]}


def perm_stats(pm, computed, treshold, runs, perm_ms, pop):
    """Permutations actually run per window, from p = (hits + 1) / (run + 1): an early exit
    (hits = mcT) leaves p > mcT / (mcR + 1), a full run p <= mcT / (mcR + 1)."""
    p = pm[computed]
    early = p * (runs + 1) > treshold + 0.5
    nrun = np.where(early, np.rint((treshold + 1) / p) - 1, runs)
    perms = float(nrun.sum())
    return {"total": perms, "mean_per_window": float(nrun.mean()),
            "hist": [int((nrun <= 10).sum()), int(((nrun > 10) & (nrun <= 100)).sum()),
                     int(((nrun > 100) & (nrun < runs)).sum()), int((nrun >= runs).sum())],
            "per_s": perms / (perm_ms * 1e-3) if perm_ms > 0 else None, "kernel_ms": perm_ms}


def timed_steps(env, fn, steps):
    """Run fn() `steps` times, each bracketed by a barrier + sync; per step the max over
    ranks.  Returns the list of step seconds."""
    out = []
    for k in range(steps):
        env.sync()
        t0 = time.perf_counter()
        fn(k)
        env.sync()
        out.append(env.max_over_ranks(time.perf_counter() - t0))
    return out


def c3_leg(env, args, chroms, nch, windows, avals, bvals, apos, bpos, scores):
    """configs[2] shape on the FET leg's resident chromosomes (20+20, runs=0); median of
    --css-steps timed steps."""
    torch, lib, _lib, check = env.torch, env.lib, env._lib, env.check
    pv = torch.zeros_like(scores)
    kms = []

    def step(_k):
        check(lib.gd_css_scan_device(env.ctx, chroms, nch, avals.data_ptr(), bvals.data_ptr(), apos.data_ptr(),
                                     bpos.data_ptr(), args.wsize, args.wstep, 10, 0, _lib.GD_WINDOWS_THREADED,
                                     scores.data_ptr(), pv.data_ptr(), env.stream))
        kms.append(_lib.last_stage_ms()[1])  # bit planes -> scores (HIP events)

    step(-1)
    kms.clear()
    ts = timed_steps(env, step, args.css_steps)
    med = float(np.median(ts))
    kmed = float(np.median(kms))
    m = args.asize + args.bsize
    flops = (4.0 / 3.0 * m ** 3 + 10.0 * m * m) * windows
    out = {"value": windows * env.world / med, "unit": "windows/s", "ms_per_step": med * 1e3,
           "ms_mean": float(np.mean(ts)) * 1e3, "steps": args.css_steps,
           "workload": f"configs[2] shape: {nch} x {args.nsnp} SNPs per GPU, {args.asize}+{args.bsize}, runs=0",
           "windows_per_gpu": windows, "kernel_ms": kmed,
           "fp64_frac": flops / (kmed * 1e-3) / 1e12 / FP64_PEAK_TFLOPS if kmed > 0 else 0.0,
           "alg_flops_per_window": flops / max(windows, 1)}
    out.update(css_valu("c3", windows, kmed))
    db = dist_build("c3", m, kmed, windows)
    if db:
        out["distance_build"] = db
    if env.rank == 0 and not args.no_cpu and not args.dry_run:
        out["cpu_baseline"] = css_cpu_baseline(args, args.asize, 10, 0)
    return out


def c45_leg(env, args, name, treshold, runs, queue):
    """configs[3] (runs=0, static shards) / configs[4] (mcR=1000, shared queue) per-GPU share:
    args.c45_chroms chromosomes x 500k SNPs per GPU at 40+40; median of --c45-steps timed
    steps.  C4: each rank generates its plan_shards share once and scans it in one call.
    C5: ranks pull chromosome tickets from a store counter and the input moves with the
    ticket (queue_pull_pipelined): a rank generates only the chromosomes it pulls, into
    two rotating slots, the next one on a side stream while the current one scans -- its
    input memory is two chromosomes at any world size.  The (score, p) track of every
    rank is gathered to rank 0 after the timed steps (timed separately)."""
    from gdscan.shard import default_store, gather_lists, gather_tracks_to, plan_shards, queue_pull_pipelined
    torch, lib, _lib, check, synth = env.torch, env.lib, env._lib, env.check, env.synth
    pop, nsnp, world, rank = 40, args.nsnp, env.world, env.rank
    total = args.c45_chroms * world
    alen = nsnp * pop
    regends = [synth.regend(1000 + c, nsnp) for c in range(total)]  # positions only (host)
    wins = [g // args.wstep for g in regends]
    wcount = [lib.gd_window_count(g, args.wsize, args.wstep, _lib.GD_WINDOWS_THREADED) for g in regends]
    gofs = np.concatenate([[0], np.cumsum(wins)]).astype(np.int64)
    shards = plan_shards([nsnp] * total, world)
    nbuf = 2 if queue else len(shards[rank])
    av = torch.empty(nbuf * alen, dtype=torch.float64, device=env.dev)
    bv = torch.empty(nbuf * alen, dtype=torch.float64, device=env.dev)
    ap = torch.empty(nbuf * alen, dtype=torch.int32, device=env.dev)
    bp = torch.empty(nbuf * alen, dtype=torch.int32, device=env.dev)
    qtab = torch.from_numpy(synth.freq_table()).to(env.dev)
    gen = torch.cuda.Stream(env.dev)
    ready = [torch.cuda.Event() for _ in range(nbuf)]

    def generate(c, slot, stream):
        check(lib.gd_synth_device(1000 + c, nsnp, pop, pop, synth.MASTER_SEED, qtab.data_ptr(),
                                  av.data_ptr() + slot * alen * 8, bv.data_ptr() + slot * alen * 8,
                                  ap.data_ptr() + slot * alen * 4, bp.data_ptr() + slot * alen * 4, stream))

    def desc(slot, c, w_out, d):
        d.a_off = d.b_off = slot * alen
        d.alen = d.blen = alen
        d.regend = regends[c]
        d.w_out = w_out
        d.seed = synth.MASTER_SEED + 1000 + c

    # outputs: genome order (queue) / the rank's shard concatenated (static, gather layout)
    nout = int(gofs[-1]) if queue else sum(wins[c] for c in shards[rank])
    sc = torch.zeros(max(nout, 1), dtype=torch.float64, device=env.dev)
    pv = torch.zeros_like(sc)
    stage = [0.0, 0.0]
    one = (env.Chrom * 1)()

    def scan(ch, n):
        check(lib.gd_css_scan_device(env.ctx, ch, n, av.data_ptr(), bv.data_ptr(), ap.data_ptr(), bp.data_ptr(),
                                     args.wsize, args.wstep, treshold, runs, _lib.GD_WINDOWS_THREADED,
                                     sc.data_ptr(), pv.data_ptr(), env.stream))
        st = _lib.last_stage_ms()
        stage[0] += st[1]
        stage[1] += st[2]

    if not queue:
        mine = shards[rank]
        chroms = (env.Chrom * len(mine))()
        w = 0
        for i, c in enumerate(mine):
            generate(c, i, env.stream)
            desc(i, c, w, chroms[i])
            w += wins[c]
        torch.cuda.synchronize()
    store = default_store() if (queue and env.dist) else None
    tick = [0]

    def prepare(c, slot):
        generate(c, slot, gen.cuda_stream)
        ready[slot].record(gen)

    def work(c, slot):
        torch.cuda.current_stream(env.dev).wait_event(ready[slot])
        desc(slot, c, int(gofs[c]), one[0])
        scan(one, 1)  # returns after the scan's stream sync: the slot is free again

    class Local:  # one rank without a process group: the queue is the chromosome order
        def __init__(self):
            self.n = {}

        def add(self, key, v):
            self.n[key] = self.n.get(key, 0) + v
            return self.n[key]

    local_store = Local()

    done_last = []

    def step(k):
        nonlocal done_last
        if not queue:
            scan(chroms, len(shards[rank]))
            done_last = list(shards[rank])
        else:
            done_last = queue_pull_pipelined(store if store is not None else local_store, f"gd_{name}_{k}", total,
                                             prepare, work)

    step(-1)  # warmup (sizes the workspace)
    env.sync()
    stage[:] = [0.0, 0.0]
    ts = timed_steps(env, step, args.c45_steps)
    stage = [x / args.c45_steps for x in stage]
    med = float(np.median(ts))
    all_windows = sum(wcount)
    mine = done_last
    mine_w = sum(wcount[c] for c in mine)
    out = {"value": all_windows / med, "unit": "windows/s", "n_gpus": world, "ms_per_step": med * 1e3,
           "ms_mean": float(np.mean(ts)) * 1e3, "steps": args.c45_steps,
           "workload": f"{total} chromosomes x {nsnp} SNPs ({args.c45_chroms} per GPU), 40+40, mcT={treshold}, "
                       f"mcR={runs}", "windows": all_windows,
           "sharding": "store-counter ticket queue, input generated per pulled ticket (2 slots)" if queue
           else "plan_shards (LPT by SNP count), whole chromosomes per rank",
           "resident_input_bytes_per_rank": int(nbuf * alen * 24)}
    perm_ms = float(stage[1])
    if env.dist and runs > 0:  # GPU-time of the permutation kernel summed over ranks (every rank
        # takes part, before the ranks other than 0 return below)
        t = torch.tensor([perm_ms], dtype=torch.float64, device=env.cdev)
        env.dist.all_reduce(t)
        perm_ms = float(t.item())
    # the one collective: (score, p) of every rank's chromosomes, gathered to rank 0
    if env.dist:
        shard_done = gather_lists(mine) if queue else shards
        if queue:
            local = torch.cat([torch.stack([sc[gofs[c]:gofs[c + 1]], pv[gofs[c]:gofs[c + 1]]], 1) for c in mine]) \
                if mine else torch.zeros((0, 2), dtype=torch.float64, device=env.dev)
        else:
            local = torch.stack([sc[:nout], pv[:nout]], 1)
        env.sync()
        g0 = time.perf_counter()
        track = gather_tracks_to(local.to(env.cdev), shard_done, wins, dst=0)
        torch.cuda.synchronize()
        out["track_gather_ms"] = env.max_over_ranks((time.perf_counter() - g0) * 1e3)
        if queue:
            out["chromosomes_per_rank"] = [len(x) for x in shard_done]
            # the queue hands every chromosome to exactly one rank
            out["queue_each_once"] = sorted(c for x in shard_done for c in x) == list(range(total))
        if rank != 0:
            return out
        sc_all, p_all = track[:, 0], track[:, 1]
    else:
        sc_all, p_all = sc[:nout], pv[:nout]
    pm, sm = p_all.cpu().numpy(), sc_all.cpu().numpy()
    computed = sm != 0
    m = 2 * pop
    flops = (4.0 / 3.0 * m ** 3 + 10.0 * m * m)
    out["kernel_ms"] = float(stage[0])
    out["fp64_frac"] = flops * mine_w / (stage[0] * 1e-3) / 1e12 / FP64_PEAK_TFLOPS if stage[0] > 0 else 0.0
    out.update(css_valu("c4", mine_w, float(stage[0])))
    if not runs:
        db = dist_build("c4", m, float(stage[0]), mine_w)
        if db:
            out["distance_build"] = db
    out["mean_p"] = float(pm[computed].mean()) if computed.any() else None
    if runs > 0 and computed.any():
        out["permutations"] = perm_stats(pm, computed, treshold, runs, perm_ms, pop)
        pv_ = css_valu("c5_perm", mine_w, float(stage[1]))
        out["permutations"].update(pv_)
        doc = json.loads(CSS_VALU_FILE.read_text()).get("c5_perm", {}) if CSS_VALU_FILE.exists() else {}
        if "mfma" in doc and stage[1] > 0:
            mf = doc["mfma"]
            busy = mf["busy_simd_cycles_per_dispatch"] / doc["windows_per_dispatch"] * mine_w
            out["permutations"]["mfma_busy"] = busy / (1024 * 2.4e9 * stage[1] * 1e-3)
    if env.rank == 0 and not args.no_cpu and not args.dry_run:
        out["cpu_baseline"] = css_cpu_baseline(args, pop, treshold, runs)
    del av, bv, ap, bp
    return out


# ----------------------------------------------------------------------------- dry run (CPU)
class _DryStream:
    cuda_stream = 0

    def wait_event(self, _e):
        pass

    def synchronize(self):
        pass


class _DryEvent:
    def record(self, _stream=None):
        pass

    def synchronize(self):
        pass


def install_dry_cuda(torch):
    """--dry-run: the torch.cuda calls the legs make become no-ops on the CPU"""
    c = torch.cuda
    c.synchronize = lambda *a, **k: None
    c.current_stream = lambda *a, **k: _DryStream()
    c.Stream = lambda *a, **k: _DryStream()
    c.Event = lambda *a, **k: _DryEvent()
    c.empty_cache = lambda: None
    c.set_device = lambda *a, **k: None


class DryLib:
    """--dry-run: libgdscan with its device entry points as no-ops (status GD_OK); every other
    symbol (window counts, modes, stage times) is the real library's host code"""
    DEVICE = {"gd_ctx_create": 1, "gd_ctx_destroy": None, "gd_synth_device": 0, "gd_fet_scan_device": 0,
              "gd_css_scan_device": 0, "gd_pack_chrom_device": 0, "gd_fet_scan_packed_device": 0}

    def __init__(self, real):
        self._real = real

    def __getattr__(self, name):
        if name in DryLib.DEVICE:
            v = DryLib.DEVICE[name]
            return lambda *a: v
        return getattr(self._real, name)


def dry_run(args, rank, world, dist):
    """The distributed plumbing without a GPU: shard plan, the chromosome queue over the
    default store with the input moving with the ticket (queue_pull_pipelined: a rank
    materialises only what it pulls, at most two tickets at a time), the all-gather and the
    gather-to-rank-0 of the track (gloo), checked against the expected genome order."""
    import torch
    from gdscan.shard import (default_store, gather_lists, gather_tracks, gather_tracks_to, plan_shards,
                              queue_pull_pipelined)
    total = args.c45_chroms * world
    wins = [100 + 7 * c for c in range(total)]
    offs = np.concatenate([[0], np.cumsum(wins)])
    store = default_store()
    slots = {}
    made = []
    peak = [0]

    def prepare(c, slot):  # the "input" of ticket c: its window indices, produced only when pulled
        slots[slot] = (c, torch.arange(offs[c], offs[c + 1], dtype=torch.float64))
        made.append(c)
        peak[0] = max(peak[0], len(slots))

    parts = {}

    def work(c, slot):
        cc, data = slots[slot]
        assert cc == c
        time.sleep(0.001 * (1 + c % 3))
        parts[c] = torch.stack([data, data], 1)

    done = queue_pull_pipelined(store, "gd_dry", total, prepare, work)
    lists = gather_lists(done)
    assert sorted(c for s in lists for c in s) == list(range(total))
    local = torch.cat([parts[c] for c in done]) if done else torch.zeros((0, 2), dtype=torch.float64)
    want = torch.arange(offs[-1], dtype=torch.float64)
    track = gather_tracks(local, lists, wins)
    ok = bool(torch.equal(track[:, 0], want))
    t0 = gather_tracks_to(local, lists, wins, dst=0)
    ok0 = bool(torch.equal(t0[:, 1], want)) if rank == 0 else t0 is None
    ok0 = gather_lists([int(ok0)])
    made_all = gather_lists(made)
    shards = plan_shards([args.nsnp] * total, world)
    dist.barrier()
    return {"dry_run": True, "n_gpus": world, "backend": args.backend, "queue_per_rank":
            [len(s) for s in lists], "static_per_rank": [len(s) for s in shards], "gather_ok": ok,
            "gather_to_0_ok": all(x[0] == 1 for x in ok0),
            "materialised_only_pulled": all(sorted(m) == sorted(d) for m, d in zip(made_all, lists)),
            "max_live_inputs": peak[0]}


# ----------------------------------------------------------------------------- main
def note(rank, msg):
    """a progress line on stderr (rank 0): the JSON line on stdout stays the only output there"""
    if rank == 0:
        print(f"bench: {msg} ({time.strftime('%H:%M:%S')})", file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.trace_hang > 0:
        import faulthandler
        faulthandler.dump_traceback_later(args.trace_hang, repeat=True, file=sys.stderr)
    rc = maybe_launch(args)
    if rc is not None:
        sys.exit(rc)
    import torch

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    plumbing = None
    if args.dry_run:
        # the distributed plumbing checks, then every leg in the bench's real order with the
        # device work stubbed out (install_dry_cuda, DryLib): the same collectives, barriers
        # and queue pulls as a GPU run, on CPU tensors over gloo
        if world == 1:
            print(json.dumps({"dry_run": True, "n_gpus": 1}), flush=True)
            return
        import torch.distributed as dist_mod
        args.backend = "gloo"
        args.no_extra = args.no_cpu = True  # host-buffer and CPU-baseline legs need the device results
        dist_mod.init_process_group("gloo")
        dist = dist_mod
        plumbing = dry_run(args, rank, world, dist_mod)
        install_dry_cuda(torch)
    # more ranks than GPUs (a rehearsal of --gpus N on a smaller box): ranks share the
    # devices round-robin, and the collectives go over gloo (RCCL refuses two ranks on one
    # GPU); device_count() does not initialise the GPU
    from gdscan.shard import choose_backend
    ndev = 1 if args.dry_run else max(1, torch.cuda.device_count())
    args.backend, _on_device = choose_backend(world, ndev, args.backend)
    local = local % ndev
    torch.cuda.set_device(local)
    if (world > 1 or args.force_dist) and dist is None:
        import torch.distributed as dist_mod
        if world == 1:  # --force-dist: a one-rank group, so the collectives really run (RCCL on the GPU)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                sk = socket.socket()
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
                sk.close()
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.backend == "gloo":
            dist_mod.init_process_group("gloo")
        else:
            dist_mod.init_process_group(args.backend, device_id=torch.device("cuda", local))
        dist = dist_mod

    env = Env(args, rank, world, local, dist)
    lib, _lib, synth, check = env.lib, env._lib, env.synth, env.check
    dev, stream, ctx = env.dev, env.stream, env.ctx
    a, b, nsnp, nch = args.asize, args.bsize, args.nsnp, args.nchrom
    alen, blen = nsnp * a, nsnp * b
    avals = torch.empty(nch * alen, dtype=torch.float64, device=dev)
    bvals = torch.empty(nch * blen, dtype=torch.float64, device=dev)
    apos = torch.empty(nch * alen, dtype=torch.int32, device=dev)
    bpos = torch.empty(nch * blen, dtype=torch.int32, device=dev)
    qtab = torch.from_numpy(synth.freq_table()).to(dev)
    for c in range(nch):
        gc = rank * nch + c
        check(lib.gd_synth_device(gc, nsnp, a, b, synth.MASTER_SEED, qtab.data_ptr(),
                                  avals.data_ptr() + c * alen * 8, bvals.data_ptr() + c * blen * 8,
                                  apos.data_ptr() + c * alen * 4, bpos.data_ptr() + c * blen * 4, stream))
    torch.cuda.synchronize()
    # regend of each chromosome = last position + 1
    last = apos.view(nch, alen)[:, -1].cpu().numpy().astype(np.int64)
    if args.dry_run:  # no generator ran: the host restatement of its positions
        last = np.array([synth.regend(rank * nch + c, nsnp) - 1 for c in range(nch)], dtype=np.int64)
    chroms = (env.Chrom * nch)()
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

    def step():
        check(lib.gd_fet_scan_device(ctx, chroms, nch, avals.data_ptr(), bvals.data_ptr(), apos.data_ptr(),
                                     bpos.data_ptr(), args.wsize, args.wstep, args.perc,
                                     _lib.GD_WINDOWS_THREADED, scores.data_ptr(), stddev.data_ptr(), stream))

    note(rank, f"FET: {world} rank(s), {windows} windows per rank")
    for _ in range(args.warmup):
        step()
    stage = np.zeros(_lib.GD_NSTAGES)
    env.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        stage += np.array(_lib.last_stage_ms())
    env.sync()
    elapsed = env.max_over_ranks(time.perf_counter() - t0)
    stage /= args.steps
    ms_per_step = elapsed * 1e3 / args.steps
    gather_ms = None
    if dist:
        # the one collective of the path: all ranks' (score, stddev) tracks gathered in
        # genome order; measured once, outside the timed steps
        from gdscan.shard import gather_tracks_to
        wt = torch.zeros(world * nch, dtype=torch.int64, device=env.cdev)
        wt[rank * nch:(rank + 1) * nch] = torch.tensor([chroms[c].regend // args.wstep for c in range(nch)])
        dist.all_reduce(wt)  # every rank learns every chromosome's window count
        shards = [list(range(r * nch, (r + 1) * nch)) for r in range(world)]
        loc = torch.stack([scores, stddev], 1)
        env.sync()
        g0 = time.perf_counter()
        gather_tracks_to(loc.to(env.cdev), shards, wt.tolist(), dst=0)
        torch.cuda.synchronize()
        gather_ms = env.max_over_ranks((time.perf_counter() - g0) * 1e3)
    total_windows = windows * world
    value = total_windows * args.steps / elapsed

    kernel_ms = float(stage[_lib.GD_NSTAGES - 1])  # first kernel -> last kernel of the scan
    alg_bytes = 12.0 * (nch * (alen + blen)) + 16.0 * windows
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    sources = {}
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None, "alg_bytes_per_step": alg_bytes,
            "kernel_ms": kernel_ms, "kernel": "whole scan: k_fet_setup, k_bounds, k_fet_window_fast (HIP events)"}
    if TRAFFIC_FILE.exists():
        tr = json.loads(TRAFFIC_FILE.read_text())
        if tr.get("config") == [nch, nsnp, a, b]:
            roof["traffic"] = tr["bytes_per_scan"]
            sources["traffic"] = f"{TRAFFIC_FILE.relative_to(ROOT)}: {tr['method']}"
    if VALU_FILE.exists():
        # what binds the scan: VALU issue (the bootstrap's nrand48 draws), not HBM --
        # wave-instructions per scan (PMC SQ_INSTS_VALU, committed profile) over this run's
        # scan time against VALU_PEAK_GINSTS
        vr = json.loads(VALU_FILE.read_text())
        if vr.get("config") == [nch, nsnp, a, b] and kernel_ms > 0:
            gi = vr["valu_wave_insts_per_scan"] / (kernel_ms * 1e-3) / 1e9
            roof["valu"] = {"achieved_ginsts": gi, "peak_ginsts": VALU_PEAK_GINSTS, "frac": gi / VALU_PEAK_GINSTS,
                            "insts_per_scan": vr["valu_wave_insts_per_scan"],
                            "note": "peak = one wave64 instruction per SIMD per 2 cycles at 2.4 GHz (the 2-cycle "
                                    "class); the bootstrap draws are 4-cycle instructions, ceiling 0.5 of it"}
            sources["valu"] = f"{VALU_FILE.relative_to(ROOT)}: {vr['method']}"
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
            "workload": "FET configs[1]: 20 x 500k SNPs per GPU, 20+20, wsize 2500, wstep 500, perc 0.95, 100 reps",
            "chromosomes_per_gpu": nch, "snps_per_gpu": nch * nsnp, "windows_per_gpu": windows,
            "asize": a, "bsize": b, "parallelism": f"window-sharded x{world} (whole chromosomes per rank)",
            "ranks_per_gpu": -(-world // ndev), "collective_backend": args.backend if dist else None,
            "track_gather_ms": gather_ms,
        },
        "roofline": roof,
    }
    note(rank, f"FET: {ms_per_step:.3f} ms/step")
    if rank == 0 and not args.no_cpu and not args.dry_run:
        # after the timed region, at any world size: the other ranks wait at the next leg's barrier
        cb = fet_cpu_baseline(args, scores, chroms)
        sources["cpu_baseline"] = cb.pop("what")
        out["cpu_baseline"] = cb
    # HIP events of the last scans, from the scan's first kernel (include/gdscan.h GD_STAGE_*)
    out["stage_ms"] = {"prologue": float(stage[0]), "through_window_kernels": float(stage[1]),
                       "general_path": float(stage[2]), "scan": float(stage[3])}

    if not args.no_extra:
        note(rank, "region-filter and packed-track legs")
        out["regions"] = regions_run(args, scores, stddev, chroms, nch, rank, world, dev)
        out["packed"], codes = packed_run(args, lib, _lib, check, ctx, stream, dev, avals, bvals, apos, bpos, chroms,
                                          nch, scores, stddev)
        if rank == 0 and world == 1:
            out["host_path"] = host_run(args, lib, _lib, check, avals, bvals, apos, bpos, chroms, nch, scores, stddev,
                                        codes)
        if rank == 0 and not args.no_cpu:
            note(rank, "C1 (configs[0]) and the per-chromosome drop-in call")
            out["c1"] = c1_run(args)
        del codes

    if not args.no_css:
        note(rank, "CSS C3")
        css = {"c3": c3_leg(env, args, chroms, nch, windows, avals, bvals, apos, bpos, scores)}
        del avals, bvals, apos, bpos, scores, stddev
        torch.cuda.empty_cache()
        if not args.no_c45:
            note(rank, "CSS C4")
            css["c4"] = c45_leg(env, args, "c4", 10, 0, queue=False)
            torch.cuda.empty_cache()
            note(rank, "CSS C5")
            css["c5"] = c45_leg(env, args, "c5", 10, 1000, queue=True)
        out["css"] = css
        if CSS_VALU_FILE.exists():
            sources["css_valu"] = f"{CSS_VALU_FILE.relative_to(ROOT)} (SQ_INSTS_VALU per window over this run's " \
                                  "kernel time, against VALU_PEAK_GINSTS)"
        if CSS_PHASE_FILE.exists():
            sources["distance_build"] = f"{CSS_PHASE_FILE.relative_to(ROOT)} (GD_CSS_PROFILE phase cycles, " \
                                        "k_css_pack share from the kernel trace)"
        sources["css_cpu"] = "oracle/css_oracle.c threaded over the host cores (the reference CSS needs GSL, absent)"
    lib.gd_ctx_destroy(ctx)
    out["sources"] = sources
    if plumbing is not None:
        out.update(plumbing)
    if rank == 0:
        print(json.dumps(out, separators=(",", ":")), flush=True)
    if dist:
        dist.barrier()
        if args.dry_run:
            print(f"bench: rank {rank} reached the final barrier", file=sys.stderr, flush=True)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
