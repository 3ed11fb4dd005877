"""GPU parity: the HIP FET scan (through the C-ABI) against the oracle restatement.

Tolerance (north star): 1e-9 relative.  Integer work (window bounds, counts, the
nrand48 stream, order statistics) is exact; the only inexact step is -log10, which
reproduces glibc's formula over a correctly rounded log (<= 1 ulp apart on ~0.1% of
arguments), so scores are typically bit-identical and always within ~1e-15.
"""
import numpy as np
import pytest

from conftest import close, oracle_fet_scan

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["host_packed", "reference_layout"])
def _host_route(request, monkeypatch):
    """every host-API test twice: the drop-in calls pack whole-row genotype tracks on the host
    (gd_api.hip host_packed) -- and once with that route off, so the reference-layout device
    scan (self bounds, the window kernel's own ranges) sees the same inputs"""
    if request.param == "reference_layout":
        monkeypatch.setenv("GD_HOST_NOPACK", "1")


def _synth(c, nsnp, a, b):
    from gdscan import synth
    return synth.chromosome(c, nsnp, a, b)


@pytest.mark.parametrize("asize,bsize,nsnp", [(10, 10, 12000), (20, 20, 12000), (7, 13, 6000)])
def test_threaded_scan_matches_oracle(oracle, asize, bsize, nsnp):
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(1, nsnp, asize, bsize)
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend)
    s, d = fet.scan(av, bv, ap, bp, regend, seed=20261015)
    assert (s_ref != 0).sum() > 100
    assert close(s, s_ref) and close(d, d_ref)
    # computed-window mask identical (zeros elsewhere)
    assert np.array_equal(s_ref == 0, s == 0)
    exact = np.mean(s == s_ref)
    assert exact > 0.99, exact


def test_serial_window_set(oracle):
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(2, 3000, 10, 10)
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend, serial=True)
    s, d = fet.scan(av, bv, ap, bp, regend, seed=20261015, serial=True)
    assert close(s, s_ref) and close(d, d_ref)


@pytest.mark.parametrize("wsize,wstep", [(1000, 500), (5000, 500), (2000, 1000), (2500, 250)])
def test_geometries(oracle, wsize, wstep):
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(3, 8000, 10, 10)
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend, wsize, wstep)
    s, d = fet.scan(av, bv, ap, bp, regend, wsize, wstep, seed=20261015)
    assert close(s, s_ref) and close(d, d_ref)


def test_small_region_threaded_computes_nothing(oracle):
    """Quirk Q3: regend/wstep - 3 < 100 -> the threaded driver runs no task."""
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(4, 800, 10, 10)  # ~40 kb
    s, d = fet.scan(av, bv, ap, bp, regend)
    assert not s.any() and not d.any()
    s2, d2 = fet.scan(av, bv, ap, bp, regend, serial=True)
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend, serial=True)
    assert s2.any() and close(s2, s_ref) and close(d2, d_ref)


def test_reference_entry_point_in_place(oracle):
    """fisher_exact_tester writes in place, leaves non-computed windows untouched."""
    import fisher_cython_parallel as fcp
    from gdscan import lib
    av, bv, ap, bp, regend = _synth(5, 4000, 10, 10)
    n = regend // 500
    s = np.full(n, 7.0)
    d = np.full(n, 7.0)
    lib.gd_set_seed(99)
    fcp.fisher_exact_tester(av, bv, ap, bp, 0, regend, 2500, 500, len(av), len(bv), 0.95, s, d)
    s_ref = np.full(n, 7.0)
    d_ref = np.full(n, 7.0)
    oracle.orc_fet_scan(av, bv, ap, bp, regend, 2500, 500, len(av), len(bv), 0.95, 99, 0, s_ref, d_ref)
    lib.gd_set_seed(20261015)
    assert close(s, s_ref) and close(d, d_ref)
    assert s[-1] == 7.0 and s[-3] == 7.0  # quirk Q2: last windows never computed


def test_dtype_errors():
    import fisher_cython_parallel as fcp
    z = np.zeros(4)
    with pytest.raises(ValueError):
        fcp.fisher_exact_tester(np.zeros(4, np.float32), z, np.zeros(4, np.int32), np.zeros(4, np.int32), 0, 100,
                                25, 5, 4, 4, 0.95, z, z)
    with pytest.raises(ValueError):
        fcp.fisher_exact_tester(z, z, np.zeros(4, np.int64), np.zeros(4, np.int32), 0, 100, 25, 5, 4, 4, 0.95,
                                z, z)


def test_unsorted_positions_rejected():
    from gdscan import GdError, fet
    av, bv, ap, bp, regend = _synth(6, 6000, 10, 10)
    ap = ap.copy()
    ap[5000:5010] = 1
    with pytest.raises(GdError):
        fet.scan(av, bv, ap, bp, regend)


def test_misaligned_populations(oracle):
    """B holds one extra leading SNP: every window's B slice starts on a different
    row than A's -> per-window recomputation from the raw slices (general path)."""
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(7, 6000, 10, 12)
    bv2 = np.concatenate([np.full(12, 3.0), bv])
    bp2 = np.concatenate([np.full(12, 0, np.int32), bp])
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv2, ap, bp2, regend)
    s, d = fet.scan(av, bv2, ap, bp2, regend, seed=20261015)
    assert close(s, s_ref) and close(d, d_ref)


def test_dense_windows_global_scratch(oracle):
    """npos > LDS capacity -> 256-thread workgroups with HBM scratch."""
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(8, 20000, 4, 4)
    # squeeze positions: 1 SNP per bp so a 2500-bp window holds ~2500 SNPs
    ap = (ap // 50).astype(np.int32)
    bp = (bp // 50).astype(np.int32)
    regend = int(ap[-1]) + 1
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend, 2500, 100)
    s, d = fet.scan(av, bv, ap, bp, regend, 2500, 100, seed=20261015)
    assert (s_ref != 0).sum() > 50
    assert close(s, s_ref) and close(d, d_ref)


def test_large_cohort_overflow_semantics(oracle):
    """40+40: binomial() overflow to 0 (first at C(68,31)) gives inf/NaN p for some
    SNPs; NaN windows use glibc's merge-sort order on the GPU too."""
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(9, 6000, 40, 40)
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend)
    s, d = fet.scan(av, bv, ap, bp, regend, seed=20261015)
    assert close(s, s_ref) and close(d, d_ref)


def test_percentiles(oracle):
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(10, 6000, 10, 10)
    for perc in (0.0, 0.5, 0.8, 1.0):
        s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend, perc=perc)
        s, d = fet.scan(av, bv, ap, bp, regend, perc=perc, seed=20261015)
        assert close(s, s_ref) and close(d, d_ref), perc


def test_device_synth_matches_numpy():
    import torch
    from gdscan import synth
    from gdscan._lib import check, lib
    nsnp, a, b = 3000, 5, 7
    av, bv, ap, bp, regend = synth.chromosome(11, nsnp, a, b)
    dev = torch.device("cuda", 0)
    t = [torch.empty(nsnp * a, dtype=torch.float64, device=dev), torch.empty(nsnp * b, dtype=torch.float64, device=dev),
         torch.empty(nsnp * a, dtype=torch.int32, device=dev), torch.empty(nsnp * b, dtype=torch.int32, device=dev)]
    q = torch.from_numpy(synth.freq_table()).to(dev)
    check(lib.gd_synth_device(11, nsnp, a, b, synth.MASTER_SEED, q.data_ptr(), *[x.data_ptr() for x in t],
                              torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    for x, y in zip(t, (av, bv, ap, bp)):
        assert np.array_equal(x.cpu().numpy(), y)


@pytest.mark.parametrize("groups", [None, "1", "2", "4", "2g1", "3g2"])
def test_device_batch_api_matches_host(oracle, monkeypatch, groups):
    """Several chromosomes in one device scan == per-chromosome scans; with GD_GROUPS the
    scan pipelines chromosome groups over the context's streams (the default, two groups,
    their window kernels on alternating streams, running concurrently; one group runs every
    pass on the caller's stream); "<g>g<n>": g groups, the first of n chromosomes (GD_GROUP0)."""
    if groups:
        g, _, n0 = groups.partition("g")
        monkeypatch.setenv("GD_GROUPS", g)
        if n0:
            monkeypatch.setenv("GD_GROUP0", n0)
    import torch
    from gdscan import _lib, synth
    from gdscan._lib import Chrom, check, lib
    dev = torch.device("cuda", 0)
    data = [synth.chromosome(20 + c, n, 10, 10) for c, n in enumerate((5000, 7000, 600, 6000))]
    A = np.concatenate([x[0] for x in data]); B = np.concatenate([x[1] for x in data])
    AP = np.concatenate([x[2] for x in data]); BP = np.concatenate([x[3] for x in data])
    chroms = (Chrom * len(data))()
    off_a = off_b = w = 0
    for i, (av, bv, ap, bp, regend) in enumerate(data):
        chroms[i].a_off, chroms[i].b_off, chroms[i].alen, chroms[i].blen = off_a, off_b, len(av), len(bv)
        chroms[i].regend, chroms[i].w_out, chroms[i].seed = regend, w, 1000 + i
        off_a += len(av); off_b += len(bv); w += regend // 500
    tens = [torch.from_numpy(x).to(dev) for x in (A, B, AP, BP)]
    sc = torch.zeros(w, dtype=torch.float64, device=dev); sd = torch.zeros_like(sc)
    ctx = lib.gd_ctx_create(0)
    check(lib.gd_fet_scan_device(ctx, chroms, len(data), *[t.data_ptr() for t in tens], 2500, 500, 0.95,
                                 _lib.GD_WINDOWS_THREADED, sc.data_ptr(), sd.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream))
    lib.gd_ctx_destroy(ctx)
    sc = sc.cpu().numpy(); sd = sd.cpu().numpy()
    w = 0
    for i, (av, bv, ap, bp, regend) in enumerate(data):
        s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend, seed=1000 + i)
        n = regend // 500
        assert close(sc[w:w + n], s_ref) and close(sd[w:w + n], d_ref), i
        w += n


def test_fast_path_equals_literal_path_full_chromosome(monkeypatch):
    """Size-independent property at full chromosome scale (500k SNPs, 20+20, ~50k
    windows): the register order-statistic bootstrap equals the literal
    sort-and-histogram path bit for bit."""
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(0, 500_000, 20, 20)
    s_fast, d_fast = fet.scan(av, bv, ap, bp, regend, seed=5)
    monkeypatch.setenv("GD_FORCE_GENERAL", "1")
    s_lit, d_lit = fet.scan(av, bv, ap, bp, regend, seed=5)
    monkeypatch.delenv("GD_FORCE_GENERAL")
    assert (s_fast != 0).sum() > 49_000
    assert np.array_equal(s_fast, s_lit) and np.array_equal(d_fast, d_lit)


def _windows_with_rejections(regend, wsize, wstep, ap, asize, seed, nrep=100):
    """Host replica of the per-window nrand48 stream: which windows reject a draw."""
    from gdscan.synth import _mix64
    nwin = regend // wstep
    starts = np.arange(nwin) * wstep
    lo = np.searchsorted(ap, starts, side="left")
    hi = np.searchsorted(ap, starts + wsize, side="right")
    n = (hi - lo) // asize
    w = np.arange(nwin, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = _mix64(np.uint64(seed) ^ _mix64(np.uint64(0) + np.uint64(0x9E3779B97F4A7C15) * (w + np.uint64(1))))
    x &= np.uint64(0xFFFFFFFFFFFF)
    nn = np.maximum(n, 1).astype(np.int64)
    limit = 0x7FFFFFFF - (0x80000000 % nn)
    hit = np.zeros(nwin, bool)
    for t in range(int(nrep * nn.max())):
        with np.errstate(over="ignore"):
            x = (x * np.uint64(0x5DEECE66D) + np.uint64(0xB)) & np.uint64(0xFFFFFFFFFFFF)
        r = (x >> np.uint64(17)).astype(np.int64)
        hit |= (r > limit) & (t < nrep * nn)
    return hit & (n > 0)


def test_rejected_draws_are_redrawn(oracle):
    """Dense windows (n ~ 250, perc 0.99 keeps them on the fast path) make the
    modulo-bias rejection of random_int_nrand48 (cFisher.c:550-552) happen; the
    fast path must redraw exactly like the reference."""
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(12, 60000, 5, 5)
    wsize, wstep, perc, seed = 12500, 500, 0.99, 4242
    hit = _windows_with_rejections(regend, wsize, wstep, ap, 5, seed)
    assert hit.sum() >= 1
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend, wsize, wstep, perc, seed)
    s, d = fet.scan(av, bv, ap, bp, regend, wsize, wstep, perc, seed=seed)
    assert close(s, s_ref) and close(d, d_ref)
    assert close(d[hit], d_ref[hit])


def test_empty_population_writes_nothing():
    """alen or blen == 0: the reference computes nothing; outputs keep the caller's values."""
    import fisher_cython_parallel as fcp
    av, bv, ap, bp, regend = _synth(30, 3000, 4, 4)
    for a_cut, b_cut in ((0, len(bv)), (len(av), 0)):
        s, d = np.full(regend // 500, 7.0), np.full(regend // 500, 7.0)
        fcp.fisher_exact_tester(av[:a_cut], bv[:b_cut], ap[:a_cut], bp[:b_cut], 0, regend, 2500, 500, a_cut, b_cut,
                                0.95, s, d)
        assert np.all(s == 7.0) and np.all(d == 7.0)


def test_mid_size_windows_counting_rank(oracle):
    """64 < n <= 256 SNPs per window: the fast path's counting ranks."""
    from gdscan import fet
    av, bv, ap, bp, regend = _synth(31, 20000, 6, 6)
    rows = len(ap) // 6
    pos = (np.arange(rows, dtype=np.int32) + 1) * 20  # ~125 SNPs per 2.5 kb window
    ap, bp = np.repeat(pos, 6), np.repeat(pos, 6)
    regend = int(pos[-1]) + 1
    s, d = fet.scan(av, bv, ap, bp, regend, seed=5)
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend, seed=5)
    assert (s_ref != 0).sum() > 500
    assert close(s, s_ref) and close(d, d_ref)


@pytest.mark.parametrize("name", ["10x10", "20x20", "7x13_w1000", "small_serial", "perc50"])
def test_golden_reference_fixtures(name):
    """The HIP scan against the committed outputs of the reference's own C
    (tests/golden/make_golden.py: threadcompute / compute scores, the seeded
    fisher_exact_test stddev), with no oracle in between."""
    from conftest import SCAN_FIXTURES, load_scan_fixture
    from gdscan import fet
    assert name in SCAN_FIXTURES
    f = load_scan_fixture(name)
    s, d = fet.scan(f["av"], f["bv"], f["ap"], f["bp"], f["regend"], f["wsize"], f["wstep"], f["perc"],
                    seed=f["seed"], serial=f["serial"])
    assert (f["scores"] != 0).sum() > 50
    assert np.array_equal(s == 0, f["scores"] == 0)
    assert close(s, f["scores"]) and close(d, f["stddev"])
    assert np.mean(s == f["scores"]) > 0.99



def _irregular(kind):
    av, bv, ap, bp, regend = _synth(11, 9000, 10, 10)
    ap, bp = ap.copy(), bp.copy()
    if kind == "gaps":  # a 40 kb hole and a late start: windows with no SNP
        ap[ap > 150_000] += 40_000
        bp[bp > 150_000] += 40_000
        ap += 3_000
        bp += 3_000
        regend = int(ap[-1]) + 1
    elif kind == "stacked":  # runs of SNP rows sharing one position (the first row alone)
        ap = (-(-ap // 700) * 700).astype(np.int32)
        bp = (-(-bp // 700) * 700).astype(np.int32)
        ap[:10] = 0
        bp[:10] = 0
        assert (ap[10:] > 0).all() and (bp[10:] > 0).all()
    elif kind == "misaligned":  # B one row ahead of A
        bv = np.concatenate([np.full(10, 3.0), bv])
        bp = np.concatenate([np.zeros(10, np.int32), bp])
    return av, bv, ap, bp, regend


@pytest.mark.parametrize("kind,wsize,wstep", [("gaps", 2500, 500), ("stacked", 2500, 500), ("misaligned", 2500, 500),
                                              ("plain", 2500, 250), ("plain", 1000, 500)])
def test_irregular_geometries(oracle, kind, wsize, wstep):
    """Window bounds (slide_right, comparative.c:49-71) on gaps (windows without SNPs, a
    late first position), runs of rows sharing a position, B one row ahead of A, and other
    window geometries: the device scan equals the oracle."""
    from gdscan import fet
    av, bv, ap, bp, regend = _irregular(kind)
    s, d = fet.scan(av, bv, ap, bp, regend, wsize, wstep, seed=5)
    s_ref, d_ref = oracle_fet_scan(oracle, av, bv, ap, bp, regend, wsize, wstep, seed=5)
    assert (s_ref != 0).sum() > 50 and np.isfinite(s_ref).mean() > 0.9
    assert close(s, s_ref) and close(d, d_ref)
