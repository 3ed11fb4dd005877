"""GPU: the HIP CSS scan (through the C-ABI) against the CPU oracle.

Tolerance: CSS scores within 1e-9 relative (north star).  The eigen-solvers differ
(Householder + bisection here, Jacobi in the oracle, GSL QR in the reference), so
scores agree to ~1e-13 except in windows whose 2nd and 3rd eigenvalues nearly
coincide; permutation p-values are compared exactly and may differ only where a
permuted score ties the observed one to within rounding."""
import ctypes

import numpy as np
import pytest

from conftest import assert_p_mismatches_are_ties, close, oracle_css_scan

pytestmark = pytest.mark.gpu


def _synth(c, nsnp, a, b):
    from gdscan import synth
    return synth.chromosome(c, nsnp, a, b)


def _cmp_scores(s, s_ref, rel=1e-9):
    assert np.array_equal(s == 0, s_ref == 0), "computed-window sets differ"
    assert np.array_equal(np.isnan(s), np.isnan(s_ref))
    ok = np.isnan(s_ref) | (np.abs(s - s_ref) <= rel * np.abs(s_ref) + 1e-12)
    assert ok.mean() == 1.0, (np.flatnonzero(~ok)[:10], s[~ok][:5], s_ref[~ok][:5])


@pytest.mark.parametrize("asize,bsize,nsnp", [(10, 10, 60_000), (20, 20, 30_000), (7, 13, 30_000), (40, 40, 4_000),
                                              (1, 1, 20_000), (33, 31, 6_000), (45, 45, 3_000),
                                              # the two-windows-per-wave 40 tier below m = 40: rows 0-31 of
                                              # each window in its half wave, rows 32-39 in the LDS tail quads
                                              # (m = 25, 31, 32: no tail row; 33: one; 34, 35, 39)
                                              (12, 13, 8_000), (15, 16, 8_000), (16, 16, 8_000), (16, 17, 8_000),
                                              (17, 17, 8_000), (19, 20, 8_000), (13, 14, 8_000), (5, 30, 8_000),
                                              # the one-wave 80 tier: 1, 8 and 9 tail rows (m = 65, 72, 73)
                                              (33, 32, 3_000), (30, 42, 3_000), (43, 30, 3_000)])
def test_scores_match_oracle(oracle, asize, bsize, nsnp):
    from gdscan import css
    av, bv, ap, bp, regend = _synth(3, nsnp, asize, bsize)
    s, p = css.scan(av, bv, ap, bp, regend, runs=0)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, runs=0)
    _cmp_scores(s, s_ref)
    assert np.array_equal(p, p_ref)


def test_serial_window_set(oracle):
    from gdscan import css
    av, bv, ap, bp, regend = _synth(4, 20_000, 10, 10)
    s, p = css.scan(av, bv, ap, bp, regend, serial=True)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, serial=True)
    _cmp_scores(s, s_ref)
    assert np.array_equal(p, p_ref)


@pytest.mark.parametrize("asize,bsize,treshold,runs,nsnp", [(10, 10, 10, 300, 15_000), (20, 20, 5, 100, 15_000),
                                                            (6, 9, 50, 1000, 15_000), (40, 40, 10, 300, 3_000),
                                                            (33, 31, 10, 200, 3_000)])
def test_permutation_p_matches_oracle(oracle, asize, bsize, treshold, runs, nsnp):
    """The C5 shape (40+40, the two-rows-per-lane composition and the 80-tier MDS
    coordinates) included."""
    from gdscan import css
    av, bv, ap, bp, regend = _synth(5, nsnp, asize, bsize)
    s, p = css.scan(av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=77)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=77)
    _cmp_scores(s, s_ref)
    comp = s_ref != 0
    assert np.all(p[~comp] == 0)
    # every p that differs from the oracle scan's is a near-tie on the device's coordinates
    assert_p_mismatches_are_ties(oracle, av, bv, ap, bp, regend, asize, bsize, np.where(comp, p, 0.0),
                                 np.where(comp, p_ref, 0.0), treshold, runs, 77)


@pytest.mark.parametrize("asize,bsize,nsnp,nbad", [(8, 8, 20_000, 400), (40, 40, 3_000, 400), (20, 20, 10_000, 40),
                                                   (13, 14, 10_000, 40), (33, 40, 3_000, 30)])
def test_irregular_values_take_the_literal_path(oracle, asize, bsize, nsnp, nbad):
    """Values outside {3,0,-3,-10000} (including NaN and huge values) follow the
    reference predicate (int)v_i * v_j == -9 with x86 cast semantics.  With few bad
    values most windows stay on the popcount build, so literal and popcount windows
    share the two-window waves of the 40 tier."""
    from gdscan import css
    av, bv, ap, bp, regend = _synth(6, nsnp, asize, bsize)
    rng = np.random.default_rng(0)
    for arr in (av, bv):
        idx = rng.choice(len(arr), nbad, replace=False)
        arr[idx] = rng.choice([1.0, -1.0, 9.0, -9.0, 4.5, -2.25, 0.5, -18.0, np.nan, 1e10, -3.0000001], nbad)
    s, p = css.scan(av, bv, ap, bp, regend)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend)
    _cmp_scores(s, s_ref)


def test_misaligned_populations(oracle):
    """Positions that are not repeated once per individual shift the slices off
    SNP rows; the literal path reads the raw values like the reference."""
    from gdscan import css
    av, bv, ap, bp, regend = _synth(7, 10_000, 6, 6)
    ap = ap.copy()
    ap[1000:1003] = ap[1003]
    s, p = css.scan(av, bv, ap, bp, regend)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend)
    _cmp_scores(s, s_ref)


def test_reference_entry_point_in_place(oracle):
    import css_cython_parallel as ccp
    from gdscan import lib
    av, bv, ap, bp, regend = _synth(8, 20_000, 10, 10)
    lib.gd_set_seed(20261015)
    scores = np.full(regend // 500, 0.0)
    p = np.full(regend // 500, -7.0)
    ccp.cluster_separation_scorer(av, bv, ap, bp, 0, regend, 2500, 500, len(av), len(bv), 10, 50, 0, 0, scores, p)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, runs=50)
    _cmp_scores(scores, s_ref)
    assert np.all(p[s_ref == 0] == -7.0)  # untouched at uncomputed windows


def test_cohort_above_largest_tier_takes_the_general_path(oracle):
    """70 + 70 individuals: above the register tiers, scored by k_css_mds_big
    (tests/test_css_big.py covers that path in depth)."""
    from gdscan import css
    av, bv, ap, bp, regend = _synth(10, 1_100, 70, 70)
    s, p = css.scan(av, bv, ap, bp, regend)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend)
    _cmp_scores(s, s_ref)


def test_device_batch_api_matches_host(oracle):
    import torch
    from gdscan import _lib, synth
    from gdscan._lib import Chrom, check, lib
    dev = torch.device("cuda", 0)
    data = [synth.chromosome(30 + c, n, 10, 10) for c, n in enumerate((5000, 7000, 600, 6000))]
    A = np.concatenate([x[0] for x in data]); B = np.concatenate([x[1] for x in data])
    AP = np.concatenate([x[2] for x in data]); BP = np.concatenate([x[3] for x in data])
    chroms = (Chrom * len(data))()
    off_a = off_b = w = 0
    for i, (av, bv, ap, bp, regend) in enumerate(data):
        chroms[i].a_off, chroms[i].b_off, chroms[i].alen, chroms[i].blen = off_a, off_b, len(av), len(bv)
        chroms[i].regend, chroms[i].w_out, chroms[i].seed = regend, w, 2000 + i
        off_a += len(av); off_b += len(bv); w += regend // 500
    tens = [torch.from_numpy(x).to(dev) for x in (A, B, AP, BP)]
    sc = torch.zeros(w, dtype=torch.float64, device=dev); pv = torch.zeros_like(sc)
    ctx = lib.gd_ctx_create(0)
    check(lib.gd_css_scan_device(ctx, chroms, len(data), *[t.data_ptr() for t in tens], 2500, 500, 10, 100,
                                 _lib.GD_WINDOWS_THREADED, sc.data_ptr(), pv.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream))
    lib.gd_ctx_destroy(ctx)
    sc = sc.cpu().numpy(); pv = pv.cpu().numpy()
    w = 0
    for i, (av, bv, ap, bp, regend) in enumerate(data):
        s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, runs=100, seed=2000 + i)
        n = regend // 500
        _cmp_scores(sc[w:w + n], s_ref)
        assert_p_mismatches_are_ties(oracle, av, bv, ap, bp, regend, 10, 10, pv[w:w + n], p_ref, 10, 100, 2000 + i)
        w += n


@pytest.mark.parametrize("shapes", [
    # 40 tier: different (a, b) splits and m inside one two-window wave at every
    # chromosome boundary; odd per-chromosome window counts shift the pairing, and the
    # batch's total is odd (the last wave holds one window)
    [(20, 20, 5_001), (12, 13, 3_007), (19, 20, 2_203), (15, 16, 4_111), (25, 8, 2_600)],
    # tiers 24 and 64/80 mixed with smaller cohorts in one batch
    [(10, 10, 3_001), (4, 7, 2_500), (40, 40, 1_300), (30, 20, 1_500)],
])
def test_device_batch_mixed_cohorts(oracle, shapes):
    import torch
    from gdscan import _lib, synth
    from gdscan._lib import Chrom, check, lib
    dev = torch.device("cuda", 0)
    data = [synth.chromosome(50 + c, n, a, b) for c, (a, b, n) in enumerate(shapes)]
    A = np.concatenate([x[0] for x in data]); B = np.concatenate([x[1] for x in data])
    AP = np.concatenate([x[2] for x in data]); BP = np.concatenate([x[3] for x in data])
    chroms = (Chrom * len(data))()
    off_a = off_b = w = 0
    total = 0
    for i, (av, bv, ap, bp, regend) in enumerate(data):
        chroms[i].a_off, chroms[i].b_off, chroms[i].alen, chroms[i].blen = off_a, off_b, len(av), len(bv)
        chroms[i].regend, chroms[i].w_out, chroms[i].seed = regend, w, 3000 + i
        off_a += len(av); off_b += len(bv); w += regend // 500
        total += lib.gd_window_count(regend, 2500, 500, _lib.GD_WINDOWS_THREADED)
    if shapes[0] == (20, 20, 5_001):
        assert total % 2 == 1
    tens = [torch.from_numpy(x).to(dev) for x in (A, B, AP, BP)]
    sc = torch.zeros(w, dtype=torch.float64, device=dev); pv = torch.zeros_like(sc)
    ctx = lib.gd_ctx_create(0)
    check(lib.gd_css_scan_device(ctx, chroms, len(data), *[t.data_ptr() for t in tens], 2500, 500, 10, 60,
                                 _lib.GD_WINDOWS_THREADED, sc.data_ptr(), pv.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream))
    lib.gd_ctx_destroy(ctx)
    sc = sc.cpu().numpy(); pv = pv.cpu().numpy()
    w = 0
    for i, (av, bv, ap, bp, regend) in enumerate(data):
        s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, runs=60, seed=3000 + i)
        n = regend // 500
        _cmp_scores(sc[w:w + n], s_ref)
        comp = s_ref != 0
        a_, b_ = shapes[i][0], shapes[i][1]
        assert_p_mismatches_are_ties(oracle, av, bv, ap, bp, regend, a_, b_, np.where(comp, pv[w:w + n], 0.0),
                                     np.where(comp, p_ref, 0.0), 10, 60, 3000 + i)
        w += n


def test_popcount_path_equals_literal_path_full_chromosome(monkeypatch):
    """Size-independent property at full chromosome scale (500k SNPs, 20+20): the
    bit-plane popcount distance build equals the literal per-SNP predicate."""
    from gdscan import css
    av, bv, ap, bp, regend = _synth(0, 500_000, 20, 20)
    s_fast, _ = css.scan(av, bv, ap, bp, regend)
    monkeypatch.setenv("GD_CSS_FORCE_LITERAL", "1")
    s_lit, _ = css.scan(av, bv, ap, bp, regend)
    monkeypatch.delenv("GD_CSS_FORCE_LITERAL")
    assert np.array_equal(s_fast, s_lit, equal_nan=True)
    assert (s_fast != 0).sum() > 45_000


def _dense(av, bv, ap, bp, a, b, step):
    """Re-space the SNPs every `step` bp (denser windows: more than 64 SNPs each)."""
    rows = len(ap) // a
    pos = (np.arange(rows, dtype=np.int32) + 1) * step
    return av, bv, np.repeat(pos, a), np.repeat(pos, b), int(pos[-1]) + 1


def test_dense_windows_multi_chunk(oracle):
    """Windows of ~250 SNPs: the popcount build runs 4 64-SNP chunks per window."""
    from gdscan import css
    av, bv, ap, bp, _ = _synth(12, 6_000, 8, 8)
    av, bv, ap, bp, regend = _dense(av, bv, ap, bp, 8, 8, 10)
    s, p = css.scan(av, bv, ap, bp, regend, treshold=5, runs=40, seed=3)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, treshold=5, runs=40, seed=3)
    _cmp_scores(s, s_ref)
    assert_p_mismatches_are_ties(oracle, av, bv, ap, bp, regend, 8, 8, p, p_ref, 5, 40, 3)


def test_largest_tier_64_plus_64(oracle):
    from gdscan import css
    av, bv, ap, bp, regend = _synth(13, 1_800, 64, 64)
    s, p = css.scan(av, bv, ap, bp, regend)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend)
    _cmp_scores(s, s_ref)


def test_empty_population_writes_nothing():
    from gdscan import css
    av, bv, ap, bp, regend = _synth(14, 3_000, 4, 4)
    import css_cython_parallel as ccp
    out_s, out_p = np.full(regend // 500, 7.0), np.full(regend // 500, 7.0)
    ccp.cluster_separation_scorer(av, bv[:0], ap, bp[:0], 0, regend, 2500, 500, len(av), 0, 10, 0, 0, 0, out_s,
                                  out_p)
    assert np.all(out_s == 7.0) and np.all(out_p == 7.0)


def test_serial_window_set_with_permutations(oracle):
    from gdscan import css
    av, bv, ap, bp, regend = _synth(15, 12_000, 9, 11)
    s, p = css.scan(av, bv, ap, bp, regend, treshold=10, runs=200, seed=9, serial=True)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, treshold=10, runs=200, seed=9, serial=True)
    _cmp_scores(s, s_ref)
    comp = s_ref != 0
    assert_p_mismatches_are_ties(oracle, av, bv, ap, bp, regend, 9, 11, np.where(comp, p, 0.0),
                                 np.where(comp, p_ref, 0.0), 10, 200, 9, serial=True)


@pytest.mark.parametrize("asize,bsize,treshold,runs,nsnp,dup", [(10, 10, 100_000, 500, 15_000, False),
                                                                (40, 40, 100_000, 300, 3_000, False),
                                                                (6, 9, 100_000, 1000, 10_000, True),
                                                                (40, 40, 10, 1000, 3_000, True),
                                                                (20, 20, 100_000, 400, 6_000, True),
                                                                (45, 45, 100_000, 200, 1_800, False),
                                                                (12, 12, 100_000, 300, 8_000, False),
                                                                (48, 48, 100_000, 100, 1_600, False),
                                                                (64, 64, 100_000, 100, 1_400, True)])
def test_fp32_prefilter_changes_no_p(asize, bsize, treshold, runs, nsnp, dup, monkeypatch):
    """The permutation kernel decides hits from an estimate -- the matrix-core score
    (score_mfma, fp16 S on v_mfma_f32_32x32x16_f16) up to 80 individuals, the FP32 copy of
    S above -- and recomputes in FP64 only where the estimate is within its error bound
    of the observed score; GD_PERM_EXACT=1 scores every permutation in FP64.  The
    p-values must be identical, including windows full of exact ties (duplicated
    individuals), at the MFMA tiers (24, 40, 80) and the FP32 tiers (96, 128)."""
    from gdscan import css
    av, bv, ap, bp, regend = _synth(8, nsnp, asize, bsize)
    if dup:
        for arr, size in ((av, asize), (bv, bsize)):
            v = arr.reshape(-1, size)
            v[:, 1::2] = v[:, 0:size - 1:2][:, :v[:, 1::2].shape[1]]
    s, p = css.scan(av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=5)
    monkeypatch.setenv("GD_PERM_EXACT", "1")
    s2, p2 = css.scan(av, bv, ap, bp, regend, treshold=treshold, runs=runs, seed=5)
    assert np.array_equal(s, s2)
    assert (s != 0).sum() > 10
    assert np.array_equal(p, p2), np.flatnonzero(p != p2)[:10]


@pytest.mark.parametrize("asize,bsize,nsnp,serial", [(20, 20, 20_000, False), (12, 12, 20_000, False),
                                                     (40, 40, 6_000, False), (80, 70, 2_000, True)])
def test_fill_averages_discards(oracle, asize, bsize, nsnp, serial):
    """Windows whose count matrix is more than half zeros are discarded (fill_averages,
    css.c:337-366; outputs untouched): a stretch of the chromosome where every individual
    carries the same genotype has all-zero counts, its edges partly.  The computed-window
    set and the scores must equal the oracle's in every tier, discarded and computed
    windows sharing the waves of the 40 tier (one window per half wave)."""
    from gdscan import css
    av, bv, ap, bp, regend = _synth(30 + asize, nsnp, asize, bsize)
    av, bv = av.copy(), bv.copy()
    lo, hi = regend // 3, regend // 2
    av[(ap >= lo) & (ap < hi)] = 3.0
    bv[(bp >= lo) & (bp < hi)] = 3.0
    s, p = css.scan(av, bv, ap, bp, regend, runs=0, serial=serial)
    s_ref, p_ref = oracle_css_scan(oracle, av, bv, ap, bp, regend, runs=0, serial=serial)
    _cmp_scores(s, s_ref)
    w0, w1 = lo // 500, (hi - 2500) // 500
    assert np.all(s[w0 + 1:w1] == 0) and (s != 0).sum() > 0  # the uniform stretch is discarded
