"""Packed genotype tracks (include/gdscan.h gd_pack_*, gd_*_scan_packed_*).

CPU: the host packer's codes, round trip and refusals (values outside the four
VCFConvert.py:8-17 codes, rows whose individuals do not share a position, A/B
misalignment).  GPU: a packed batch scans exactly like the reference-layout batch of
the same tracks -- FET scores and seeded bootstrap stddev, CSS scores and permutation
p, bit for bit -- and like the oracle; the device packer equals the host packer."""
import numpy as np
import pytest

from conftest import oracle_fet_scan


def _synth(c, nsnp, a, b):
    from gdscan import synth
    return synth.chromosome(c, nsnp, a, b)


def test_pack_codes_and_round_trip():
    from gdscan import packed
    av, bv, ap, bp, regend = _synth(3, 2000, 20, 20)
    pc = packed.pack(av, bv, ap, bp, regend)
    assert (pc.asize, pc.bsize, pc.nrows) == (20, 20, 2000)
    assert pc.acodes.dtype == np.uint64 and pc.acodes.shape == (2000,)
    assert np.array_equal(pc.rowpos, ap[::20])
    # individual 3 of row 7: bits 6..7 of word 7
    code = int(pc.acodes[7] >> np.uint64(6)) & 3
    assert packed.VALUES[code] == av[7 * 20 + 3]
    rav, rbv, rap, rbp = pc.unpack()
    assert np.array_equal(rav, av) and np.array_equal(rbv, bv)
    assert np.array_equal(rap, ap) and np.array_equal(rbp, bp)
    # padding codes are zero: 20 individuals use 40 of 64 bits
    assert np.all(pc.acodes >> np.uint64(40) == 0)


def test_pack_wide_rows_span_words():
    from gdscan import packed
    av, bv, ap, bp, regend = _synth(5, 300, 45, 33)
    pc = packed.pack(av, bv, ap, bp, regend)
    assert pc.acodes.shape == (300 * 2,) and pc.bcodes.shape == (300 * 2,)
    rav, rbv, _, _ = pc.unpack()
    assert np.array_equal(rav, av) and np.array_equal(rbv, bv)


def test_pack_refuses_what_it_cannot_hold():
    from gdscan import packed
    av, bv, ap, bp, regend = _synth(4, 500, 6, 6)
    bad = av.copy()
    bad[17] = 1.5
    with pytest.raises(ValueError, match="genotype codes"):
        packed.pack(bad, bv, ap, bp, regend)
    bad = av.copy()
    bad[9] = np.nan
    with pytest.raises(ValueError):
        packed.pack(bad, bv, ap, bp, regend)
    bp2 = bp.copy()
    bp2[6 * 11 + 2] += 1  # one B individual off its row's position
    with pytest.raises(ValueError, match="position"):
        packed.pack(av, bv, ap, bp2, regend)
    with pytest.raises(ValueError, match="whole rows"):
        packed.pack(av[:-1], bv, ap[:-1], bp, regend)


def test_shape_is_get_population_size():
    from gdscan import packed
    ap = np.repeat(np.array([5, 9, 12], dtype=np.int32), 4)
    bp = np.repeat(np.array([5, 9, 12], dtype=np.int32), 3)
    assert packed.shape(ap, bp) == (4, 3, 3)
    with pytest.raises(ValueError, match="whole rows"):  # partial trailing row: no packed form
        packed.shape(ap[:-1], bp)
    with pytest.raises(ValueError, match="whole rows"):  # A and B hold different row counts
        packed.shape(ap, bp[:-3])


@pytest.mark.gpu
def test_packed_fet_equals_reference_layout(oracle):
    from gdscan import fet, packed
    chroms = [_synth(c, 30000 + 7000 * c, 20, 20) for c in range(3)]
    pcs = [packed.pack(av, bv, ap, bp, regend) for av, bv, ap, bp, regend in chroms]
    res = packed.fet_scan(pcs, seed=99)
    for (av, bv, ap, bp, regend), (s, d) in zip(chroms, res):
        s_ref, d_ref = fet.scan(av, bv, ap, bp, regend, seed=99)
        assert np.array_equal(s, s_ref) and np.array_equal(d, d_ref)
    av, bv, ap, bp, regend = chroms[0]
    s_o, d_o = oracle_fet_scan(oracle, av, bv, ap, bp, regend, seed=99)
    s, d = res[0]
    rel = lambda x, y: np.all(np.abs(x - y) <= 1e-9 * np.maximum(np.abs(x), np.abs(y)) + 1e-12)
    assert (s_o != 0).sum() > 1000 and rel(s, s_o) and rel(d, d_o)


@pytest.mark.gpu
def test_packed_fet_serial_dense_and_exact():
    """Serial window set, uneven populations, dense windows (general path), exact mode."""
    from gdscan import fet, packed
    av, bv, ap, bp, regend = _synth(12, 60000, 5, 7)
    pc = packed.pack(av, bv, ap, bp, regend)
    for kw in (dict(serial=True), dict(wsize=12500, perc=0.99), dict(exact=True)):
        (s, d), = packed.fet_scan([pc], seed=7, **kw)
        s_ref, d_ref = fet.scan(av, bv, ap, bp, regend, seed=7, **kw)
        assert np.array_equal(s, s_ref) and np.array_equal(d, d_ref), kw


@pytest.mark.gpu
@pytest.mark.parametrize("mds,runs", [(0, 0), (0, 200), (1, 0), (2, 50)])
def test_packed_css_equals_reference_layout(mds, runs):
    from gdscan import css, packed
    chroms = [_synth(20 + c, 8000, 10, 10) for c in range(2)]
    pcs = [packed.pack(av, bv, ap, bp, regend) for av, bv, ap, bp, regend in chroms]
    res = packed.css_scan(pcs, treshold=10, runs=runs, mds=mds, seed=5)
    for (av, bv, ap, bp, regend), (s, p) in zip(chroms, res):
        s_ref, p_ref = css.scan(av, bv, ap, bp, regend, treshold=10, runs=runs, mds=mds, seed=5)
        assert (s_ref != 0).sum() > 200
        assert np.array_equal(s, s_ref) and np.array_equal(p, p_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("a,b", [(45, 33), (33, 45), (64, 40)])
def test_packed_multiword_rows(a, b):
    """Rows wider than one 64-bit word (more than 32 individuals per population): the
    per-word popcounts of k_snp_fet_packed and the word select of k_css_pack_codes."""
    from gdscan import css, fet, packed
    av, bv, ap, bp, regend = _synth(60, 3_000, a, b)
    pc = packed.pack(av, bv, ap, bp, regend)
    assert pc.acodes.shape[0] == 3_000 * ((a + 31) // 32)
    (s, d), = packed.fet_scan([pc], seed=11)
    s_ref, d_ref = fet.scan(av, bv, ap, bp, regend, seed=11)
    assert (s_ref != 0).sum() > 50  # >= 68 individuals: the reference's overflow NaNs included
    assert np.array_equal(s, s_ref, equal_nan=True) and np.array_equal(d, d_ref, equal_nan=True)
    (s, p), = packed.css_scan([pc], treshold=10, runs=40, seed=11)
    s_ref, p_ref = css.scan(av, bv, ap, bp, regend, treshold=10, runs=40, seed=11)
    assert np.array_equal(s, s_ref, equal_nan=True) and np.array_equal(p, p_ref)


@pytest.mark.gpu
def test_device_packer_equals_host_packer():
    import torch
    from gdscan import packed
    from gdscan._lib import check, lib
    av, bv, ap, bp, regend = _synth(8, 20000, 20, 40)
    pc = packed.pack(av, bv, ap, bp, regend)
    dev = torch.device("cuda:0")
    t = [torch.from_numpy(x).to(dev) for x in (av, bv, ap, bp)]
    ac = torch.zeros(pc.acodes.shape[0], dtype=torch.int64, device=dev)
    bc = torch.zeros(pc.bcodes.shape[0], dtype=torch.int64, device=dev)
    rp = torch.zeros(pc.nrows, dtype=torch.int32, device=dev)
    check(lib.gd_pack_chrom_device(*(x.data_ptr() for x in t), pc.asize, pc.bsize, pc.nrows, ac.data_ptr(),
                                   bc.data_ptr(), rp.data_ptr(), None))
    assert np.array_equal(ac.cpu().numpy().view(np.uint64), pc.acodes)
    assert np.array_equal(bc.cpu().numpy().view(np.uint64), pc.bcodes)
    assert np.array_equal(rp.cpu().numpy(), pc.rowpos)
    bad = t[0].clone()
    bad[5] = 2.0
    assert lib.gd_pack_chrom_device(bad.data_ptr(), *(x.data_ptr() for x in t[1:]), pc.asize, pc.bsize, pc.nrows,
                                    ac.data_ptr(), bc.data_ptr(), rp.data_ptr(), None) != 0
