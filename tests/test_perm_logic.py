"""CPU restatements of two pieces of the CSS permutation kernel (gd_css_perm.hip) that
are not visible in its outputs on ordinary data, checked against their definitions:

* perm_rd's limit and shift from the magic number alone == gd_randint_make's
  (random_int_nrand48, css.c:675-690) for every n in 2..128;
* score_f32's error bound: a sum of n FP32-rounded non-negative terms lies within
  (n + 2) 2^-24 (1.001) of its computed value."""
import numpy as np


def test_divisor_constants_from_magic():
    for n in range(2, 129):
        l = (n - 1).bit_length()  # ceil(log2 n)
        magic = -(-(1 << (31 + l)) // n)
        shift = 31 - (32 - (n - 1).bit_length())  # 31 - clz32(n - 1)
        assert shift == l - 1
        q = ((0x7FFFFFFF * magic) >> 32) >> shift
        t = (0x7FFFFFFF - q * n + 1) & 0xFFFFFFFF
        limit = 0x7FFFFFFF - (0 if t == n else t)
        assert limit == 0x7FFFFFFF - (2 ** 31 % n), n


def test_fp32_sum_bound():
    rng = np.random.default_rng(3)
    u = 2.0 ** -24 * 1.001
    for n in (1, 7, 39, 780, 2016):
        for scale in (1e-3, 1.0, 37.5, 1e6):
            x = rng.random(n) * scale
            x[rng.random(n) < 0.1] *= 1e-4  # mixed magnitudes
            acc = np.float32(0)
            for v in x.astype(np.float32):
                acc = np.float32(acc + v)
            exact = float(np.sum(x, dtype=np.float64))
            assert abs(float(acc) - exact) <= (n + 2) * u * float(acc) + 1e-300
