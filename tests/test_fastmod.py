"""The sampler's index reduction r mod npool (hg_ransac.hpp fastmod_u32 / fastmod_magic:
one umulhi + one mullo, round-up division by an invariant integer) restated with Python
integers at 32-bit width and checked against % for divisors across the whole uint32
range -- every d up to 4096, powers of two and their neighbours, random large d -- and
the numerators where such schemes break (0, d-1, d, multiples of d, 2^32-1, ...).  The
binary64 form (fmod_f64_u32 / fmod_f64_magic, d < 2^31) the same way, its one rounded
product restated in numpy float64.  The GPU tests (test_gpu_ransac.py) check the device
code itself against the oracle's %."""
import numpy as np

M32 = (1 << 32) - 1


def magic(d):
    if d <= 2:
        return 0, 0
    l = d.bit_length() - 1
    if d & (d - 1) == 0:
        return 0, l - 1
    M = (1 << (33 + l)) // d + 1
    assert (1 << 32) < M < (1 << 33)
    return M - (1 << 32), l


def fastmod(r, m, sh, d):
    hi = (r * m) >> 32
    q = ((((r - hi) & M32) >> 1) + hi) >> sh
    rem = (r - q * d) & M32
    return min(rem, d - 1)


def _numerators(d, rng):
    base = {0, 1, 2, d - 1, d, d + 1, 2 * d - 1, 2 * d, M32, M32 - 1, M32 - d, (1 << 31),
            (1 << 31) - 1, (M32 // d) * d, (M32 // d) * d - 1}
    base |= set(int(x) for x in rng.integers(0, 1 << 32, 64, dtype=np.uint64))
    return [r for r in base if 0 <= r <= M32]


def test_fastmod_matches_modulo_everywhere():
    rng = np.random.default_rng(3)
    ds = set(range(1, 4097))
    for k in range(1, 32):
        ds |= {(1 << k) - 1, 1 << k, (1 << k) + 1}
    ds |= {M32, M32 - 1, 2540, 20_000, 65_537}
    ds |= set(int(x) for x in rng.integers(1, 1 << 32, 400, dtype=np.uint64))
    for d in sorted(ds):
        m, sh = magic(d)
        for r in _numerators(d, rng):
            assert fastmod(r, m, sh, d) == r % d, (d, r)


def fmod_f64_magic(d):
    u = np.float64(1.0) / np.float64(d)
    if int(u.as_integer_ratio()[0]) * d < u.as_integer_ratio()[1]:  # u < 1/d exactly
        u = np.nextafter(u, np.float64(2.0))
    return u


def fmod_f64(r, u, d):
    q = int(np.trunc(np.float64(r) * u))      # the one rounded product (RN), truncated
    rem = r - q * d                           # one FMA: exact, every term an integer < 2^33
    assert -(1 << 31) <= rem < (1 << 31)      # the int32 conversion is exact
    return rem + d if rem < 0 else rem


def test_fmod_f64_matches_modulo_below_2_31():
    rng = np.random.default_rng(5)
    ds = set(range(1, 4097))
    for k in range(1, 31):
        ds |= {(1 << k) - 1, 1 << k, (1 << k) + 1}
    ds |= {(1 << 31) - 1, 2540, 9088, 20_000, 65_537}
    ds |= set(int(x) for x in rng.integers(1, 1 << 31, 400, dtype=np.uint64))
    for d in sorted(ds):
        u = fmod_f64_magic(d)
        assert u >= 0 and u.as_integer_ratio()[0] * d >= u.as_integer_ratio()[1]
        for r in _numerators(d, rng):
            assert fmod_f64(r, u, d) == r % d, (d, r)


def t8_index(w, u, d):
    """mrg::step_index (hg_mrg32k3a.hpp): q = trunc(RN(w u + u/2)) with ONE rounding (the FMA,
    restated with exact rationals: float(Fraction) rounds to nearest), then w - q d exactly."""
    from fractions import Fraction
    uf = Fraction(float(u))
    q = int(float(Fraction(w) * uf + uf / 2))  # trunc: the value is >= 0
    assert q == int(Fraction(2 * w + 1, 2 * d))  # floor((w + 1/2) / d) = floor(w / d): no correction
    return w - q * d


def test_table8_index_form_matches_modulo():
    rng = np.random.default_rng(7)
    ds = set(range(1, 1025)) | {2540, 4096, 5120, 9088, 20_000, 65_537, M32, M32 - 1, (1 << 31) + 1}
    for k in range(1, 32):
        ds |= {(1 << k) - 1, 1 << k, (1 << k) + 1}
    ds |= set(int(x) for x in rng.integers(1, 1 << 32, 120, dtype=np.uint64))
    for d in sorted(ds):
        u = fmod_f64_magic(d)
        for w in _numerators(d, rng):
            assert t8_index(w, u, d) == w % d, (d, w)
