"""The HIP kernels divide by loop-invariant divisors through a precomputed reciprocal
with one fma correction (cpp_volume_rendering_amd/csrc/cvr_device.h div_by_recip:
q = RN(a*y), r = fma(-b, q, a), RN(q + r*y), y = RN(1/b)).  Markstein's theorem makes
that the correctly rounded a / b while nothing underflows; this checks it against IEEE
division on 3e8 random pairs spanning the ranges the EBS shadow chains use (and far
beyond), so the shortcut cannot change a bit of any image."""


def test_div_by_recip_matches_ieee(oracle):
    assert oracle.check_div_by_recip(200_000_000, 7, -20, 20) == 0
    assert oracle.check_div_by_recip(100_000_000, 11, -100, 100) == 0
