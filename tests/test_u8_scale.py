"""The MNIST step kernels turn uint8 inputs into k/255 with q = k * r (r = fp32(1/255)) and
one fma residual correction (csrc/include/convnet_dev.h u8_over_255) instead of a division:
pinned here, in exact rational arithmetic with IEEE round-to-nearest-even at every fp32
rounding point, to equal float32(k / 255.0) -- the value the fp32 reference path feeds --
for all 256 k."""
from fractions import Fraction

import numpy as np


def _rne32(x: Fraction) -> np.float32:
    """The fp32 nearest to the exact rational x (ties to even)."""
    c = np.float32(float(x))  # within one fp32 ulp of the answer
    cands = [np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))]

    def key(v):
        odd = int(np.frombuffer(np.float32(v).tobytes(), dtype=np.uint32)[0]) & 1
        return (abs(Fraction(float(v)) - x), odd)

    return min(cands, key=key)


def test_fma_corrected_reciprocal_matches_division():
    r = np.float32(1.0) / np.float32(255.0)
    fr = Fraction(float(r))
    for k in range(256):
        q = _rne32(k * fr)                                        # q = k * r
        e = _rne32(Fraction(k) - Fraction(float(q)) * 255)        # fma(-q, 255, k)
        v = _rne32(Fraction(float(e)) * fr + Fraction(float(q)))  # fma(e, r, q)
        assert v == np.float32(k / 255.0), k
