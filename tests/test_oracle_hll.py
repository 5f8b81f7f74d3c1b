"""CPU: the HLL restatement (oracle/hll.py, and lakeside_amd/csrc/hll.cpp through the same vectors on the GPU path)
-- MurmurHash3_x64_128 against its published vector, coupon layout, estimator regimes (SURVEY.md §8(f) f4 `ces`)."""
from oracle import hll


def test_murmur3_x64_128_vectors():
    assert hll.murmur3_x64_128(b"", 0) == (0, 0)
    h1, h2 = hll.murmur3_x64_128(b"hello", 0)
    assert (h2 << 64) | h1 == 0x5B1E906A48AE1D19CBD8A7B341BD9B02
    # every tail length is exercised (1..31 bytes) without error and deterministically
    for n in range(1, 32):
        assert hll.murmur3_x64_128(bytes(range(n)), 9001) == hll.murmur3_x64_128(bytes(range(n)), 9001)


def test_coupon_layout_and_empty_string():
    assert hll.coupon("") == 0
    c = hll.coupon("svc-001:ns-02")
    assert 1 <= (c >> 26) <= 63 and c & 0x3FFFFFF == hll.murmur3_x64_128(b"svc-001:ns-02", 9001)[0] & 0x3FFFFFF


def test_estimate_regimes():
    assert hll.estimate([]) == 0.0
    assert hll.estimate([""]) == 0.0
    small = [f"k{i}" for i in range(300)]
    assert hll.estimate(small + small) == 300.0          # exact while the sketch would hold coupons
    for n in (1000, 20000, 200000):
        e = hll.estimate(f"key-{i}" for i in range(n))
        assert abs(e - n) / n < 0.05, (n, e)               # HLL_4 lgK=12: ~1.6% standard error
