"""Counter-based RNG (the drop-in replacement of srfi-27 random-real, SURVEY.md
§0.6 / Appendix B): Philox4x32-10 known-answer vectors from the Random123
distribution (kat_vectors, philox4x32 10 rounds) and agreement of the three
implementations (Python host stream, oracle C, and — on the GPU — the kernels,
which the parity tests cover)."""
import math

import pytest

from rtamd import rng

# Random123 kat_vectors: philox4x32 R=10  ctr[4] key[2] -> out[4]
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_philox_kat_python(ctr, key, out):
    assert rng.philox4x32_10(ctr, key) == out


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_philox_kat_oracle(ctr, key, out, oracle_mod):
    assert oracle_mod.philox(ctr, key) == out


def test_unit_conversion_exact_and_open_interval():
    # (hi, lo) -> (2k+1)*2^-53, k = (hi>>12)<<32 | lo : never 0 or 1
    assert rng.u32pair_unit(0, 0) == 2.0 ** -53
    top = rng.u32pair_unit(0xFFFFFFFF, 0xFFFFFFFF)
    assert top < 1.0 and top == (2 * (2 ** 52 - 1) + 1) * 2.0 ** -53
    # every value is an exact odd multiple of 2^-53
    for hi, lo in ((123, 456), (0xABCDEF01, 0x12345678)):
        u = rng.u32pair_unit(hi, lo)
        k = u * 2 ** 53
        assert k == int(k) and int(k) % 2 == 1


@pytest.mark.parametrize("seed,pix,smp", [(0x5EED0002, 0, 0), (0x5EED0002, 1919, 1023), (2**64 - 1, 2**31, 7),
                                          (0, 12345, 99)])
def test_path_stream_python_vs_oracle(seed, pix, smp, oracle_mod):
    want = [rng.path_draw(seed, pix, smp, d) for d in range(11)]
    got = oracle_mod.stream(seed, pix, smp, 0, 11)
    assert got == want
    # a stream resumed at an odd draw index continues identically
    assert oracle_mod.stream(seed, pix, smp, 5, 6) == want[5:]


def test_streams_are_distinct_and_uniformish():
    vals = [rng.path_draw(1, p, s, d) for p in range(40) for s in range(5) for d in range(10)]
    assert len(set(vals)) == len(vals)
    assert all(0.0 < v < 1.0 for v in vals)
    mean = sum(vals) / len(vals)
    assert abs(mean - 0.5) < 0.03
    var = sum((v - mean) ** 2 for v in vals) / len(vals)
    assert abs(var - 1 / 12) < 0.01


def test_host_stream_sequence():
    h = rng.HostStream(0x5EED0001)
    a = [h() for _ in range(9)]
    h2 = rng.HostStream(0x5EED0001)
    assert [h2.random_real() for _ in range(9)] == a
    # host stream = Philox with counter (d>>1, 0, 0xFFFFFFFF, 1)
    w = rng.philox4x32_10((1, 0, 0xFFFFFFFF, 1), rng.split_seed(0x5EED0001))
    assert a[3] == rng.u32pair_unit(w[2], w[3])
    assert not math.isnan(sum(a))
