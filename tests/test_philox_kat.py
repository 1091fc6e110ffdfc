"""Known-answer tests of the RNG that replaces randf() (include/randf.h:6-11).

DESIGN.md §3 claims the per-path stream is Philox4x32-10 (Salmon, Moraes,
Dror & Shaw, "Parallel random numbers: as easy as 1, 2, 3", SC'11). These
vectors are the philox4x32 10-round entries of Random123's published
known-answer file (kat_vectors: counter words, key words, expected output),
so they pin the generator itself -- not just the agreement of the kernel
with the oracle, which were written from the same description. Checked for
the oracle (test infrastructure), the library's host build (CPU) and, on the
GPU, the device build the path kernel inlines.
"""
import numpy as np
import pytest

import oracle_binding as ob
from ipt_amd import capi

# (ctr0..3, key0..1) -> out0..3, Random123 kat_vectors "philox4x32 10"
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_oracle_philox_kat(oracle, ctr, key, want):
    assert [int(x) for x in ob.philox(ctr, key)] == list(want)


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_library_host_philox_kat(ctr, key, want):
    assert [int(x) for x in capi.philox([ctr], key)[0]] == list(want)


def test_stream_composition(oracle):
    """Draw k of path (pass s, pixel p) is word k%4 of philox({k/4, s, p, 0},
    seed) mapped (w >> 8) * 2^-24: the oracle's randf() stream
    against the library's blocks."""
    seed = 20241223
    key = (seed & 0xffffffff, seed >> 32)
    rng = np.random.default_rng(5)
    for _ in range(50):
        s, p, k = (int(x) for x in rng.integers(0, [4096, 1 << 24, 700]))
        w = capi.philox([(k // 4, s, p, 0)], key)[0][k % 4]
        want = np.float32(int(w) >> 8) * np.float32(2.0 ** -24)
        assert np.float32(oracle.ipt_oracle_randf(seed, s, p, k)) == want


@pytest.mark.gpu
def test_device_philox_kat(gpu_ctx):
    for ctr, key, want in KAT:
        assert [int(x) for x in capi.philox([ctr], key, gpu_ctx)[0]] == list(want)
    # and a batch of random counters against the host build
    rng = np.random.default_rng(11)
    ctr = rng.integers(0, 1 << 32, size=(4096, 4), dtype=np.uint64).astype(np.uint32)
    key = (0x9E3779B9, 0x13371337)
    assert np.array_equal(capi.philox(ctr, key, gpu_ctx), capi.philox(ctr, key))
