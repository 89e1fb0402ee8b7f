"""Synthetic action stream: Philox4x32-10 host mirror pinned by the Random123 known-answer
vectors (kat_vectors: philox4x32_10), and the action mapping used by bench.py and the kernel."""
import numpy as np

from avr import _lib

KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def test_philox_known_answers():
    for ctr, key, want in KAT:
        got = _lib.philox4x32_10([np.array([c], np.uint64) for c in ctr], key[0], key[1])
        assert tuple(int(g[0]) for g in got) == want


def test_random_actions_range_and_shape():
    a = _lib.random_actions(1001, np.arange(64), 5)
    assert a.shape == (64, 7) and a.dtype == np.float32
    assert np.all(a >= -1) and np.all(a < 1)
    # 24-bit uniform grid: (k / 2^24) * 2 - 1
    k = (a.astype(np.float64) + 1) / 2 * 2 ** 24
    assert np.allclose(k, np.round(k))


def test_random_actions_keyed_by_global_env_and_step():
    a = _lib.random_actions(1001, np.arange(8), 3)
    b = _lib.random_actions(1001, np.arange(4, 8), 3)
    assert np.array_equal(a[4:], b)                       # independent of batch composition
    c = _lib.random_actions(1001, np.arange(8), 4)
    assert not np.array_equal(a, c)
    d = _lib.random_actions(1002, np.arange(8), 3)
    assert not np.array_equal(a, d)
    big = _lib.random_actions(1001, np.arange(2), (1 << 32) + 3)   # 64-bit step counter
    assert not np.array_equal(big, a[:2])


def test_random_actions_moments():
    a = _lib.random_actions(7, np.arange(4096), 0).astype(np.float64)
    assert abs(a.mean()) < 0.02 and abs(a.var() - 1 / 3) < 0.02
