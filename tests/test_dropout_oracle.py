"""CPU checks of the dropout oracle (oracle/dropout_ref.py), the checker of the GPU dropout tests."""
import numpy as np

from oracle.dropout_ref import dropout_keep_mask, keep_threshold, philox


def test_keep_threshold_matches_reference_formula():
    # flash_api.cpp:94-100: p = 1.f - p_dropout; uint8_t(std::floor(p * 255.0))
    for p, t in [(0.0, 255), (0.1, 229), (0.17, 211), (0.5, 127), (0.9, 25)]:
        assert keep_threshold(p) == t


def test_philox_is_deterministic_and_keyed():
    a = philox(1234, np.arange(8, dtype=np.uint64), 7)
    b = philox(1234, np.arange(8, dtype=np.uint64), 7)
    c = philox(1235, np.arange(8, dtype=np.uint64), 7)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert not all(np.array_equal(x, y) for x, y in zip(a, c))
    assert all(int(x.max()) < 2 ** 32 for x in a)


def test_element_map_is_a_bijection_per_block():
    # within a 16 x 32 block every (lane, byte) pair is used by exactly one element
    r = np.arange(16)[:, None]
    c = np.arange(32)[None, :]
    lane = 4 * (r % 8) + (c % 8) // 2
    byte = 8 * (c // 16) + (c % 2) + 2 * (r // 8) + 4 * ((c % 16) // 8)
    keys = (lane * 16 + byte).ravel()
    assert len(set(keys.tolist())) == 512 and keys.min() == 0 and keys.max() == 511


def test_mask_rate_and_independence():
    m = dropout_keep_mask(42, 0, 0, 0, 1, 512, 512, 0.3)
    assert abs(m.mean() - (keep_threshold(0.3) + 1) / 256) < 0.01
    m2 = dropout_keep_mask(42, 0, 0, 1, 2, 512, 512, 0.3)     # another head: another stream
    m3 = dropout_keep_mask(42, 64, 0, 0, 1, 512, 512, 0.3)    # another offset
    assert (m != m2).mean() > 0.3 and (m != m3).mean() > 0.3
    # a sub-block is the top-left corner of the larger mask (the stream depends on (row, col) only)
    assert np.array_equal(dropout_keep_mask(42, 0, 0, 0, 1, 100, 70, 0.3), m[:100, :70])
