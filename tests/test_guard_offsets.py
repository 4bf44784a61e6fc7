"""The reuse / window guard's sampling restated on the host (tests/helpers.py guard_words,
guard_chunk -- kernels.hip guard_offset): the chunks partition the payload's words, the last
chunk is the last word alone, each generation samples one word per chunk plus the first word,
and every word is sampled within W consecutive generations (W = the longest chunk), from any
starting generation."""
import pytest

from tests.helpers import GUARD_SAMPLES, guard_chunk, guard_period, guard_words


@pytest.mark.parametrize("n16", [1, 2, 7, 4095, 4096, 4097, 25_008, 100_000, 2_793_490])
def test_chunks_partition_and_rotation_covers(n16):
    s = min(n16, GUARD_SAMPLES)
    W = guard_period(n16)
    # chunk ranges are disjoint, in order, cover [0, n16)
    prev_hi, k_prev = 0, -1
    probe = sorted({0, n16 - 1, n16 // 2, n16 // 3} | set(range(0, n16, max(1, n16 // 500))))
    for w in probe:
        k, (lo, hi) = guard_chunk(n16, w)
        assert lo <= w < hi and k >= k_prev
        if k != k_prev:
            assert lo >= prev_hi
            prev_hi, k_prev = hi, k
    assert guard_chunk(n16, n16 - 1)[1] == (n16 - 1, n16)     # the last word alone
    for g in (0, 1, 5, 12345):
        words = guard_words(n16, g)
        assert 0 in words and n16 - 1 in words and len(words) <= s + 1
    if n16 > 100_000:
        return                               # the full coverage sweep below is O(W * s)
    for start in (0, 3):
        covered = set()
        for g in range(start, start + W):
            covered |= guard_words(n16, g)
        assert covered == set(range(n16)), (n16, start, W)
    assert W == 1 or any(len(guard_words(n16, g) ^ guard_words(n16, g + 1)) for g in range(3))
