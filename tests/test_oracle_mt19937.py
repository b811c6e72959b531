"""The restated np_random stream (oracle/mt19937.py) against numpy's RandomState itself:
the draws of choice(4) (coverage.py:861-864), singly and batched, across key
regenerations, and the stream state after them (the C-ABI's cov_set_rng layout)."""
import numpy as np
import pytest

from oracle import mt19937 as mt


@pytest.mark.parametrize("seed", [0, 6, 13, 1000])
@pytest.mark.parametrize("skip", [0, 1, 400, 623, 624, 1500])
def test_choice4_stream_matches_randomstate(seed, skip):
    rs = np.random.RandomState(seed)
    rs.randint(0, 4, size=skip)  # move the position (one output per draw)
    _, key, pos, _, _ = rs.get_state()
    n = 700  # crosses a regeneration from any position
    got, key2, pos2 = mt.choice4(key, pos, n)
    want = [rs.choice(4) for _ in range(n)]
    assert got == want
    st = rs.get_state()
    assert pos2 == st[2]
    np.testing.assert_array_equal(np.array(key2, np.uint32), st[1])


def test_batched_choice_is_the_same_stream():
    """The env's batched fallback draw (choice(4, size=k), envs/spatial/coverage.py) takes
    the same outputs as k single draws in robot order, as the device does."""
    a, b = np.random.RandomState(3), np.random.RandomState(3)
    for k in (1, 5, 200, 624, 31):
        np.testing.assert_array_equal(a.choice(4, size=k), [b.choice(4) for _ in range(k)])


def test_reset_draws_then_fallbacks():
    """The stream a reference env's fallbacks continue: seed, reset's two choice draws
    without replacement (coverage.py:405-424), then choice(4)s."""
    rs = np.random.RandomState(6)
    rs.choice(np.arange(90), size=(6,), replace=False)
    rs.choice(np.arange(90) + 6, size=(45,), replace=False)
    _, key, pos, _, _ = rs.get_state()
    got, _, _ = mt.choice4(key, pos, 50)
    assert got == [rs.choice(4) for _ in range(50)]


@pytest.mark.parametrize("s", [0, 1, 40, 2 ** 32 - 1])
def test_seed_matches_randomstate(s):
    key, pos = mt.seed(s)
    st = np.random.RandomState(s).get_state()
    np.testing.assert_array_equal(np.array(key, np.uint32), st[1])
    assert pos == st[2]


@pytest.mark.parametrize("s,n", [(0, 552), (7, 1), (7, 2), (13, 90), (40, 1000)])
def test_permutation_and_choice_without_replacement(s, n):
    """The reset's draws: two choices without replacement from one stream
    (VecCoverage.reset, coverage.py:405-424), then the stream state."""
    rs = np.random.RandomState(s)
    key, pos = mt.seed(s)
    r = max(1, n // 3)
    want1 = rs.choice(np.arange(n), size=(r,), replace=False)
    want2 = rs.choice(np.arange(n) + 5, size=(int(n * 0.5),), replace=False)
    p1, key, pos = mt.permutation(key, pos, n)
    p2, key, pos = mt.permutation(key, pos, n)
    np.testing.assert_array_equal(np.array(p1[:r]), want1)
    np.testing.assert_array_equal(np.array(p2[:int(n * 0.5)]) + 5, want2)
    st = rs.get_state()
    assert pos == st[2]
    np.testing.assert_array_equal(np.array(key, np.uint32), st[1])
