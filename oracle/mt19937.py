"""CPU restatement of np_random's generator for the Coverage expert's fallback draws.

TEST INFRASTRUCTURE ONLY: imported by tests/ (never by the product). The reference's
controller(greedy=True) gives a robot with no reachable unvisited target
`self.np_random.choice(self.n_actions)` (gym_flock/envs/spatial/coverage.py:861-864), a
numpy legacy RandomState (numpy is the reference's dependency, not vendored: its
MT19937 is the published Matsumoto & Nishimura 1998 generator). This restates, in
plain Python loops, what the device does for COV_GREEDY_RNG (coverage_internal.h
mt_regen / mt_temper): choice(4) with uniform p is randint(0, 4), one tempered 32-bit
output masked to 2 bits (no rejection: the mask equals the range); the 624-word key is
regenerated when the position reaches 624. Pinned against numpy.random.RandomState
itself (tests/test_oracle_mt19937.py), whose state layout (get_state: key words and
position) is also the C-ABI's (cov_set_rng). Also restated: RandomState(seed)'s seeding
(mt19937_seed, the generator's init_genrand) and the legacy permutation / choice without
replacement (Fisher-Yates from the top, random_interval's masked rejection), which
VecCoverage.reset's draws (coverage.py:405-424) use and the device reset
(cov_reset_seeded) restates.
"""
N, M = 624, 397
UPPER, LOWER, MATRIX_A = 0x80000000, 0x7FFFFFFF, 0x9908B0DF


def regenerate(key):
    """The next 624 key words (in place on a list of ints)."""
    for i in range(N):
        y = (key[i] & UPPER) | (key[(i + 1) % N] & LOWER)
        key[i] = key[(i + M) % N] ^ (y >> 1) ^ (MATRIX_A if y & 1 else 0)
    return key


def temper(y):
    y ^= y >> 11
    y ^= (y << 7) & 0x9D2C5680
    y ^= (y << 15) & 0xEFC60000
    return (y ^ (y >> 18)) & 0xFFFFFFFF


def choice4(key, pos, n):
    """n draws of choice(4) from the stream (key, pos); returns (draws, key, pos) with the
    stream advanced, as RandomState.get_state() would show it."""
    key = [int(k) for k in key]
    out = []
    for _ in range(n):
        if pos == N:
            regenerate(key)
            pos = 0
        out.append(temper(key[pos]) & 3)
        pos += 1
    return out, key, pos


def seed(s):
    """RandomState(s)'s state for an integer seed in [0, 2**32): (key, pos = 624)."""
    key = [0] * N
    s &= 0xFFFFFFFF
    for p in range(N):
        key[p] = s
        s = (1812433253 * (s ^ (s >> 30)) + p + 1) & 0xFFFFFFFF
    return key, N


def _next(state):
    key, pos = state
    if pos == N:
        regenerate(key)
        pos = 0
    state[1] = pos + 1
    return temper(key[pos])


def permutation(key, pos, n):
    """RandomState.permutation(n) from the stream (key, pos): (perm, key, pos).
    choice(a, size, replace=False) is a[permutation(len(a))[:size]]."""
    state = [[int(k) for k in key], pos]
    x = list(range(n))
    for i in range(n - 1, 0, -1):
        mask = i
        for sh in (1, 2, 4, 8, 16):
            mask |= mask >> sh
        while True:
            v = _next(state) & mask
            if v <= i:
                break
        x[i], x[v] = x[v], x[i]
    return x, state[0], state[1]
