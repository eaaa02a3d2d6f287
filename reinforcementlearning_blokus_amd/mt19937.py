"""numpy's legacy MT19937 (`np.random.RandomState(seed)`) for many integer seeds at once.

The arena builds one MCTSAgent per game and search seat, and each one seeds two
RandomState streams with its agent seed: ZobristHash(seed) draws the 2,088 uint64 keys
(reference mcts/zobrist.py:41-68) and the rollout HeuristicAgent(seed) keeps the fresh
state (reference agents/heuristic_agent.py:23-27).  Constructing a RandomState costs
about 0.1-0.3 ms of interpreter work, which for 1,024 games added a sixth to a config-4
step.  These functions run the same generator on arrays of seeds:

* `seed_states(seeds)`: the 624-word state after RandomState(seed) (init_genrand; numpy
  accepts integer seeds 0 .. 2**32 - 1 and raises ValueError otherwise, as here);
* `uint64_draws(seeds, k)`: the first k values of RandomState(seed).randint(0, 2**64,
  dtype=np.uint64) -- a full-range uint64 draw is one next_uint64 per value, the high
  word first.

`tests/test_mt19937.py` checks both against RandomState on random seeds; callers check a
sample against the agents they replace and fall back to building them.
"""
from __future__ import annotations

import numpy as np

N, M = 624, 397
ROWS = 48  # seeds per block in uint64_draws: 48 x 624 x 4 B = 117 KB
_MATRIX_A = np.uint32(0x9908B0DF)
_UPPER, _LOWER = np.uint32(0x80000000), np.uint32(0x7FFFFFFF)
_ONE = np.uint32(1)


def seed_states(seeds) -> np.ndarray:
    """uint32[n, 624]: init_genrand(seed) for each seed (the state RandomState(seed) holds
    before its first draw; its position is 624)."""
    s = np.asarray(list(seeds) if not isinstance(seeds, np.ndarray) else seeds)
    if s.size and (s.dtype.kind not in "iu" or int(s.min()) < 0 or int(s.max()) > 0xFFFFFFFF):
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    s = s.astype(np.uint32).reshape(-1)
    mt = np.empty((len(s), N), np.uint32)
    mt[:, 0] = s
    prev = s
    with np.errstate(over="ignore"):  # arithmetic mod 2**32, as the C code's
        for i in range(1, N):
            prev = np.uint32(1812433253) * (prev ^ (prev >> np.uint32(30))) + np.uint32(i)
            mt[:, i] = prev
    return mt


def _mix(cur, nxt, far):
    y = (cur & _UPPER) | (nxt & _LOWER)
    return far ^ (y >> _ONE) ^ ((y & _ONE) * _MATRIX_A)


def _twist(mt: np.ndarray) -> np.ndarray:
    """One generation of all 624 words (uint32 [n, 624]) in the order the scalar loop
    writes them: words 0..226 read old words 397..623, words 227..622 read the new words
    0..395, word 623 reads the new words 0 and 396."""
    new = np.empty_like(mt)
    new[:, :N - M] = _mix(mt[:, :N - M], mt[:, 1:N - M + 1], mt[:, M:])
    for lo in range(N - M, N - 1, N - M):  # 227..453, 454..622: each reads new words 227 back
        hi = min(lo + (N - M), N - 1)
        new[:, lo:hi] = _mix(mt[:, lo:hi], mt[:, lo + 1:hi + 1], new[:, lo - (N - M):hi - (N - M)])
    new[:, N - 1] = _mix(mt[:, N - 1], new[:, 0], new[:, M - 1])
    return new


def _temper(y: np.ndarray) -> np.ndarray:
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def uint32_draws(states: np.ndarray, count: int) -> np.ndarray:
    """uint32[n, count]: the first count genrand_int32 outputs of fresh states (position
    624, so the first output follows a twist)."""
    mt = np.asarray(states, np.uint32)
    out = np.empty((mt.shape[0], count), np.uint32)
    done = 0
    while done < count:
        mt = _twist(mt)
        k = min(N, count - done)
        out[:, done:done + k] = _temper(mt[:, :k])
        done += k
    return out


def uint64_draws(seeds, k: int, states=None) -> np.ndarray:
    """uint64[n, k]: RandomState(seed).randint(0, 2**64, size=k, dtype=np.uint64) for each
    seed (next_uint64 = high word << 32 | low word); `states`: seed_states(seeds), if the
    caller has them."""
    states = seed_states(seeds) if states is None else np.asarray(states, np.uint32)
    n = states.shape[0]
    pairs = np.empty((n, k, 2), np.uint32)  # (low, high) words: a little-endian uint64
    # blocks of ROWS seeds: the generator's temporaries stay below glibc's mmap threshold
    # (128 KB), so they come from the heap instead of fresh pages (a first call over
    # 1,024 seeds otherwise spends most of its time in page faults)
    for r0 in range(0, n, ROWS):
        w = uint32_draws(states[r0:r0 + ROWS], 2 * k)
        pairs[r0:r0 + ROWS, :, 0] = w[:, 1::2]
        pairs[r0:r0 + ROWS, :, 1] = w[:, 0::2]
    return pairs.view("<u8").reshape(n, k).astype(np.uint64, copy=False)


def python_random_states(seeds) -> np.ndarray:
    """uint32[n, 625]: random.Random(seed).getstate()[1] for each non-negative integer seed
    (CPython's init_by_array over the seed's 32-bit words, least significant first; the
    position word is 624).  Seeds with different word counts run as separate groups."""
    seeds = [int(s) for s in seeds]
    out = np.zeros((len(seeds), N + 1), np.uint32)
    out[:, N] = N
    if any(s < 0 for s in seeds):  # (random.seed takes abs(); the arena's seeds are >= 0)
        raise ValueError("python_random_states: negative seed")
    nwords = [max(1, (s.bit_length() + 31) // 32) for s in seeds]
    for kl in sorted(set(nwords)):
        rows = np.array([i for i, w in enumerate(nwords) if w == kl], np.int64)
        key = np.array([[(seeds[i] >> (32 * j)) & 0xFFFFFFFF for j in range(kl)] for i in rows], np.uint32)
        mt = np.repeat(seed_states([19650218]), len(rows), axis=0)
        with np.errstate(over="ignore"):
            i, j = 1, 0
            for _ in range(max(N, kl)):
                prev = mt[:, i - 1]
                mt[:, i] = (mt[:, i] ^ ((prev ^ (prev >> np.uint32(30))) * np.uint32(1664525))) + key[:, j] + \
                    np.uint32(j)
                i, j = i + 1, j + 1
                if i >= N:
                    mt[:, 0] = mt[:, N - 1]
                    i = 1
                if j >= kl:
                    j = 0
            for _ in range(N - 1):
                prev = mt[:, i - 1]
                mt[:, i] = (mt[:, i] ^ ((prev ^ (prev >> np.uint32(30))) * np.uint32(1566083941))) - np.uint32(i)
                i += 1
                if i >= N:
                    mt[:, 0] = mt[:, N - 1]
                    i = 1
        mt[:, 0] = 0x80000000
        out[rows, :N] = mt
    return out
