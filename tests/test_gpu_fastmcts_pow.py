"""k_fastmcts's UCB1 selection on the device reproduces the reference's argmax at
near-ties decided by the last ulp of (2 * math.log(N) / v) ** 0.5
(agents/fast_mcts_agent.py:45-56): constructed children whose UCB values tie exactly
under sqrt but not under CPython's pow, in both directions, through the
bk_debug_fastmcts_select diagnostic (the same device function k_fastmcts calls).
Tolerance: exact (argmax index)."""
import math

import numpy as np
import pytest

from reinforcementlearning_blokus_amd import _native as N

pytestmark = pytest.mark.gpu
C = 1.414
NMAX = 4097
LOGS = np.array([0.0] + [math.log(k) for k in range(1, NMAX + 1)])


@pytest.fixture(scope="module")
def gpu():
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU
    return BlokusGPU(0)


def ucb_ref(total, visits, n):
    """FastMCTSNode.ucb1_value, verbatim arithmetic (fast_mcts_agent.py:51-53)."""
    exploitation = total / visits
    exploration = C * (2 * math.log(n) / visits) ** 0.5
    return exploitation + exploration


def ref_select(children, n):
    """max(children, key=ucb1_value): the first child with the largest value."""
    vals = [ucb_ref(t, v, n) for v, t in children]
    return vals.index(max(vals))


def near_ties(up: bool, want=6):
    """(N, [(visits, total) ...]) with two children that tie under sqrt arithmetic and
    are separated by CPython's pow; the pow-favoured child is listed second when up
    (pow rounds above sqrt), first otherwise."""
    off, ent = N.pow_half_fix(LOGS)
    found = []
    for n in range(50, NMAX + 1):
        fixed = {w >> 1: w & 1 for w in ent[off[n]:off[n + 1]].tolist()}
        for va, f in fixed.items():
            if bool(f) != up:
                continue
            xa = 2 * math.log(n) / va
            ua_sqrt, ua_pow = C * math.sqrt(xa), C * xa ** 0.5
            if ua_sqrt == ua_pow:  # the ulp vanished in c * s
                continue
            vb = next((v for v in range(max(1, va - 20), va + 20) if v != va and v <= n and v not in fixed), None)
            if vb is None:
                continue
            xb = 2 * math.log(n) / vb
            tb = (ua_sqrt - C * math.sqrt(xb)) * vb
            for _ in range(200):  # walk tb until B's value equals A's sqrt value exactly
                ub = tb / vb + C * math.sqrt(xb)
                if ub == ua_sqrt:
                    break
                tb = math.nextafter(tb, math.inf if ub < ua_sqrt else -math.inf)
            else:
                continue
            a, b = (va, 0.0), (vb, tb)
            kids = [b, a] if up else [a, b]
            assert ucb_ref(*kids[0][::-1], n) != ucb_ref(*kids[1][::-1], n)
            found.append((n, kids))
            break
        if len(found) >= want:
            break
    assert found
    return found


@pytest.mark.parametrize("up", [True, False])
def test_near_tie_follows_cpython_pow(gpu, up):
    for n, kids in near_ties(up):
        visits = [v for v, _ in kids]
        totals = [t for _, t in kids]
        want = ref_select(kids, n)
        # the tie under sqrt would pick child 0; the reference picks the other one
        sqrt_vals = [t / v + C * math.sqrt(2 * math.log(n) / v) for v, t in kids]
        assert sqrt_vals[0] == sqrt_vals[1] and want == 1
        got = gpu.fastmcts_select(visits, totals, n, LOGS, C)
        assert got == want, (n, kids)


def test_random_children_match_reference_argmax(gpu):
    rng = np.random.RandomState(5)
    for _ in range(40):
        k = int(rng.randint(1, 300))
        n = int(rng.randint(k, NMAX))
        visits = rng.randint(1, max(2, n // k + 2), size=k)
        totals = rng.rand(k) * visits * 2.0
        kids = list(zip(visits.tolist(), totals.tolist()))
        assert gpu.fastmcts_select(visits, totals, n, LOGS, C) == ref_select(kids, n)
