"""SURVEY 8(c) P3 on the timed path: the bench's exact config-3 call (bench.py
run_config3, naive order, BK_RNG_PHILOX) replayed playout by playout on the oracle.

* Roots: 256 synthetic positions from bk_advance (20 Philox plies from the empty board,
  seed 20260301, playout ids 0..255), equal to the oracle's replay of the same streams.
* Playouts: 256 roots x 1,024 rollouts = 262,144 arena playouts with seed
  20260301 * 7919 + 1000 (the first timed step), game j's rollouts contiguous (root j //
  1,024), on device buffers as the bench runs them.  A strided sample is compared field
  for field with the oracle's Philox replay (scores, winner mask, plies, passes, turns,
  draws, status); all 262,144 are checked by size-independent properties.

The oracle's move lists are the reference's (tests/test_oracle_golden.py), and its
Philox is pinned by Random123's known-answer vectors (tests/test_oracle_philox.py), so
an equal result record means the GPU played the reference engine's game for that stream.
Reference: engine/move_generator.py:153-259 (naive order), analytics/tournament/
arena_runner.py:652-697 (arena loop), engine/game.py:182-349 (game over, scoring).
Tolerance: exact.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import pyoracle as O
from reinforcementlearning_blokus_amd import _native as N

pytestmark = pytest.mark.gpu

SEED = 20260301              # bench.py --seed default, rank 0
GAMES, ROLLOUTS, PLIES = 256, 1024, 20


@pytest.fixture(scope="module")
def gpu():
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU
    return BlokusGPU(0)


def _oracle_root(pid):
    b = O.new_board()
    O.playout_arena_philox(b, SEED, pid, O.ORDER_NAIVE, max_plies=PLIES)
    return b


@pytest.fixture(scope="module")
def roots(gpu):
    from reinforcementlearning_blokus_amd.gpu import empty_state
    st = gpu.advance(empty_state(), GAMES, PLIES, seed=SEED, root_index=np.zeros(GAMES, dtype=np.int32))
    return st


def test_bench_roots_equal_oracle_replay(roots):
    with ThreadPoolExecutor(16) as ex:
        boards = list(ex.map(_oracle_root, range(GAMES)))
    ref = np.frombuffer(bytes(O.states_array(boards)), dtype=N.STATE_DTYPE)
    for f in ("planes", "used", "first_move", "current_player", "move_count"):
        assert np.array_equal(roots[f], ref[f]), f
    assert (roots["move_count"] == PLIES).all()


def test_bench_config3_playouts_replay_exactly(gpu, roots):
    import torch
    dev = torch.device("cuda", 0)
    n = GAMES * ROLLOUTS
    seed = SEED * 7919 + 1000
    rt = torch.from_numpy(roots.view(np.uint8).reshape(GAMES, 256).copy()).to(dev)
    idx = torch.arange(n, dtype=torch.int32, device=dev) // ROLLOUTS
    out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    gpu.rollout(rt, n, semantics=N.SEM_ARENA, rng=N.RNG_PHILOX, seed=seed, root_index=idx, out=out)
    torch.cuda.synchronize()
    res = out.cpu().numpy().view(N.RESULT_DTYPE).reshape(-1)

    # size-independent properties over all 262,144 playouts
    assert (res["status"] == 0).all()
    sc = res["scores"].astype(np.int32)
    best = sc.max(axis=1, keepdims=True)
    assert np.array_equal(((sc == best) * (1 << np.arange(4))).sum(axis=1), res["winner_mask"])
    assert (res["draws"] >= res["plies"] // 2).all()  # a forced move (one legal) draws nothing
    assert (res["turns"] == res["plies"].astype(np.int32) + res["passes"]).all()
    root_cells = np.array([[bin(int(x)).count("1") for x in roots["planes"][g].reshape(-1)] for g in range(GAMES)])
    assert (res["plies"] > 0).mean() > 0.99 and (res["plies"] <= 84 - PLIES).all()
    # all 21 pieces used by nobody at the root: cells grow by >= 1 per own placement
    assert (sc.sum(axis=1) >= root_cells.sum(axis=1)[np.arange(n) // ROLLOUTS] + res["plies"]).all()

    # strided sample, field for field against the oracle's replay of the same streams
    oroots = (O.State * GAMES).from_buffer_copy(roots.tobytes())
    sample = list(range(0, n, 37)) + [n - 1]

    def one(pid):
        b = O.unpack(oroots[pid // ROLLOUTS])
        r, _ = O.playout_arena_philox(b, seed, pid, O.ORDER_NAIVE)
        return pid, bytes(r)

    with ThreadPoolExecutor(16) as ex:
        refs = list(ex.map(one, sample))
    bad = [pid for pid, rb in refs if res[pid].tobytes() != rb]
    assert not bad, (len(bad), bad[:8])
