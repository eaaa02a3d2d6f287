"""Cooperative bk_mcts (k_mcts_coop / k_mcts_coop_h: one 64-lane wave per search, the
kernel bk_mcts picks for batches of <= 4 searches per CU) against the one-search-per-lane
kernels (k_mcts / k_mcts_h) on the same batches: every output bit-identical -- results,
per-iteration rewards and TT-hit flags, the rollout agent's MT state, the TTs and the
node pools.  Both are pinned to the reference elsewhere (tests/test_gpu_mcts.py,
tests/test_gpu_heuristic*.py run the default kernel; test_gpu_config5.py the per-lane one).

Reference: mcts/mcts_agent.py:304-582 (search), agents/heuristic_agent.py:39-244
(rollout policy), agents/random_agent.py:33-50.  Tolerance: exact.
"""
import numpy as np
import pytest

from reinforcementlearning_blokus_amd import _native as N

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from reinforcementlearning_blokus_amd.gpu import BlokusGPU
    return BlokusGPU(0)


def _run(gpu, roots, sets, iters, policy, max_roll, coop, monkeypatch, seed0=100, time_limit_us=0, env=None):
    from reinforcementlearning_blokus_amd.gpu import MctsTT
    from reinforcementlearning_blokus_amd.mcts.zobrist import ZobristHash, flat_keys, hash_states
    from reinforcementlearning_blokus_amd.workloads import numpy_mt_states
    # the handle's overrides (bk_set_tuning; the library reads the environment only when
    # a handle is created)
    gpu.tune(MCTS_COOP=1 if coop else 0, MCTS_SPREAD=None, MCTS_PAIR=None, COOP_BAL=None, COOP_WALK=None)
    gpu.tune(**{k[3:]: int(v) for k, v in (env or {}).items()})
    n = len(roots)
    zob = np.stack([flat_keys(ZobristHash(seed=t)) for t in range(3)])
    zi = (np.arange(n) % 3).astype(np.int32)
    rh = np.array([hash_states(roots[g:g + 1], zob[zi[g]])[0] for g in range(n)], np.uint64)
    pl = (roots["current_player"] & 3).astype(np.uint8)
    mt = numpy_mt_states(range(seed0, seed0 + n))
    tt = MctsTT(n)
    r = gpu.mcts(roots, sets, pl, rh, iterations=iters, zobrist=zob, zobrist_index=zi, mt_state=mt, tt=tt,
                 max_rollout_moves=max_roll, want_nodes=True, rollout_policy=policy, time_limit_us=time_limit_us)
    return r, mt, tt


@pytest.mark.parametrize("policy,n,iters,max_roll", [
    (N.MCTS_ROLLOUT_RANDOM, 70, 160, 50),
    (N.MCTS_ROLLOUT_RANDOM, 5, 600, 12),
    (N.MCTS_ROLLOUT_HEURISTIC, 40, 48, 50),
    (N.MCTS_ROLLOUT_HEURISTIC, 3, 200, 8),
])
def test_coop_equals_per_lane(gpu, monkeypatch, policy, n, iters, max_roll):
    from reinforcementlearning_blokus_amd.workloads import frontier_roots
    roots, sets = frontier_roots(gpu, n, 14 + n % 9, seed=777 + n)
    a, mta, tta = _run(gpu, roots, sets, iters, policy, max_roll, True, monkeypatch)
    b, mtb, ttb = _run(gpu, roots, sets, iters, policy, max_roll, False, monkeypatch)
    assert (a["out"]["status"] & ~np.uint32(N.MCTS_EUNCERT) == 0).all()
    assert (a["out"]["iterations_run"] == iters).all()
    assert a["out"].tobytes() == b["out"].tobytes()
    assert np.array_equal(a["rewards"], b["rewards"]) and np.array_equal(a["hit_flags"], b["hit_flags"])
    assert np.array_equal(mta, mtb)
    assert np.array_equal(tta.keys, ttb.keys) and np.array_equal(tta.count, ttb.count)
    assert a["nodes"].tobytes() == b["nodes"].tobytes()


@pytest.mark.parametrize("n,iters,max_roll", [(70, 160, 50), (333, 96, 50), (9, 400, 20)])
def test_pair_split_equals_single_lane(gpu, monkeypatch, n, iters, max_roll):
    """k_mcts_pair (spread 2: the odd lane of each pair counts half of the even lane's
    stencil entries, count_class_pair) against k_mcts with one lane per search (spread 1)
    and against k_mcts at spread 2 without the split: every output bit-identical."""
    from reinforcementlearning_blokus_amd.workloads import frontier_roots
    roots, sets = frontier_roots(gpu, n, 10 + n % 13, seed=4242 + n)
    pol = N.MCTS_ROLLOUT_RANDOM
    a, mta, tta = _run(gpu, roots, sets, iters, pol, max_roll, False, monkeypatch,
                       env={"BK_MCTS_SPREAD": "2", "BK_MCTS_PAIR": "1"})
    for env in ({"BK_MCTS_SPREAD": "1", "BK_MCTS_PAIR": "0"}, {"BK_MCTS_SPREAD": "2", "BK_MCTS_PAIR": "0"}):
        b, mtb, ttb = _run(gpu, roots, sets, iters, pol, max_roll, False, monkeypatch, env=env)
        assert (a["out"]["status"] == 0).all()
        assert (a["out"]["iterations_run"] == iters).all()
        assert a["out"].tobytes() == b["out"].tobytes()
        assert np.array_equal(a["rewards"], b["rewards"]) and np.array_equal(a["hit_flags"], b["hit_flags"])
        assert np.array_equal(mta, mtb)
        assert np.array_equal(tta.keys, ttb.keys) and np.array_equal(tta.count, ttb.count)
        assert a["nodes"].tobytes() == b["nodes"].tobytes()


def test_coop_time_limit_stops(gpu, monkeypatch):
    """A timed cooperative search stops at an iteration boundary past its limit."""
    from reinforcementlearning_blokus_amd.workloads import frontier_roots
    roots, sets = frontier_roots(gpu, 4, 20, seed=99)
    r, _, _ = _run(gpu, roots, sets, 200000, N.MCTS_ROLLOUT_RANDOM, 50, True, monkeypatch, time_limit_us=30000)
    it = r["out"]["iterations_run"]
    assert (it >= 1).all() and (it < 200000).all()


@pytest.mark.parametrize("n,iters,root_plies", [(40, 48, 6), (24, 64, 30)])
def test_coop_balanced_heuristic_pass_equals_per_lane_sums(gpu, monkeypatch, n, iters, root_plies):
    """k_mcts_coop_h's balanced HeuristicAgent pass (the ply's legal moves listed in LDS,
    e evaluated 64 moves at a time, coop_heur_balanced) against the per-lane orientation
    sums it replaces (BK_COOP_BAL=0, also its fallback above 2,048 legal moves), early
    (6-ply roots: many legal moves) and late (30-ply roots): every output bit-identical."""
    from reinforcementlearning_blokus_amd.workloads import frontier_roots
    roots, sets = frontier_roots(gpu, n, root_plies, seed=31337 + n)
    pol = N.MCTS_ROLLOUT_HEURISTIC
    a, mta, tta = _run(gpu, roots, sets, iters, pol, 50, True, monkeypatch, env={"BK_COOP_BAL": "1"})
    b, mtb, ttb = _run(gpu, roots, sets, iters, pol, 50, True, monkeypatch, env={"BK_COOP_BAL": "0"})
    assert (a["out"]["status"] & ~np.uint32(N.MCTS_EUNCERT) == 0).all()
    assert (a["out"]["iterations_run"] == iters).all()
    assert a["out"].tobytes() == b["out"].tobytes()
    assert np.array_equal(a["rewards"], b["rewards"]) and np.array_equal(a["hit_flags"], b["hit_flags"])
    assert np.array_equal(mta, mtb)
    assert np.array_equal(tta.keys, ttb.keys) and np.array_equal(tta.count, ttb.count)
    assert a["nodes"].tobytes() == b["nodes"].tobytes()


@pytest.mark.parametrize("coop", ["1", "0"])
def test_device_root_hash_equals_host_hash(monkeypatch, coop):
    """bk_mcts with root_hash NULL hashes the roots on the device (k_root_hash,
    ZobristHash.hash_board): the searches -- results, rewards, TT, RNG states -- equal the
    ones given the host's hash_states values, per-agent key tables included."""
    import torch

    from reinforcementlearning_blokus_amd.gpu import BlokusGPU
    from reinforcementlearning_blokus_amd.workloads import MctsBatch, frontier_roots
    monkeypatch.setenv("BK_MCTS_COOP", coop)
    gpu = BlokusGPU(0)
    roots, sets = frontier_roots(gpu, 48, 18, seed=77)
    outs = []
    for host_hash in (True, False):
        b = MctsBatch(gpu, roots, sets, iterations=24, seed0=5, n_tables=3, want_rewards=True)
        if not host_hash:
            b.root_hash = None
        b.run()
        torch.cuda.synchronize()
        outs.append((b.results().copy(), b.mt.cpu().numpy(), b.tt_keys.cpu().numpy(), b.rewards.cpu().numpy()))
    for x, y in zip(*outs):
        assert np.array_equal(x, y)
