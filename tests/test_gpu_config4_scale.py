"""Config 4 at its per-GPU size (BASELINE.json configs[3]: 8,192 games over 8 GPUs =
1,024 per GPU): bench.py's exact call -- run_games_batched over games 0..1023 of run
seed 20260301 with bench.CONFIG4_AGENTS (Random / Heuristic / MCTS 64 iterations with
HeuristicAgent rollouts / FastMCTS 1,000 iterations, round-robin seats).

* Every record is checked by size-independent properties (turns = moves + passes,
  winners = the argmax of the final scores, seats = the arena's round-robin, MCTS
  simulations whole searches of 64 iterations, no invalid or truncated games).
* A strided sample of 13 games is compared field for field with the oracle's own
  restatement of the same games (tests/oracle_arena.py, pinned by the reference's
  records in tests/test_oracle_arena.py).
Reference: analytics/tournament/arena_runner.py:578-777.  Tolerance: exact.
"""
import json
from concurrent.futures import ThreadPoolExecutor

import pytest

from tests.oracle_arena import oracle_arena_game

pytestmark = pytest.mark.gpu

N_GAMES = 1024


@pytest.fixture(scope="module")
def run():
    import bench
    from reinforcementlearning_blokus_amd.arena.config import RunConfig
    from reinforcementlearning_blokus_amd.arena.runner import run_games_batched
    cfg = RunConfig.from_dict({"agents": bench.CONFIG4_AGENTS, "num_games": N_GAMES, "seed": 20260301,
                               "seat_policy": "round_robin"})
    return cfg, run_games_batched(cfg, list(range(N_GAMES)))


def test_config4_per_gpu_records_properties(run):
    from reinforcementlearning_blokus_amd.arena.config import game_seed_from_run_seed, seat_assignment_for_game
    cfg, recs = run
    assert [r["game_index"] for r in recs] == list(range(N_GAMES))
    iters = 64
    for r in recs:
        gi = r["game_index"]
        assert r["error"] is None and not r["truncated"] and r["invalid_actions"] == 0, gi
        assert r["moves_made"] + r["passes"] == r["turn_count"], gi
        assert r["seat_assignment"] == seat_assignment_for_game(cfg.agent_names, gi,
                                                                game_seed_from_run_seed(cfg.seed, gi), cfg.seat_policy)
        sc = {int(k): v for k, v in r["final_scores"].items()}
        best = max(sc.values())
        assert r["winner_ids"] == [p for p in range(1, 5) if sc[p] == best], gi
        assert r["is_tie"] == (len(r["winner_ids"]) > 1)
        assert all(0 <= v <= 89 + 15 + 4 * 5 + 16 * 2 for v in sc.values()), gi
        m = r["agent_move_stats"]["mcts"]
        sims = int(m["total_simulations"] or 0)
        assert sims % iters == 0 and sims <= iters * int(m["moves"]), gi
        assert r["moves_made"] >= 4, gi  # every seat has a first move on the empty board


def test_config4_per_gpu_sample_equals_oracle_games(run):
    cfg, recs = run
    sample = list(range(0, N_GAMES, 85))
    with ThreadPoolExecutor(8) as ex:  # ctypes releases the GIL inside the oracle
        refs = list(ex.map(lambda gi: oracle_arena_game(cfg, gi), sample))
    for ref in refs:
        got = recs[ref["game_index"]]
        for f in ("seat_assignment", "winner_ids", "final_scores", "moves_made", "turn_count", "passes"):
            assert got[f] == json.loads(json.dumps(ref[f])), (ref["game_index"], f)
        assert int(got["agent_move_stats"]["mcts"]["total_simulations"] or 0) == ref["simulations"]["mcts"]
