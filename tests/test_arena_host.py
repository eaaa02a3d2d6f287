"""Arena configuration, seeding and summary statistics (CPU) against the reference's
own outputs (tests/golden/arena_runs.json, made by tools/gen_fixtures.py)."""
import json

import pytest

from reinforcementlearning_blokus_amd.arena import RunConfig, compute_summary, game_seed_from_run_seed
from reinforcementlearning_blokus_amd.arena.config import seat_assignment_for_game
from tests.conftest import load_golden

FX = load_golden("arena_runs.json")


def test_seeds_and_randomized_seats_match_reference():
    cfg = RunConfig.from_dict(FX["config"])
    for g in FX["games"]:
        gs = game_seed_from_run_seed(cfg.seed, g["game_index"])
        assert gs == g["game_seed"]
        assert seat_assignment_for_game(cfg.agent_names, g["game_index"], gs, cfg.seat_policy) == g["seat_assignment"]


def test_round_robin_seats():
    names = ["a", "b", "c", "d"]
    assert seat_assignment_for_game(names, 1, 0, "round_robin") == {"1": "b", "2": "c", "3": "d", "4": "a"}


def test_compute_summary_matches_reference():
    cfg = FX["config"]
    got = compute_summary(FX["summary_input"], run_id="fx2", run_seed=cfg["seed"], seat_policy="randomized",
                          agent_names=[a["name"] for a in cfg["agents"]],
                          thinking_time_ms_by_agent={a["name"]: None for a in cfg["agents"]}, run_config=cfg)
    assert json.loads(json.dumps(got, sort_keys=True)) == json.loads(json.dumps(FX["summary"], sort_keys=True))


@pytest.mark.parametrize("bad", [
    {"num_games": 0},
    {"agents": [{"name": "a", "type": "random"}] * 3},
    {"agents": [{"name": "a", "type": "random"}] * 4},
    {"seat_policy": "alphabetical"},
    {"max_turns": 0},
])
def test_run_config_validation(bad):
    base = dict(FX["config"])
    base.update(bad)
    with pytest.raises(ValueError):
        RunConfig.from_dict(base)


def test_legacy_config_shape():
    cfg = RunConfig.from_dict({"a": {"type": "random"}, "b": {"type": "random", "time_limit": 0.2},
                               "c": {"type": "random"}, "d": {"type": "random"}, "num_games": 3, "seed": 1})
    assert cfg.agent_names == ["a", "b", "c", "d"] and cfg.agents[1].thinking_time_ms == 200


@pytest.mark.parametrize("kind", ["fast_mcts", "gameplay_fast_mcts"])
def test_wall_clock_fastmcts_seat_plays_in_host_loop(kind, tmp_path, monkeypatch):
    """A FastMCTS seat with deterministic_time_budget false has a wall-clock iteration
    count (arena_runner.py:352-369): run_experiment must send its games to the host loop
    (run_single_game), never to run_games_batched, which needs fixed iteration counts."""
    from reinforcementlearning_blokus_amd.arena import runner
    calls = {"batched": 0, "single": 0}

    def fake_batched(*a, **k):
        calls["batched"] += 1
        raise AssertionError("batched path taken")

    def fake_single(*, game_index, game_seed, seat_assignment, **k):
        calls["single"] += 1
        return {"game_index": game_index, "game_seed": game_seed, "seat_assignment": seat_assignment,
                "final_scores": {}, "winner_ids": [], "winner_agents": [], "is_tie": False,
                "moves_made": 0, "error": None, "agent_move_stats": {}}

    monkeypatch.setattr(runner, "run_games_batched", fake_batched)
    monkeypatch.setattr(runner, "run_single_game", fake_single)
    monkeypatch.setattr(runner, "compute_summary", lambda records, **k: {"completed_games": len(records)})
    cfg = RunConfig.from_dict({"agents": [
        {"name": "r", "type": "random"}, {"name": "h", "type": "heuristic"},
        {"name": "m", "type": "mcts", "params": {"iterations": 8}},
        {"name": "f", "type": kind, "thinking_time_ms": 20, "params": {"deterministic_time_budget": False}}],
        "num_games": 3, "seed": 5, "seat_policy": "round_robin", "output_root": str(tmp_path)})
    seats = seat_assignment_for_game(cfg.agent_names, 0, game_seed_from_run_seed(5, 0), "round_robin")
    assert not runner._batchable(cfg, seats)
    runner.run_experiment(cfg)
    assert calls == {"batched": 0, "single": 3}
    cfg2 = RunConfig.from_dict(dict(cfg.to_dict(), agents=[
        {"name": "r", "type": "random"}, {"name": "h", "type": "heuristic"},
        {"name": "m", "type": "mcts", "params": {"iterations": 8}},
        {"name": "f", "type": kind, "thinking_time_ms": 20}]))
    seats2 = seat_assignment_for_game(cfg2.agent_names, 0, game_seed_from_run_seed(5, 0), "round_robin")
    assert runner._batchable(cfg2, seats2)


def test_mt_state_views_match_get_state():
    """search_packed moves rollout streams through direct views of numpy's MT19937 state
    (mcts_agent._mt_view): a view reads what get_state returns and a write through it is
    what set_state would leave, Gaussian cache included."""
    import numpy as np

    from reinforcementlearning_blokus_amd.mcts.mcts_agent import _mt_view
    r = np.random.RandomState(99)
    r.standard_normal()  # has_gauss set
    r.random_sample(1000)
    v = _mt_view(r)
    assert v is not None
    st = r.get_state()
    assert np.array_equal(v[:624], st[1]) and int(v[624]) == st[2]
    ref = np.random.RandomState(0)
    ref.set_state(st)
    nxt = np.random.RandomState(5).get_state()
    v[:624] = nxt[1]
    v[624] = nxt[2]
    ref.set_state((st[0], nxt[1], nxt[2], st[3], st[4]))
    assert r.get_state()[1].tolist() == ref.get_state()[1].tolist()
    assert r.get_state()[2:] == ref.get_state()[2:]
    assert r.randint(0, 1000, size=50).tolist() == ref.randint(0, 1000, size=50).tolist()
    assert r.standard_normal() == ref.standard_normal()


def test_arena_options_are_arguments_not_environment(monkeypatch):
    """run_games_batched's pipeline settings are explicit ArenaOptions fields (VERDICT r05
    item 8): the runner reads one environment variable, the BK_ARENA_CAPTURE diagnostics
    switch, and rejects stream counts above the validated 16."""
    import re
    from pathlib import Path

    from reinforcementlearning_blokus_amd.arena import runner
    src = Path(runner.__file__).read_text()
    assert re.findall(r"os\.environ[^\n]*", src) == ['os.environ.get("BK_ARENA_CAPTURE") or None)']
    assert runner.ArenaOptions().search_streams == 8
    for bad in (0, 17, 32):
        with pytest.raises(ValueError):
            runner.ArenaOptions(search_streams=bad)
    with pytest.raises(ValueError):
        runner.ArenaOptions(job_games=0)
    monkeypatch.setenv("BK_ARENA_MCTS_STREAMS", "24")  # ignored: no longer read
    assert runner.ArenaOptions().search_streams == 8
