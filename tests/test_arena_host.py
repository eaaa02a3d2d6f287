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
