"""Arena driver (reference: analytics/tournament/arena_runner.py, arena_stats.py).

Same run configuration, seeding, seat policies, per-game records (``games.jsonl``) and
``summary.json`` as the reference.  Two execution paths:

* all four seats ``random``: every game of the run (or of this rank's shard) is played
  inside one ``bk_rollout_frontier`` launch, in the reference's frontier move order with
  each seat's numpy RandomState stream -- the reference's games, move for move;
* any other mix: the reference's per-game loop over ``BlokusGame`` and the agents,
  with GPU move generation.
"""
from .config import AgentConfig, RunConfig, game_seed_from_run_seed, load_run_config, stable_hash_int
from .runner import build_agent, run_experiment, run_games_gpu, run_single_game
from .stats import compute_summary

__all__ = ["AgentConfig", "RunConfig", "load_run_config", "stable_hash_int", "game_seed_from_run_seed",
           "build_agent", "run_single_game", "run_games_gpu", "run_experiment", "compute_summary"]
