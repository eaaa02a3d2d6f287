"""A mixed-agent arena game on the ORACLE (test infrastructure): the config-4 checker.

Plays `run_single_game` (analytics/tournament/arena_runner.py:578-777; loop :652-697:
pass when stuck, game over when no player can move, max_turns) for one game index of a
RunConfig with every seat restated on oracle/ primitives, never the GPU:

* random     RandomAgent(seed): numpy RandomState(seed).randint over the frontier-order
             list (agents/random_agent.py:29-50);
* heuristic  HeuristicAgent(seed): pyoracle.heuristic_choice, the numpy restatement
             pinned by tests/golden/heuristic.json (agents/heuristic_agent.py:39-244);
* mcts       MCTSAgent(iterations, seed): or_mcts with HeuristicAgent rollouts drawing
             from the rollout agent's RandomState(seed), ZobristHash(seed) and one TT kept
             across the seat's moves (mcts/mcts_agent.py:202-341, :470-554; zobrist.py);
             a single legal move is answered without a search (:313-318), and the arena
             then reads the previous search's iterations_run again (stale stats);
* fast_mcts  FastMCTSAgent(seed) with deterministic_time_budget: or_fastmcts_mt with
             iterations = round(iterations_per_ms * thinking_time_ms) on the agent's one
             random.Random(seed) stream (agents/fast_mcts_agent.py:89-226, arena :333-371).

Seat assignment and agent seeds are the arena's (arena_runner.py:241-292), taken from
the package's arena.config (pinned by the arena fixtures).  The checker itself is pinned
by tests/golden/arena_bench.json (tests/test_oracle_arena.py).
"""
from __future__ import annotations

import numpy as np

from oracle import pyoracle as O


def _game_over(b) -> bool:
    return all(O.lib().or_has_moves(b, p) == 0 for p in range(4))


def oracle_arena_game(cfg, game_index: int) -> dict:
    from reinforcementlearning_blokus_amd.arena.config import (agent_seed, game_seed_from_run_seed,
                                                               seat_assignment_for_game)
    gs = game_seed_from_run_seed(cfg.seed, game_index)
    seats = seat_assignment_for_game(cfg.agent_names, game_index, gs, cfg.seat_policy)
    conf = {a.name: a for a in cfg.agents}
    state = {}
    for name in set(seats.values()):
        s = agent_seed(cfg.seed, game_index, name)
        a = conf[name]
        kind = a.type.lower()
        if kind in ("random", "heuristic"):
            state[name] = {"rng": np.random.RandomState(s)}
        elif kind == "mcts":
            state[name] = {"z": O.zobrist_table(s), "rng": O.numpy_mt(s), "tt": O.TT(), "last": 0,
                           "iters": int(a.params.get("iterations", 1000)),
                           "roll": int(a.params.get("max_rollout_moves", 50)),
                           "c": float(a.params.get("exploration_constant", 1.414))}
        elif kind == "fast_mcts":
            assert a.params.get("deterministic_time_budget", True)
            state[name] = {"mt": O.python_mt(s),
                           "iters": max(1, int(round(float(a.params.get("iterations_per_ms", 20.0)) *
                                                     int(a.thinking_time_ms))))}
        else:
            raise ValueError(kind)
    b = O.new_board()
    turns = passes = 0
    sims = {n: 0 for n in state}
    while not _game_over(b) and turns < cfg.max_turns:
        p = b.cur
        name = seats[str(p + 1)]
        kind = conf[name].type.lower()
        st = state[name]
        legal = O.legal_moves(b, p, O.ORDER_FRONTIER)
        turns += 1
        if not legal:
            passes += 1
            b.cur = (p + 1) & 3
            continue
        if kind == "random":
            mv = legal[st["rng"].randint(0, len(legal))]
        elif kind == "heuristic":
            mv = O.heuristic_choice(b, p, st["rng"])
        elif kind == "mcts":
            if len(legal) == 1:
                mv = legal[0]
            else:
                r = O.mcts(b, p, st["iters"], st["c"], st["roll"], st["z"], st["rng"], st["tt"], heuristic=True)
                mv = r["move"]
                st["last"] = st["iters"]
            sims[name] += st["last"]
        else:
            mv = O.fastmcts_mt(b, p, st["mt"], st["iters"])
        O.place_move(b, p, mv)
        b.cur = (p + 1) & 3
    scores, wm = O.game_scores(b)
    return {"game_index": game_index, "seat_assignment": seats,
            "final_scores": {str(p + 1): int(scores[p]) for p in range(4)},
            "winner_ids": [p + 1 for p in range(4) if wm >> p & 1],
            "moves_made": int(b.move_count), "turn_count": turns, "passes": passes,
            "simulations": sims}
