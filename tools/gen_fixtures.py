#!/usr/bin/env python3
"""Generate golden fixtures from the reference implementation (container-only tool).

This script imports the read-only reference checkout (default ``/root/reference``)
and records input/output vectors for the hot path into ``tests/golden/``.  It is
never shipped to, or needed on, the GPU box: only its JSON outputs are committed.

Run from /tmp with ``PYTHONDONTWRITEBYTECODE=1`` so nothing is written into the
reference tree::

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tools/gen_fixtures.py

What is recorded (all reference behaviour, nothing re-implemented here):

* ``pieces.json``      -- ALL_PIECE_ORIENTATIONS (engine/pieces.py:257)
* ``positions.json``   -- generate_random_valid_state (tests/utils_game_states.py:12)
                          states, the place_piece call log that built them, the
                          live frontier-set iteration order, and per-player legal
                          move lists in both frontier (default) and naive order
                          (engine/move_generator.py:153, :261)
* ``rng.json``         -- numpy RandomState randint / uint64 streams and stdlib
                          random.Random streams (agents/random_agent.py:49,
                          agents/fast_mcts_agent.py:99, mcts/zobrist.py:41)
* ``playouts_<order>.json`` -- terminal random playouts (arena semantics,
                          analytics/tournament/arena_runner.py:652-697) from the
                          recorded positions, one RandomAgent per seat
* ``rollouts_a_<order>.json`` -- MCTSAgent._rollout rewards (mcts/mcts_agent.py:470)
* ``fastmcts.json``    -- FastMCTSAgent.think results (agents/fast_mcts_agent.py:112)
* ``zobrist.json``     -- ZobristHash.hash_board values (mcts/zobrist.py:70)
* ``arena_small.json`` -- run_single_game records for 4 random agents
* ``arena_cap.json`` -- run_single_game records cut by (or ending exactly at) max_turns
* ``mcts.json``        -- MCTSAgent (UCT + Zobrist transposition table) searches with
                          RandomAgent rollouts (mcts/mcts_agent.py:304-582): two
                          consecutive select_action calls per agent, the root children
                          (move, visits, total_reward), stats and rollout-RNG state
* ``heuristic.json``   -- HeuristicAgent (agents/heuristic_agent.py): per-move
                          _evaluate_move scores (float hex) and softmax probabilities for
                          legal lists, select_action sequences in 12-ply heuristic
                          self-play, full 4-heuristic games, MCTSAgent searches with its
                          default HeuristicAgent rollouts, and run_single_game records of
                          mixed random/heuristic/mcts/fast_mcts arenas
* ``arena_bench.json`` -- run_single_game records of bench.py's config-4 seats (MCTS 64
                          iterations with 50-ply heuristic rollouts, FastMCTS 1,000
                          iterations), games 0..3 of run seed 20260301 (``arena_bench``
                          only, not part of ``all``)
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
from multiprocessing import Pool

REF = os.environ.get("BLOKUS_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")

# Positions: (num_moves, seed).  Small and mid-game plus late game.
POSITION_SPECS = (
    [(0, 0), (1, 0), (2, 0), (3, 0), (4, 1), (5, 2), (8, 3), (8, 4)]
    + [(12, s) for s in range(5, 9)]
    + [(16, s) for s in range(9, 13)]
    + [(20, s) for s in range(13, 29)]
    + [(24, s) for s in range(29, 33)]
    + [(28, s) for s in range(33, 37)]
    + [(32, s) for s in range(37, 41)]
    + [(40, s) for s in range(41, 45)]
    + [(48, s) for s in range(45, 48)]
    + [(56, s) for s in range(48, 51)]
    + [(64, s) for s in range(51, 53)]
)
FULL_LIST_POSITIONS = 24  # positions whose full move lists are stored
PLAYOUT_POSITIONS = 48    # positions (ply>=8) used as playout roots


def _setup():
    sys.path.insert(0, REF)


def move_int(gid_of, m):
    return gid_of[(m.piece_id, m.orientation)] * 400 + m.anchor_row * 20 + m.anchor_col


def _gid_map():
    from engine.pieces import ALL_PIECE_ORIENTATIONS
    gid_of = {}
    g = 0
    for pid in sorted(ALL_PIECE_ORIENTATIONS):
        for o in range(len(ALL_PIECE_ORIENTATIONS[pid])):
            gid_of[(pid, o)] = g
            g += 1
    return gid_of


def _state_dict(board):
    from engine.board import Player
    return {
        "player_bits": [hex(board.player_bits[p]) for p in Player],
        "used": [sorted(board.player_pieces_used[p]) for p in Player],
        "first": [bool(board.player_first_move[p]) for p in Player],
        "current_player": board.current_player.value,
        "move_count": board.move_count,
        "frontier": [[list(x) for x in board.get_frontier(p)] for p in Player],
    }


def _sha(ints):
    return hashlib.sha256(",".join(str(i) for i in ints).encode()).hexdigest()


def gen_position(spec):
    _setup()
    import engine.board as eb
    from engine.board import Player
    from engine.move_generator import LegalMoveGenerator
    from tests.utils_game_states import generate_random_valid_state

    m, seed = spec
    log = []
    orig = eb.Board.place_piece

    def logged(self, positions, player, piece_id, validate=True):
        ok = orig(self, positions, player, piece_id, validate)
        if ok:
            log.append([player.value, piece_id, [[p.row, p.col] for p in positions]])
        return ok

    eb.Board.place_piece = logged
    try:
        board, cur = generate_random_valid_state(m, seed)
    finally:
        eb.Board.place_piece = orig
    gid_of = _gid_map()
    gen = LegalMoveGenerator()
    rec = {"num_moves": m, "seed": seed, "log": log, "state": _state_dict(board), "players": []}
    for p in Player:
        fr = [move_int(gid_of, x) for x in gen._get_legal_moves_frontier(board, p)]
        nv = [move_int(gid_of, x) for x in gen._get_legal_moves_naive(board, p)]
        rec["players"].append({
            "count": len(fr), "sha_frontier": _sha(fr), "sha_naive": _sha(nv),
            "has_moves": bool(gen.has_legal_moves(board, p)),
            "frontier_list": fr, "naive_list": nv,
        })
    return rec


def gen_pieces():
    _setup()
    from engine.pieces import ALL_PIECE_ORIENTATIONS
    out = []
    for pid in sorted(ALL_PIECE_ORIENTATIONS):
        for o in ALL_PIECE_ORIENTATIONS[pid]:
            out.append({
                "piece_id": pid, "orientation": o.orientation_id,
                "offsets": [list(x) for x in o.offsets],
                "orth_offsets": [list(x) for x in o.orth_offsets],
                "diag_offsets": [list(x) for x in o.diag_offsets],
                "shape_mask": hex(o.shape_mask), "orth_mask": hex(o.orth_mask),
                "diag_mask": hex(o.diag_mask), "anchor_indices": list(o.anchor_indices),
            })
    return out


def gen_rng():
    _setup()
    import random
    import numpy as np
    out = {"randint": [], "uint64": [], "py_random": [], "py_choice": []}
    for seed in (0, 1, 7, 12345, 2**31 - 2, 4000000000):
        rs = np.random.RandomState(seed)
        ns = [1, 2, 3, 5, 7, 58, 100, 491, 839, 1000, 1, 4096, 65537, 3]
        draws = [int(rs.randint(0, n)) for n in ns * 8]
        out["randint"].append({"seed": seed, "n": ns * 8, "draws": draws})
        rs = np.random.RandomState(seed)
        out["uint64"].append({"seed": seed, "draws": [str(int(rs.randint(0, 2**64, dtype=np.uint64))) for _ in range(8)]})
    for seed in (0, 1, 42, 2**40 + 3, 123456789012):
        r = random.Random(seed)
        out["py_random"].append({"seed": seed, "draws": [r.random().hex() for _ in range(16)]})
        random.seed(seed)
        seq = list(range(1000))
        out["py_choice"].append({"seed": seed, "n": [1, 2, 3, 58, 491, 839, 1000, 7] * 4,
                                 "draws": [random.choice(seq[:n]) for n in [1, 2, 3, 58, 491, 839, 1000, 7] * 4]})
    return out


def _playout_b(board, seeds, max_turns=2500):
    """Arena semantics (arena_runner.run_single_game loop) from a given board."""
    from agents.random_agent import RandomAgent
    from engine.board import Player
    from engine.game import BlokusGame
    game = BlokusGame(enable_telemetry=False)
    game.board = board
    gid_of = _gid_map()
    agents = {p: RandomAgent(seed=s) for p, s in zip(Player, seeds)}
    passes = turn_count = 0
    trace = []
    game._check_game_over()
    while not game.is_game_over() and turn_count < max_turns:
        cur = game.get_current_player()
        legal = game.get_legal_moves(cur)
        turn_count += 1
        if not legal:
            passes += 1
            trace.append(-1)
            game.board._update_current_player()
            game._check_game_over()
            continue
        mv = agents[cur].select_action(game.board, cur, legal)
        trace.append(move_int(gid_of, mv))
        assert game.make_move(mv, cur)
    res = game.get_game_result()
    return {"scores": [int(res.scores[p.value]) for p in Player], "winner_ids": list(res.winner_ids),
            "moves_made": game.board.move_count, "passes": passes, "turn_count": turn_count, "trace": trace}


def gen_playouts(args):
    idx, spec, seeds = args
    _setup()
    from tests.utils_game_states import generate_random_valid_state
    board, _ = generate_random_valid_state(*spec)
    rec = _playout_b(board, seeds)
    rec.update({"position": idx, "agent_seeds": seeds})
    return rec


def gen_rollout_a(args):
    idx, spec, seed = args
    _setup()
    from agents.random_agent import RandomAgent
    from mcts.mcts_agent import MCTSAgent
    from tests.utils_game_states import generate_random_valid_state
    board, cur = generate_random_valid_state(*spec)
    agent = MCTSAgent(iterations=1, rollout_agent=RandomAgent(seed=seed), seed=seed)
    start = [int(board.get_score(p)) for p in __import__("engine.board", fromlist=["Player"]).Player]
    reward = agent._rollout(board, cur)
    return {"position": idx, "seed": seed, "player": cur.value, "reward": float(reward), "start_scores": start}


def gen_fastmcts(args):
    idx, spec, seed, iters = args
    _setup()
    from agents.fast_mcts_agent import FastMCTSAgent
    from engine.move_generator import get_shared_generator
    from tests.utils_game_states import generate_random_valid_state
    board, cur = generate_random_valid_state(*spec)
    legal = get_shared_generator().get_legal_moves(board, cur)
    gid_of = _gid_map()
    agent = FastMCTSAgent(iterations=iters, time_limit=1000.0, seed=seed)
    res = agent.think(board, cur, legal, 10**9)
    mv = res["move"]
    return {"position": idx, "seed": seed, "iterations": iters, "n_legal": len(legal),
            "move": move_int(gid_of, mv) if mv is not None else None,
            "nodes": res["stats"]["nodesEvaluated"],
            "top": [[gid_of[(t["piece_id"], t["orientation"])] * 400 + t["anchor_row"] * 20 + t["anchor_col"],
                     t["visits"], t["q_value"]] for t in res["stats"]["topMoves"]]}


def gen_zobrist():
    _setup()
    from mcts.zobrist import ZobristHash
    from tests.utils_game_states import generate_random_valid_state
    out = []
    for zseed in (0, 5, 20260301):
        z = ZobristHash(seed=zseed)
        hashes = []
        for spec in POSITION_SPECS[:12]:
            board, _ = generate_random_valid_state(*spec)
            hashes.append(str(int(z.hash_board(board))))
        out.append({"seed": zseed, "hashes": hashes,
                    "table_head": [str(int(x)) for x in z.position_player_hashes.reshape(-1)[:10]],
                    "turn": [str(int(x)) for x in z.player_turn_hashes],
                    "piece_head": [str(int(x)) for x in z.piece_used_hashes.reshape(-1)[:5]]})
    return out


def gen_arena():
    _setup()
    from analytics.tournament.arena_runner import (AgentConfig, RunConfig, _seat_assignment_for_game,
                                                   game_seed_from_run_seed, run_single_game)
    cfg = RunConfig.from_dict({
        "agents": [{"name": f"r{i}", "type": "random"} for i in range(4)],
        "num_games": 2, "seed": 20260301, "seat_policy": "round_robin", "output_root": "/tmp/arena_fx",
    })
    agents = {a.name: a for a in cfg.agents}
    out = []
    for gi in range(2):
        gs = game_seed_from_run_seed(cfg.seed, gi)
        seats = _seat_assignment_for_game([a.name for a in cfg.agents], gi, gs, cfg.seat_policy)
        rec, _ = run_single_game(run_id="fx", game_index=gi, game_seed=gs, run_config=cfg,
                                 seat_assignment=seats, agent_configs=agents)
        out.append({k: rec[k] for k in ("game_index", "game_seed", "seat_assignment", "winner_ids",
                                        "final_scores", "moves_made", "turn_count", "passes", "is_tie")})
    return out


ARENA_RUN = {"agents": [{"name": f"r{i}", "type": "random"} for i in range(4)], "num_games": 16,
             "seed": 424242, "seat_policy": "randomized", "output_root": "/tmp/arena_fx2"}


def gen_arena_game(gi):
    _setup()
    from analytics.tournament.arena_runner import (RunConfig, _seat_assignment_for_game, game_seed_from_run_seed,
                                                   run_single_game)
    cfg = RunConfig.from_dict(ARENA_RUN)
    gs = game_seed_from_run_seed(cfg.seed, gi)
    seats = _seat_assignment_for_game([a.name for a in cfg.agents], gi, gs, cfg.seat_policy)
    rec, _ = run_single_game(run_id="fx2", game_index=gi, game_seed=gs, run_config=cfg, seat_assignment=seats,
                             agent_configs={a.name: a for a in cfg.agents})
    return rec


def gen_arena_runs():
    """16 run_single_game records (randomized seats) + the reference's compute_summary
    over deterministic copies of them (timings replaced by fixed values)."""
    _setup()
    from analytics.tournament.arena_stats import compute_summary
    with Pool(8) as pool:
        recs = pool.map(gen_arena_game, range(ARENA_RUN["num_games"]))
    keep = ("game_index", "game_seed", "seat_assignment", "winner_ids", "winner_agents", "winner_id", "is_tie",
            "final_scores", "final_ranks", "agent_scores", "agent_ranks", "moves_made", "turn_count", "passes",
            "invalid_actions", "truncated")
    games = [{k: r[k] for k in keep} for r in recs]
    synth = []
    for r in recs:
        d = dict(r)
        d["duration_sec"] = 0.5 + 0.01 * r["game_index"]
        d["agent_move_stats"] = {n: {"moves": st["moves"], "total_time_ms": 1.5 * st["moves"],
                                     "total_simulations": None, "moves_with_simulations": 0.0,
                                     "move_times_ms": [1.5] * int(st["moves"])}
                                 for n, st in r["agent_move_stats"].items()}
        d["error"] = None
        synth.append(d)
    summary = compute_summary(synth, run_id="fx2", run_seed=ARENA_RUN["seed"], seat_policy="randomized",
                              agent_names=[a["name"] for a in ARENA_RUN["agents"]],
                              thinking_time_ms_by_agent={a["name"]: None for a in ARENA_RUN["agents"]},
                              run_config=ARENA_RUN)
    return {"config": ARENA_RUN, "games": games, "summary_input": synth, "summary": summary}


def _arena_cap_game(job):
    """run_single_game of ARENA_RUN game gi with max_turns = cap (None: default)."""
    gi, cap = job
    _setup()
    from analytics.tournament.arena_runner import (RunConfig, _seat_assignment_for_game, game_seed_from_run_seed,
                                                   run_single_game)
    d = dict(ARENA_RUN)
    if cap is not None:
        d["max_turns"] = cap
    cfg = RunConfig.from_dict(d)
    gs = game_seed_from_run_seed(cfg.seed, gi)
    seats = _seat_assignment_for_game([a.name for a in cfg.agents], gi, gs, cfg.seat_policy)
    rec, _ = run_single_game(run_id="fx4", game_index=gi, game_seed=gs, run_config=cfg, seat_assignment=seats,
                             agent_configs={a.name: a for a in cfg.agents})
    keep = ("game_index", "game_seed", "seat_assignment", "winner_ids", "final_scores", "moves_made", "turn_count",
            "passes", "is_tie", "truncated")
    out = {k: rec[k] for k in keep}
    out["max_turns"] = cfg.max_turns
    return out


def gen_arena_cap():
    """Games cut by max_turns (arena_runner.py:653, :702): for ARENA_RUN games 0..3 the
    full game's turn count T, then the same game with max_turns = T (it ends by its own
    last move exactly at the cap: NOT truncated) and max_turns = T - 5 (truncated)."""
    with Pool(8) as pool:
        full = pool.map(_arena_cap_game, [(gi, None) for gi in range(4)])
        jobs = [(r["game_index"], r["turn_count"]) for r in full] + \
               [(r["game_index"], r["turn_count"] - 5) for r in full]
        return pool.map(_arena_cap_game, jobs)


# (position index, iterations, max_rollout_moves, use_tt, rollout seed, zobrist seed)
MCTS_CASES = [
    (8, 24, 50, True, 11, 3), (12, 40, 50, True, 12, 4), (16, 24, 50, False, 13, 5),
    (20, 60, 8, True, 14, 6), (24, 120, 4, True, 15, 7), (30, 200, 2, True, 16, 8),
    (36, 48, 50, True, 17, 9), (47, 150, 3, True, 18, 10), (50, 60, 50, True, 19, 11),
    (49, 100, 50, True, 20, 12), (53, 300, 1, True, 21, 13), (40, 64, 6, False, 22, 14),
    (46, 80, 50, True, 23, 15), (18, 450, 2, True, 24, 16), (19, 400, 3, True, 25, 17),
]


def gen_mcts_case(case):
    """MCTSAgent.select_action (mcts/mcts_agent.py:304-341) restated around the
    agent's own methods so the root node can be recorded: root = MCTSNode(board,
    player); _run_mcts_with_iterations(root); best = root.get_best_move(); the TT
    clear rule of :338-339.  Call 1 searches the position, call 2 the position
    after call 1's move (same agent: TT and rollout stream carry over)."""
    pos, iters, max_roll, use_tt, rseed, zseed = case
    _setup()
    from agents.random_agent import RandomAgent
    from engine.board import Player
    from engine.move_generator import get_shared_generator
    from mcts.mcts_agent import MCTSAgent, MCTSNode
    from tests.utils_game_states import generate_random_valid_state
    gid_of = _gid_map()
    board, cur = generate_random_valid_state(*POSITION_SPECS[pos])
    agent = MCTSAgent(iterations=iters, rollout_agent=RandomAgent(seed=rseed), seed=zseed,
                      use_transposition_table=use_tt, max_rollout_moves=max_roll)
    gen = get_shared_generator()
    calls = []
    for call in range(2):
        legal = gen.get_legal_moves(board, cur)
        rec = {"player": cur.value, "n_legal": len(legal)}
        if len(legal) <= 1:
            rec["move"] = move_int(gid_of, legal[0]) if legal else None
            rec["searched"] = False
        else:
            root = MCTSNode(board, cur)
            agent._run_mcts_with_iterations(root)
            best = root.get_best_move()
            if agent.transposition_table and len(agent.transposition_table.table) > 500000:
                agent.transposition_table.clear()
            rec.update({
                "searched": True,
                "move": move_int(gid_of, best),
                "root_children": [[move_int(gid_of, ch.move), ch.visits, float(ch.total_reward)]
                                  for ch in root.children],
                "root_visits": root.visits,
                "root_untried": len(root.untried_moves),
                "iterations_run": agent.stats["iterations_run"],
                "transposition_hits": agent.stats["transposition_hits"],
                "rollout_rewards": [float(r) for r in agent.stats["rollout_rewards"]],
                "tt_size": len(agent.transposition_table.table) if agent.transposition_table else None,
            })
            best = rec["move"]
        st = agent.rollout_agent.rng.get_state()
        rec["rng_pos"] = int(st[2])
        rec["rng_sha"] = _sha(int(x) for x in st[1])
        calls.append(rec)
        if rec["move"] is None:
            break
        mv = next(m for m in legal if move_int(gid_of, m) == rec["move"])
        board.place_piece(agent._get_move_positions(mv), cur, mv.piece_id, validate=False)
        cur = list(Player)[(list(Player).index(cur) + 1) % 4]
    return {"position": pos, "iterations": iters, "max_rollout_moves": max_roll, "use_tt": use_tt,
            "rollout_seed": rseed, "zobrist_seed": zseed, "calls": calls}


# (position index, seed): heuristic evaluation + 12-ply heuristic self-play
HEUR_CASES = [(i, 300 + i) for i in (0, 1, 4, 6, 8, 10, 14, 18, 22, 26, 30, 34, 38, 42, 46, 50)]
HEUR_FULL_LISTS = 6  # cases whose legal lists / score vectors are stored in full


def _heur_case(case):
    pos, seed = case
    _setup()
    from agents.heuristic_agent import HeuristicAgent
    from engine.board import Player
    from engine.game import BlokusGame
    from engine.move_generator import get_shared_generator
    from tests.utils_game_states import generate_random_valid_state
    gid_of = _gid_map()
    board, cur = generate_random_valid_state(*POSITION_SPECS[pos])
    gen = get_shared_generator()
    agent = HeuristicAgent(seed=seed)
    legal = gen.get_legal_moves(board, cur)
    scores = [agent._evaluate_move(board, cur, m) for m in legal]
    probs = agent._softmax(__import__("numpy").array(scores), temperature=1.0) if legal else []
    rec = {"position": pos, "seed": seed, "player": cur.value, "move_count": board.move_count,
           "n_legal": len(legal), "moves_sha": _sha(move_int(gid_of, m) for m in legal),
           "scores_sha": _sha(float(x).hex() for x in scores), "probs_sha": _sha(float(x).hex() for x in probs)}
    if HEUR_CASES.index(case) < HEUR_FULL_LISTS:
        rec["moves"] = [move_int(gid_of, m) for m in legal]
        rec["scores"] = [float(x).hex() for x in scores]
    # 12 plies of heuristic self-play (arena semantics: pass when stuck), agent per seat
    game = BlokusGame(enable_telemetry=False)
    game.board = board
    agents = {p: HeuristicAgent(seed=seed * 10 + p.value) for p in Player}
    trace = []
    for _ in range(12):
        game._check_game_over()
        if game.is_game_over():
            break
        p = game.get_current_player()
        lm = game.get_legal_moves(p)
        if not lm:
            trace.append(-1)
            game.board._update_current_player()
            continue
        mv = agents[p].select_action(game.board, p, lm)
        trace.append(move_int(gid_of, mv))
        assert game.make_move(mv, p)
    rec["selfplay_trace"] = trace
    rec["selfplay_rng"] = {p.value: [int(agents[p].rng.get_state()[2]),
                                     _sha(int(x) for x in agents[p].rng.get_state()[1])] for p in Player}
    return rec


def _heur_game(gseed):
    """A full 4-HeuristicAgent game from the empty board (arena loop semantics)."""
    _setup()
    from agents.heuristic_agent import HeuristicAgent
    from engine.board import Player
    from engine.game import BlokusGame
    gid_of = _gid_map()
    game = BlokusGame(enable_telemetry=False)
    agents = {p: HeuristicAgent(seed=gseed + p.value) for p in Player}
    trace, passes, turns = [], 0, 0
    while not game.is_game_over() and turns < 2500:
        p = game.get_current_player()
        lm = game.get_legal_moves(p)
        turns += 1
        if not lm:
            passes += 1
            trace.append(-1)
            game.board._update_current_player()
            game._check_game_over()
            continue
        mv = agents[p].select_action(game.board, p, lm)
        trace.append(move_int(gid_of, mv))
        assert game.make_move(mv, p)
    res = game.get_game_result()
    return {"seed": gseed, "trace": trace, "scores": [int(res.scores[p.value]) for p in Player],
            "winner_ids": list(res.winner_ids), "passes": passes, "turns": turns}


# MCTSAgent with its default rollout policy, HeuristicAgent(seed) (mcts/mcts_agent.py:278-281)
HEUR_MCTS_CASES = [(12, 6, 3, True, 31), (20, 8, 4, True, 32), (30, 5, 6, False, 33), (44, 8, 2, True, 34)]


def _heur_mcts_case(case):
    pos, iters, max_roll, use_tt, seed = case
    _setup()
    from engine.move_generator import get_shared_generator
    from mcts.mcts_agent import MCTSAgent, MCTSNode
    from tests.utils_game_states import generate_random_valid_state
    gid_of = _gid_map()
    board, cur = generate_random_valid_state(*POSITION_SPECS[pos])
    agent = MCTSAgent(iterations=iters, seed=seed, use_transposition_table=use_tt, max_rollout_moves=max_roll)
    legal = get_shared_generator().get_legal_moves(board, cur)
    root = MCTSNode(board, cur)
    agent._run_mcts_with_iterations(root)
    best = root.get_best_move()
    st = agent.rollout_agent.rng.get_state()
    return {"position": pos, "iterations": iters, "max_rollout_moves": max_roll, "use_tt": use_tt, "seed": seed,
            "player": cur.value, "n_legal": len(legal), "move": move_int(gid_of, best),
            "root_children": [[move_int(gid_of, ch.move), ch.visits, float(ch.total_reward)] for ch in root.children],
            "rollout_rewards": [float(r) for r in agent.stats["rollout_rewards"]],
            "transposition_hits": agent.stats["transposition_hits"],
            "rng_pos": int(st[2]), "rng_sha": _sha(int(x) for x in st[1])}


HEUR_ARENA = {"agents": [{"name": "r", "type": "random"}, {"name": "h", "type": "heuristic"},
                         {"name": "m", "type": "mcts", "params": {"iterations": 3, "max_rollout_moves": 2}},
                         {"name": "f", "type": "fast_mcts", "params": {"time_limit": 0.01}}],
              "num_games": 4, "seed": 777001, "seat_policy": "round_robin", "output_root": "/tmp/arena_fx3"}


def _heur_arena_game(gi):
    _setup()
    from analytics.tournament.arena_runner import (RunConfig, _seat_assignment_for_game, game_seed_from_run_seed,
                                                   run_single_game)
    cfg = RunConfig.from_dict(HEUR_ARENA)
    gs = game_seed_from_run_seed(cfg.seed, gi)
    seats = _seat_assignment_for_game([a.name for a in cfg.agents], gi, gs, cfg.seat_policy)
    rec, _ = run_single_game(run_id="fx3", game_index=gi, game_seed=gs, run_config=cfg, seat_assignment=seats,
                             agent_configs={a.name: a for a in cfg.agents})
    keep = ("game_index", "game_seed", "seat_assignment", "winner_ids", "final_scores", "moves_made",
            "turn_count", "passes", "invalid_actions", "is_tie", "error")
    return {k: rec[k] for k in keep}


# bench.py's config-4 seats (CONFIG4_AGENTS, run seed 20260301): MCTS 64 iterations with
# 50-ply HeuristicAgent rollouts, FastMCTS 20 iterations/ms x 50 ms deterministic budget
ARENA_BENCH = {"agents": [{"name": "random", "type": "random"}, {"name": "heuristic", "type": "heuristic"},
                          {"name": "mcts", "type": "mcts", "params": {"iterations": 64, "max_rollout_moves": 50}},
                          {"name": "fast_mcts", "type": "fast_mcts", "thinking_time_ms": 50,
                           "params": {"deterministic_time_budget": True, "iterations_per_ms": 20.0}}],
               "num_games": 4, "seed": 20260301, "seat_policy": "round_robin", "output_root": "/tmp/arena_fx4"}


def _bench_arena_game(gi):
    _setup()
    from analytics.tournament.arena_runner import (RunConfig, _seat_assignment_for_game, game_seed_from_run_seed,
                                                   run_single_game)
    cfg = RunConfig.from_dict(ARENA_BENCH)
    gs = game_seed_from_run_seed(cfg.seed, gi)
    seats = _seat_assignment_for_game([a.name for a in cfg.agents], gi, gs, cfg.seat_policy)
    rec, _ = run_single_game(run_id="fx4", game_index=gi, game_seed=gs, run_config=cfg, seat_assignment=seats,
                             agent_configs={a.name: a for a in cfg.agents})
    keep = ("game_index", "game_seed", "seat_assignment", "winner_ids", "final_scores", "moves_made",
            "turn_count", "passes", "invalid_actions", "is_tie", "error")
    out = {k: rec[k] for k in keep}
    out["mcts_total_simulations"] = rec["agent_move_stats"]["mcts"]["total_simulations"]
    return out


def gen_heuristic():
    with Pool(8) as pool:
        cases = pool.map(_heur_case, HEUR_CASES)
        games = pool.map(_heur_game, [9001, 9002])
        searches = pool.map(_heur_mcts_case, HEUR_MCTS_CASES)
        arena = pool.map(_heur_arena_game, range(HEUR_ARENA["num_games"]))
    return {"cases": cases, "games": games, "mcts": searches, "arena_config": HEUR_ARENA, "arena": arena}


def dump(name, obj):
    path = os.path.join(OUT, name)
    with open(path, "w") as f:
        json.dump(obj, f, separators=(",", ":"))
    print(f"wrote {path} ({os.path.getsize(path)} bytes)", flush=True)


def main_naive_mode(what):
    """Run inside a subprocess with BLOKUS_USE_FRONTIER_MOVEGEN=0 (naive order)."""
    _run_order_dependent(what, "naive")


def _run_order_dependent(what, order):
    specs = [s for s in POSITION_SPECS if s[0] >= 8][:PLAYOUT_POSITIONS]
    idx_of = {s: POSITION_SPECS.index(s) for s in specs}
    with Pool(8) as pool:
        if what in ("all", "playouts"):
            jobs = [(idx_of[s], s, [1000 * s[1] + k for k in range(4)]) for s in specs]
            dump(f"playouts_{order}.json", pool.map(gen_playouts, jobs))
        if what in ("all", "rollouts"):
            jobs = [(idx_of[s], s, 77 + s[1]) for s in specs[:32]]
            dump(f"rollouts_a_{order}.json", pool.map(gen_rollout_a, jobs))


def main():
    os.makedirs(OUT, exist_ok=True)
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "--naive":
        assert os.environ.get("BLOKUS_USE_FRONTIER_MOVEGEN") == "0"
        main_naive_mode(sys.argv[2] if len(sys.argv) > 2 else "all")
        return
    if what in ("all", "pieces"):
        dump("pieces.json", gen_pieces())
    if what in ("all", "rng"):
        dump("rng.json", gen_rng())
    if what in ("all", "positions"):
        with Pool(8) as pool:
            recs = pool.map(gen_position, POSITION_SPECS)
        for i, r in enumerate(recs):
            if i >= FULL_LIST_POSITIONS:
                for p in r["players"]:
                    p.pop("frontier_list")
                    p.pop("naive_list")
        dump("positions.json", recs)
    if what in ("all", "playouts", "rollouts"):
        _run_order_dependent(what, "frontier")
        env = dict(os.environ, BLOKUS_USE_FRONTIER_MOVEGEN="0", PYTHONDONTWRITEBYTECODE="1")
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--naive", what], env=env)
    if what in ("all", "fastmcts"):
        specs = [s for s in POSITION_SPECS if 8 <= s[0] <= 40][:16]
        jobs = []
        for j, s in enumerate(specs):
            for iters in (40, 600, 2500):
                jobs.append((POSITION_SPECS.index(s), s, 500 + j, iters))
        with Pool(8) as pool:
            dump("fastmcts.json", pool.map(gen_fastmcts, jobs))
    if what in ("all", "zobrist"):
        dump("zobrist.json", gen_zobrist())
    if what in ("all", "arena"):
        dump("arena_small.json", gen_arena())
    if what in ("all", "arena_runs"):
        dump("arena_runs.json", gen_arena_runs())
    if what in ("all", "arena_cap"):
        dump("arena_cap.json", gen_arena_cap())
    if what in ("all", "mcts"):
        with Pool(8) as pool:
            dump("mcts.json", pool.map(gen_mcts_case, MCTS_CASES))
    if what in ("all", "heuristic"):
        dump("heuristic.json", gen_heuristic())
    if what == "arena_bench":  # ~30 min: MCTS seats with heuristic rollouts in Python
        with Pool(4) as pool:
            dump("arena_bench.json", {"config": ARENA_BENCH, "games": pool.map(_bench_arena_game, range(4))})


if __name__ == "__main__":
    main()
