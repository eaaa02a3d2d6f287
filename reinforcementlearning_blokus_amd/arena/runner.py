"""Arena game loop and experiment writer (reference: analytics/tournament/arena_runner.py).

``run_games_gpu`` is the batched path for all-random seatings: every game is one lane of
the frontier-order playout kernel, started from the empty board with each seat's
RandomAgent seed (``_agent_seed``), so its record equals ``run_single_game``'s for the
same run seed and game index.  ``run_single_game`` is the reference loop itself
(:578-777) over the GPU-backed ``BlokusGame`` for every other seating.
"""
from __future__ import annotations

import gc
import json
import random
import os
import time
import warnings
import traceback
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np

from ..agents.fast_mcts_agent import FastMCTSAgent
from ..agents.gameplay_fast_mcts import GameplayFastMCTSAgent
from ..agents.heuristic_agent import HeuristicAgent
from ..agents.random_agent import RandomAgent
from ..engine.board import Player
from ..engine.game import BlokusGame
from ..mcts.mcts_agent import MCTSAgent
from .config import (AgentConfig, RunConfig, agent_seed, game_seed_from_run_seed, seat_assignment_for_game)
from .stats import compute_summary

# ---------------------------------------------------------------------------- agents


class _SelectActionAdapter:
    def __init__(self, agent: Any):
        self.agent = agent

    def choose_move(self, board, player, legal_moves, thinking_time_ms):
        start = time.perf_counter()
        move = self.agent.select_action(board, player, legal_moves)
        stats: Dict[str, Any] = {"timeSpentMs": (time.perf_counter() - start) * 1000.0}
        if isinstance(self.agent, MCTSAgent):
            info = self.agent.get_action_info().get("stats", {})
            if info.get("iterations_run") is not None:
                stats["iterations_run"] = info["iterations_run"]
            if info.get("time_elapsed") is not None:
                stats["timeSpentMs"] = float(info["time_elapsed"]) * 1000.0
        return move, stats


class _FastMCTSAdapter:
    """deterministic_time_budget: iterations = round(iterations_per_ms * budget) (:333-371)."""

    def __init__(self, agent: FastMCTSAgent, *, deterministic_time_budget: bool, iterations_per_ms: float):
        self.agent = agent
        self.deterministic_time_budget = deterministic_time_budget
        self.iterations_per_ms = iterations_per_ms

    def choose_move(self, board, player, legal_moves, thinking_time_ms):
        budget = int(thinking_time_ms or max(int(self.agent.time_limit * 1000), 1))
        if self.deterministic_time_budget:
            cap = max(1, int(round(self.iterations_per_ms * budget)))
            orig, self.agent.iterations = self.agent.iterations, cap
            try:
                res = self.agent.think(board, player, legal_moves, max(10_000_000, budget))
            finally:
                self.agent.iterations = orig
            stats = dict(res.get("stats") or {})
            stats["timeBudgetMs"], stats["iterationCap"] = budget, cap
            return res.get("move"), stats
        res = self.agent.think(board, player, legal_moves, budget)
        return res.get("move"), dict(res.get("stats") or {})


class _GameplayFastMCTSAdapter:
    def __init__(self, agent: GameplayFastMCTSAgent, *, deterministic_time_budget: bool, iterations_per_ms: float):
        self.agent = agent
        self.deterministic_time_budget = deterministic_time_budget
        self.iterations_per_ms = iterations_per_ms

    def choose_move(self, board, player, legal_moves, thinking_time_ms):
        budget = int(thinking_time_ms or 1)
        if self.deterministic_time_budget:
            cap = max(1, int(round(self.iterations_per_ms * budget)))
            orig, self.agent._agent.iterations = self.agent._agent.iterations, cap
            try:
                move, stats = self.agent.choose_move(board, player, legal_moves, max(10_000_000, budget))
            finally:
                self.agent._agent.iterations = orig
            stats = dict(stats or {})
            stats["timeBudgetMs"], stats["iterationCap"] = budget, cap
            return move, stats
        move, stats = self.agent.choose_move(board, player, legal_moves, budget)
        return move, dict(stats or {})


def build_agent(config: AgentConfig, seed: int):
    """Agent adapter from configuration (:415-492).  ``mcts`` seats search with the
    reference's default HeuristicAgent rollouts (MCTSAgent "exact" backend); learned
    evaluation options are out of scope and rejected by MCTSAgent."""
    kind = config.type.lower()
    params = dict(config.params)
    if kind == "random":
        return _SelectActionAdapter(RandomAgent(seed=seed))
    if kind == "heuristic":
        agent = HeuristicAgent(seed=seed)
        weights = params.get("weights")
        if isinstance(weights, Mapping):
            agent.set_weights(dict(weights))
        return _SelectActionAdapter(agent)
    if kind == "mcts":
        deterministic = bool(params.get("deterministic_time_budget", True))
        iterations = int(params.get("iterations", 1000))
        time_limit = params.get("time_limit")
        if deterministic and config.thinking_time_ms is not None:
            iterations = max(1, int(round(float(params.get("iterations_per_ms", 10.0)) * config.thinking_time_ms)))
            time_limit = None
        elif time_limit is None and config.thinking_time_ms is not None:
            time_limit = float(config.thinking_time_ms) / 1000.0
        return _SelectActionAdapter(MCTSAgent(
            iterations=iterations, time_limit=float(time_limit) if time_limit is not None else None,
            exploration_constant=float(params.get("exploration_constant", 1.414)),
            use_transposition_table=bool(params.get("use_transposition_table", True)), seed=seed,
            learned_model_path=params.get("learned_model_path"),
            leaf_evaluation_enabled=bool(params.get("leaf_evaluation_enabled", False)),
            progressive_bias_enabled=bool(params.get("progressive_bias_enabled", False)),
            potential_shaping_enabled=bool(params.get("potential_shaping_enabled", False)),
            max_rollout_moves=int(params.get("max_rollout_moves", 50))))
    if kind == "fast_mcts":
        default_time = (float(config.thinking_time_ms) / 1000.0 if config.thinking_time_ms is not None
                        else float(params.get("time_limit", 0.1)))
        agent = FastMCTSAgent(iterations=int(params.get("iterations", 5000)), time_limit=default_time,
                              exploration_constant=float(params.get("exploration_constant", 1.414)), seed=seed)
        return _FastMCTSAdapter(agent, deterministic_time_budget=bool(params.get("deterministic_time_budget", True)),
                                iterations_per_ms=float(params.get("iterations_per_ms", 20.0)))
    if kind in {"gameplay_fast_mcts", "gameplay_mcts"}:
        agent = GameplayFastMCTSAgent(iterations=int(params.get("iterations", 5000)),
                                      exploration_constant=float(params.get("exploration_constant", 1.414)), seed=seed)
        return _GameplayFastMCTSAdapter(agent,
                                        deterministic_time_budget=bool(params.get("deterministic_time_budget", True)),
                                        iterations_per_ms=float(params.get("iterations_per_ms", 20.0)))
    raise ValueError(f"Unsupported agent type: {config.type}")


# ---------------------------------------------------------------------------- records


def _compute_ranks(scores: Mapping[str, int]) -> Dict[str, int]:
    order = sorted(set(scores.values()), reverse=True)
    rank = {s: i + 1 for i, s in enumerate(order)}
    return {pid: rank[s] for pid, s in scores.items()}


def _extract_move_telemetry(raw: Mapping[str, Any], fallback_ms: float) -> Tuple[float, Optional[float]]:
    t = raw.get("timeSpentMs")
    if t is None and raw.get("time_elapsed") is not None:
        t = float(raw["time_elapsed"]) * 1000.0
    if t is None:
        t = fallback_ms
    sims = None
    for key in ("nodesEvaluated", "iterations_run", "simulations", "rollouts"):
        if raw.get(key) is not None:
            try:
                sims = float(raw[key])
                break
            except (TypeError, ValueError):
                continue
    return float(t), sims


def _finish_stats(per_agent: Dict[str, Dict[str, Any]]) -> None:
    for e in per_agent.values():
        moves = e["moves"]
        e["avg_time_ms"] = e["total_time_ms"] / moves if moves > 0 else 0.0
        if e["moves_with_simulations"] > 0:
            e["avg_simulations_per_move"] = e["total_simulations"] / e["moves_with_simulations"]
            ts = e["total_time_ms"] / 1000.0
            e["simulations_per_second"] = e["total_simulations"] / ts if ts > 0 else None
        else:
            e["avg_simulations_per_move"] = None
            e["simulations_per_second"] = None
            e["total_simulations"] = None


def _record(*, run_id, game_index, game_seed, run_config, seats, scores, winner_ids, is_tie, moves_made,
            turn_count, passes, invalid, duration, truncated, per_agent, error) -> Dict[str, Any]:
    scores = {str(k): int(v) for k, v in scores.items()}
    ranks = _compute_ranks(scores)
    return {
        "run_id": run_id, "game_id": f"{run_id}_g{game_index:04d}", "game_index": game_index,
        "game_seed": game_seed, "seat_assignment": dict(seats), "seat_policy": run_config.seat_policy,
        "winner_ids": winner_ids, "winner_agents": [seats[str(p)] for p in winner_ids], "is_tie": bool(is_tie),
        "final_scores": scores, "final_ranks": ranks, "agent_scores": {seats[p]: s for p, s in scores.items()},
        "agent_ranks": {seats[p]: r for p, r in ranks.items()},
        "winner_id": winner_ids[0] if len(winner_ids) == 1 else None, "moves_made": int(moves_made),
        "turn_count": int(turn_count), "passes": int(passes), "invalid_actions": int(invalid),
        "duration_sec": float(duration), "truncated": bool(truncated), "agent_move_stats": per_agent,
        "snapshot_checkpoints_hit": [], "error": error,
    }


def run_single_game(*, run_id: str, game_index: int, game_seed: int, run_config: RunConfig,
                    seat_assignment: Mapping[str, str], agent_configs: Mapping[str, AgentConfig]) -> Dict[str, Any]:
    """The reference loop (:652-697): pass when stuck, validate every move, game over when
    nobody can move, max_turns truncation."""
    random.seed(game_seed)
    np.random.seed(game_seed)
    start = time.perf_counter()
    agents = {n: build_agent(agent_configs[n], seed=agent_seed(run_config.seed, game_index, n))
              for n in set(seat_assignment.values())}
    per_agent = {n: {"moves": 0.0, "total_time_ms": 0.0, "total_simulations": 0.0, "moves_with_simulations": 0.0,
                     "move_times_ms": []} for n in set(seat_assignment.values())}
    game = BlokusGame()
    passes = invalid = turns = 0
    truncated, error = False, None
    try:
        while not game.is_game_over() and turns < run_config.max_turns:
            cur = game.get_current_player()
            name = seat_assignment[str(cur.value)]
            legal = game.get_legal_moves(cur)
            turns += 1
            if not legal:
                passes += 1
                game.board._update_current_player()
                game._check_game_over()
                continue
            t0 = time.perf_counter()
            move, raw = agents[name].choose_move(game.board, cur, legal, agent_configs[name].thinking_time_ms)
            elapsed, sims = _extract_move_telemetry(raw, (time.perf_counter() - t0) * 1000.0)
            e = per_agent[name]
            e["moves"] += 1
            e["total_time_ms"] += elapsed
            e["move_times_ms"].append(elapsed)
            if sims is not None:
                e["total_simulations"] += sims
                e["moves_with_simulations"] += 1
            if move is None or not game.make_move(move, cur):
                invalid += move is not None
                passes += 1
                game.board._update_current_player()
                game._check_game_over()
    except Exception:  # noqa: BLE001 - recorded like the reference
        error = traceback.format_exc()
    if turns >= run_config.max_turns and not game.is_game_over():
        truncated = True
        game.board.game_over = True
    res = game.get_game_result()
    _finish_stats(per_agent)
    return _record(run_id=run_id, game_index=game_index, game_seed=game_seed, run_config=run_config,
                   seats=seat_assignment, scores=res.scores, winner_ids=[int(w) for w in res.winner_ids],
                   is_tie=res.is_tie, moves_made=game.board.move_count, turn_count=turns, passes=passes,
                   invalid=invalid, duration=time.perf_counter() - start, truncated=truncated,
                   per_agent=per_agent, error=error)


def _all_random(run_config: RunConfig) -> bool:
    return all(a.type.lower() == "random" for a in run_config.agents)


STATUS_CAP = 8  # bk_result.status bit 3 (include/blokus_hip.h)


def run_games_gpu(run_config: RunConfig, game_indices: Sequence[int], *, run_id: str = "gpu",
                  device: int = 0) -> List[Dict[str, Any]]:
    """All-random seatings: the games ``game_indices`` in one frontier-order playout launch.
    Per-move times are not observable inside the kernel; each game's duration is its
    share of the launch and per-agent time is split by moves made."""
    from .. import _native as N
    from ..gpu import BlokusGPU, empty_state
    if not _all_random(run_config):
        raise ValueError("run_games_gpu plays all-random seatings; use run_single_game")
    idx = list(game_indices)
    n = len(idx)
    if n == 0:
        return []
    seats, seeds, gseeds = [], np.zeros((n, 4), dtype=np.uint32), []
    for i, gi in enumerate(idx):
        gs = game_seed_from_run_seed(run_config.seed, gi)
        st = seat_assignment_for_game(run_config.agent_names, gi, gs, run_config.seat_policy)
        gseeds.append(gs)
        seats.append(st)
        seeds[i] = [agent_seed(run_config.seed, gi, st[str(p + 1)]) for p in range(4)]
    gpu = BlokusGPU(device)
    t0 = time.perf_counter()
    states, _sets, res = gpu.rollout_frontier(empty_state(), N.fset_new(1), n, semantics=N.SEM_ARENA,
                                              rng=N.RNG_NUMPY_MT, compat_seeds=seeds,
                                              max_plies=run_config.max_turns,
                                              root_index=np.zeros(n, dtype=np.int32), with_states=True)
    # A game the kernel stopped at max_turns (status bit 3) may or may not be over: it
    # stops without looking ahead.  has_legal_moves of its final position decides
    # (arena_runner.py:653, :702): still alive -> truncated; over -> it ended with its
    # last move, so the passes counted since then never happened in the reference.
    at_cap = np.flatnonzero(res["status"] & STATUS_CAP)
    alive = np.zeros(n, dtype=bool)
    if len(at_cap):
        alive[at_cap] = gpu.has_moves(states[at_cap]) != 0
    res = res.copy()
    for i in at_cap[~alive[at_cap]]:
        k = int(res["reserved"][i, 0])
        res["passes"][i] -= k
        res["turns"][i] -= k
    res["status"] &= ~np.uint8(STATUS_CAP)
    dt = time.perf_counter() - t0
    out = []
    for i, gi in enumerate(idx):
        r = res[i]
        if int(r["status"]) != 0:
            raise RuntimeError(f"game {gi}: kernel status {int(r['status'])} (stream/table overflow)")
        scores = {p + 1: int(r["scores"][p]) for p in range(4)}
        best = max(scores.values())
        winners = [p for p, s in scores.items() if s == best]
        moves = [bin(int(u)).count("1") for u in states[i]["used"]]
        per_agent = {}
        for p in range(4):
            name = seats[i][str(p + 1)]
            share = dt / n * (moves[p] / max(sum(moves), 1)) * 1000.0
            per_agent[name] = {"moves": float(moves[p]), "total_time_ms": share,
                               "total_simulations": 0.0, "moves_with_simulations": 0.0, "move_times_ms": []}
        _finish_stats(per_agent)
        turns = int(r["turns"])
        out.append(_record(run_id=run_id, game_index=gi, game_seed=gseeds[i], run_config=run_config,
                           seats=seats[i], scores=scores, winner_ids=winners, is_tie=len(winners) > 1,
                           moves_made=int(states[i]["move_count"]), turn_count=turns, passes=int(r["passes"]),
                           invalid=0, duration=dt / n, truncated=bool(alive[i]),
                           per_agent=per_agent, error=None))
    return out


_SEARCH_KINDS = ("mcts", "fast_mcts", "gameplay_fast_mcts", "gameplay_mcts")

_MOVE_TABLES = None


def _move_tables():
    """(uint64[91 * 400, 7] plane words of each move int g * 400 + anchor (0 for off-board
    anchors), int64[91] piece index 0..20 of each orientation), built once."""
    global _MOVE_TABLES
    if _MOVE_TABLES is None:
        from ..engine.pieces import ORIENT_CELLS, ORIENT_LIST
        masks = np.zeros((91 * 400, 7), np.uint64)
        for g, cells in enumerate(ORIENT_CELLS):
            for a in range(400):
                ar, ac = divmod(a, 20)
                cs = [(ar + dr, ac + dc) for dr, dc in cells]
                if all(0 <= r < 20 and 0 <= c < 20 for r, c in cs):
                    for r, c in cs:
                        k = r * 20 + c
                        masks[g * 400 + a, k // 64] |= np.uint64(1) << np.uint64(k % 64)
        pieces = np.array([pid - 1 for pid, _o in ORIENT_LIST], np.int64)
        _MOVE_TABLES = (masks, pieces)
    return _MOVE_TABLES


def _batchable(run_config: RunConfig, seats: Mapping[str, str]) -> bool:
    """run_games_batched can play this seating: random / default-weight heuristic seats
    each with their own agent (a stream per seat), search seats of the supported kinds
    (FastMCTS kinds only with deterministic_time_budget, the default)."""
    cfgs = {a.name: a for a in run_config.agents}
    names = list(seats.values())
    for name in set(names):
        c = cfgs[name]
        kind = c.type.lower()
        if kind in ("random", "heuristic"):
            if names.count(name) > 1 or (kind == "heuristic" and c.params.get("weights")):
                return False
        elif kind not in _SEARCH_KINDS:
            return False
        elif kind != "mcts" and not bool(c.params.get("deterministic_time_budget", True)):
            # a wall-clock FastMCTS budget: its iteration count depends on the seat's own
            # timing (arena_runner.py:352-369), so it plays in the host loop
            return False
    return True


LAST_BATCH_PROFILE: Dict[str, float] = {}  # phase times of the last run_games_batched call


_MCTS_WORKER: Optional[ThreadPoolExecutor] = None


def _mcts_worker() -> ThreadPoolExecutor:
    """The thread run_games_batched runs its MCTS launches on (one per process, idle
    between runs; BlokusGPU.shared gives it its own engine and stream)."""
    global _MCTS_WORKER
    if _MCTS_WORKER is None:
        _MCTS_WORKER = ThreadPoolExecutor(1, thread_name_prefix="bk-mcts")
    return _MCTS_WORKER


class _InlineWorker:
    """ArenaOptions.serial_worker: the MCTS searches run on the calling thread (profiling: cProfile
    sees one thread), the same work in the same order."""

    @staticmethod
    def submit(fn, *args):
        from concurrent.futures import Future
        f: Future = Future()
        f.set_result(fn(*args))
        return f


def _timed_search(agents, roots, sets, players):
    t0 = time.perf_counter()
    mv = MCTSAgent.search_packed(agents, roots, sets, players)
    return mv, time.perf_counter() - t0


def _device_agents(run_config: RunConfig, seats_of: Sequence[Mapping[str, str]], idx: Sequence[int]):
    """The search-seat agents of every game as run_single_game builds them (build_agent,
    agent_seed), reduced to what the device driver carries: per MCTSAgent its search
    parameters, Zobrist table and rollout agent's numpy MT19937 state; per FastMCTSAgent
    its iteration count, exploration constant and random.Random state.  None if some agent
    cannot be replayed on the device (wall-clock budgets, rollout agents the kernels do not
    implement): run_games_batched then plays the host-staged loop."""
    from .. import mt19937
    from ..mcts.mcts_agent import _search_policy
    from ..mcts.zobrist import flat_keys
    cfgs = {a.name: a for a in run_config.agents}
    mcts, fast = [], []  # (game i, name, ...)
    seat_agent = np.full((len(idx), 4), -1, np.int64)  # index into mcts / fast
    seat_kind = np.zeros((len(idx), 4), np.int8)  # 0 random/heuristic, 1 mcts, 2 fast
    # An MCTSAgent's seed only seeds its ZobristHash and its rollout HeuristicAgent, two
    # RandomState(seed) streams (build_agent).  The first agent of each name is built and
    # checked against mt19937 (keys = the first 2,088 uint64 draws, rollout state = the
    # fresh state); the others take its seed-independent fields and get their keys and
    # states from mt19937 for all seeds at once (RandomState construction was ~0.2 ms per
    # agent).  A name whose first agent does not match is built agent by agent.  Likewise
    # a FastMCTSAgent, whose seed only seeds its random.Random (python_random_states).
    tmpl: Dict[str, Optional[Dict[str, Any]]] = {}
    lazy: List[Tuple[int, int]] = []  # (index into mcts, seed)
    lazy_fast: List[Tuple[int, int]] = []  # (index into fast, seed): FastMCTSAgent's random.Random state
    for i, gi in enumerate(idx):
        st = seats_of[i]
        # RunConfig holds exactly 4 distinct agents (arena_runner.py:125-200), so an agent
        # plays one seat of a game and searches at most once per piece: the device TT
        # capacity below relies on it
        assert len({st[str(p + 1)] for p in range(4)}) == 4, st
        done: Dict[str, Tuple[int, int]] = {}
        for p in range(4):
            name = st[str(p + 1)]
            c = cfgs[name]
            kind = c.type.lower()
            if kind not in _SEARCH_KINDS:
                continue
            if name not in done:
                seed = agent_seed(run_config.seed, gi, name)
                if kind == "mcts" and tmpl.get(name) is not None and 0 <= seed <= 0xFFFFFFFF:
                    mcts.append(dict(tmpl[name], i=i, zob=None, mt=None))
                    lazy.append((len(mcts) - 1, seed))
                    done[name] = (1, len(mcts) - 1)
                    seat_kind[i, p], seat_agent[i, p] = done[name]
                    continue
                if kind == "fast_mcts" and tmpl.get(name) is not None and seed >= 0:
                    fast.append(dict(tmpl[name], i=i, mt=None))
                    lazy_fast.append((len(fast) - 1, seed))
                    done[name] = (2, len(fast) - 1)
                    seat_kind[i, p], seat_agent[i, p] = done[name]
                    continue
                ad = build_agent(c, seed)
                if isinstance(ad, _SelectActionAdapter) and isinstance(ad.agent, MCTSAgent):
                    a = ad.agent
                    pol = _search_policy(a.rollout_agent) if a.rollout_backend == "search" else None
                    if a.time_limit or pol is None:
                        return None
                    rs = a.rollout_agent.rng.get_state()
                    mt = np.zeros(625, np.uint32)
                    mt[:624], mt[624] = rs[1], rs[2]
                    mcts.append({"i": i, "name": name, "iters": int(a.iterations), "roll": int(a.max_rollout_moves),
                                 "c": float(a.exploration_constant), "tt": bool(a.use_transposition_table),
                                 "policy": int(pol), "zob": flat_keys(a.zobrist_hash), "mt": mt})
                    done[name] = (1, len(mcts) - 1)
                    if kind == "mcts" and name not in tmpl:
                        ok = 0 <= seed <= 0xFFFFFFFF
                        if ok:
                            s0 = mt19937.seed_states([seed])
                            ok = (np.array_equal(mcts[-1]["zob"], mt19937.uint64_draws([seed], 2088, s0)[0])
                                  and np.array_equal(mt[:624], s0[0]) and int(mt[624]) == 624)
                        tmpl[name] = {k: v for k, v in mcts[-1].items() if k not in ("i", "zob", "mt")} if ok else None
                elif isinstance(ad, (_FastMCTSAdapter, _GameplayFastMCTSAdapter)):
                    if not ad.deterministic_time_budget:
                        return None
                    if isinstance(ad, _FastMCTSAdapter):
                        fa = ad.agent
                        budget = int(c.thinking_time_ms or max(int(fa.time_limit * 1000), 1))
                    else:
                        fa = ad.agent._agent
                        budget = int(c.thinking_time_ms or 1)
                    fast.append({"i": i, "name": name, "iters": max(1, int(round(ad.iterations_per_ms * budget))),
                                 "c": float(fa.exploration_constant), "mt": fa._rng_words()})
                    done[name] = (2, len(fast) - 1)
                    if kind == "fast_mcts" and name not in tmpl:  # (its seed only seeds random.Random)
                        ok = seed >= 0 and np.array_equal(fast[-1]["mt"], mt19937.python_random_states([seed])[0])
                        tmpl[name] = {k: v for k, v in fast[-1].items() if k not in ("i", "mt")} if ok else None
                else:
                    return None
            seat_kind[i, p], seat_agent[i, p] = done[name]
    if lazy:
        states = mt19937.seed_states([sd for _, sd in lazy])
        zob = mt19937.uint64_draws(None, 2088, states)
        mts = np.concatenate([states, np.full((len(lazy), 1), 624, np.uint32)], axis=1)
        for j, (k, _) in enumerate(lazy):
            mcts[k]["zob"], mcts[k]["mt"] = zob[j], mts[j]
    if lazy_fast:
        words = mt19937.python_random_states([sd for _, sd in lazy_fast])
        for j, (k, _) in enumerate(lazy_fast):
            fast[k]["mt"] = words[j]
    return mcts, fast, seat_kind, seat_agent


def _capture_failed_job(capture_dir: str, job: Dict[str, Any], o, bad, zob_d, log_tables, record=None) -> str:
    """Diagnostics for a search launch that returned a failed search (ArenaOptions.capture_dir).
    Saves the launch's inputs as the kernel saw them, its outputs and the failed searches'
    node pools, then replays on a fresh handle and stream with nothing else running:
    (a) the whole launch, (b) the failed searches alone, (c) the whole launch over node
    pools pre-filled with the failed run's final pools (a dirty pool).  A clean (a)/(b)
    points at the concurrent run (another writer, a buffer lifetime); a replay that fails
    the same way points at the kernel and its inputs.  Returns the file prefix."""
    import json

    import torch

    from .. import _native as N
    from ..gpu import BlokusGPU, mcts_node_cap
    os.makedirs(capture_dir, exist_ok=True)
    base = os.path.join(capture_dir, f"mcts_fail_job{job['seq']}")
    cap = job["cap"]
    iters, roll, c, use_tt, policy = job["key"]
    dev = cap["roots"].device
    torch.cuda.synchronize(dev)
    n = cap["roots"].shape[0]
    bad_idx = np.flatnonzero(bad)
    arrs = {k: v.cpu().numpy() for k, v in cap.items()}
    if job["nodes"] is not None:
        arrs["nodes_bad"] = job["nodes"][bad_idx].cpu().numpy()
    arrs.update(out=job["o_d"].cpu().numpy(), bad_idx=bad_idx,
                games=np.asarray(job["games"]), aid=np.asarray(job["aid"]),
                zob=zob_d.index_select(0, cap["zidx"].long()).cpu().numpy(),
                key=np.array([iters, roll, use_tt, policy], np.int64), c=np.array([c]))

    def replay(sel, dirty=False, tune=None):
        s = torch.as_tensor(np.asarray(sel, np.int64), device=dev)
        k = len(sel)
        g = BlokusGPU(dev.index)
        if tune:
            g.tune(**tune)
        st = torch.cuda.Stream(dev)
        st.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(st):
            pick = lambda t: t.index_select(0, s).contiguous()  # noqa: E731
            width = mcts_node_cap(iters) * N.MCTS_NODE_DTYPE.itemsize
            nodes = pick(job["nodes"]) if dirty else torch.zeros((k, width), dtype=torch.uint8, device=dev)
            out = torch.zeros((k, N.MCTS_OUT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
            tt = (pick(cap["ttk"]), pick(cap["ttv"]), pick(cap["ttc"])) if use_tt else (None, None, None)
            g.mcts_device(pick(cap["roots"]), pick(cap["sets"]), pick(cap["players"]), None, zob_d,
                          pick(cap["zidx"]), pick(cap["mt"]), log_tables[iters], nodes, out, iterations=iters,
                          tt_keys=tt[0], tt_vals=tt[1], tt_count=tt[2], max_rollout_moves=roll, exploration=c,
                          rollout_policy=policy, asynchronous=True)
        st.synchronize()
        err = None
        try:
            g.synchronize()
        except RuntimeError as e:  # a failure record (BK_ECHECK): keep it with the replay
            err = str(e)
        return out.cpu().numpy().view(N.MCTS_OUT_DTYPE).reshape(k), g.last_kernel(), err, g.mcts_failure()

    orig = o
    fields = ["best_move", "iterations_run", "tt_hits", "rollouts", "nodes_used", "status"]
    report = {"seq": job["seq"], "n": int(n), "bad_idx": bad_idx.tolist(), "slot": job["slot"],
              "inflight_at_launch": job["inflight_at_launch"], "key": [iters, roll, c, use_tt, policy],
              "orig_status": orig["status"][bad_idx].tolist(), "failure_record": record}
    runs = [("whole", np.arange(n), False, None), ("bad_alone", bad_idx, False, None),
            ("whole_one_block_per_cu", np.arange(n), False, {"COOP_BLOCKS_PER_CU": 1}),
            ("whole_per_lane_kernel", np.arange(n), False, {"MCTS_COOP": 0})]
    if job["nodes"] is not None:
        runs.append(("whole_dirty_pool", np.arange(n), True, None))
    for name, sel, dirty, tune in runs:
        if len(sel) == 0:
            continue
        r, kname, err, rec = replay(sel, dirty, tune)
        arrs["replay_" + name] = r.view(np.uint8)
        ref = orig[sel]
        diff = [int(i) for i in range(len(sel)) if any(r[f][i] != ref[f][i] for f in fields)]
        report[name] = {"kernel": kname, "status_bad": int(np.count_nonzero(r["status"] & ~np.uint32(N.MCTS_EUNCERT))),
                        "differs_from_launch": [int(sel[i]) for i in diff][:64], "n_differs": len(diff),
                        "synchronize_error": err, "failure_record": rec,
                        "best_move": r["best_move"].tolist(), "iterations_run": r["iterations_run"].tolist(),
                        "status": r["status"].tolist()}
    np.savez_compressed(base + ".npz", **arrs)
    with open(base + ".json", "w") as f:
        json.dump(report, f, indent=1)
    return base


def _run_games_device(run_config: RunConfig, idx: List[int], seats: List[Mapping[str, str]], gseeds: List[int],
                      agents_dev, *, run_id: str, device: int, progress=None,
                      opts: "ArenaOptions") -> List[Dict[str, Any]]:
    """run_games_batched with every position, frontier table and agent stream resident in
    HBM for the whole run.  A round is: bk_arena_step over all games (each first places
    the move its stop seat chose last round, then plays random / heuristic seats to the
    next search seat or the end; at a FastMCTS seat it also returns the root's legal count
    and _quick_move_evaluation), one bk_mcts launch per MCTS parameter group on the
    stopped positions (gathered on the device), one bk_fastmcts launch for the FastMCTS
    seats; the chosen moves go back as forced moves (a move int, or a list index for
    FastMCTS).  Only results, stop infos and forced moves cross PCIe each round, plus the
    searched positions' 256 bytes for their root Zobrist hash.  Same agents, seeds, streams
    and move order as run_single_game (arena_runner.py:578-777)."""
    import torch

    from .. import _native as N
    from ..agents.fast_mcts_agent import _log_table
    from ..gpu import BlokusGPU, empty_state, mcts_log_table, mcts_node_cap
    from ..mcts.mcts_agent import SEARCH_TOTALS
    mcts, fast, seat_kind, seat_agent = agents_dev
    n = len(idx)
    cfgs = {a.name: a for a in run_config.agents}
    gpu = BlokusGPU(device)
    dev = torch.device("cuda", device)
    prof = LAST_BATCH_PROFILE
    prof.clear()
    t0 = time.perf_counter()
    masks = np.zeros(n, np.uint8)
    quick = np.zeros(n, np.uint8)
    rng = np.zeros((n, 16), np.uint32)
    cur_at, cur_seed = [], []  # (game, seat) of each random / heuristic seat, its agent seed
    for i, gi in enumerate(idx):
        for p in range(4):
            name = seats[i][str(p + 1)]
            kind = cfgs[name].type.lower()
            if kind in ("random", "heuristic"):
                cur_at.append((i, p))
                cur_seed.append(agent_seed(run_config.seed, gi, name))
                if kind == "heuristic":
                    masks[i] |= 1 << p
            else:
                masks[i] |= 16 << p
                if seat_kind[i, p] == 2:
                    quick[i] |= 1 << p
    if cur_at:  # the seats' MT cursors in one call
        cursors = N.mt_cursors(cur_seed)
        for (i, p), c in zip(cur_at, cursors):
            rng[i, 4 * p:4 * p + 4] = c
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    states_d = up(np.repeat(empty_state(), n).view(np.uint8).reshape(n, 256))
    sets_d = up(np.repeat(N.fset_new(1), n).view(np.uint8).reshape(n, -1))  # (every game starts from Board())
    masks_d, quick_d, rng_d = up(masks), up(quick), up(rng.view(np.int32))
    forced_d = torch.full((n,), -1, dtype=torch.int32, device=dev)
    out_d = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    stop_d = torch.zeros((n, N.STOP_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    # MCTS agents: Zobrist tables, rollout streams and TTs (one row each) on the device
    am = len(mcts)
    if am:
        zob_h = np.stack([a["zob"] for a in mcts])
        zob_d = up(zob_h.view(np.int64))
        mtm_d = up(np.stack([a["mt"] for a in mcts]).view(np.int32))
        it_max = max(a["iters"] for a in mcts)
        cap = 1 << 12
        while cap < 2 * (22 * it_max + 2):  # an agent searches at most once per piece
            cap *= 2
        ttk_d = torch.zeros((am, cap), dtype=torch.int64, device=dev)
        ttv_d = torch.full((am, cap), float("nan"), dtype=torch.float64, device=dev)
        ttc_d = torch.zeros(am, dtype=torch.int32, device=dev)
        last_iters = np.zeros(am, np.int64)
        log_tables = {}
    mtf = np.stack([a["mt"] for a in fast]) if fast else np.zeros((0, 625), np.uint32)
    fast_tabs: Dict[int, Tuple[Any, Any, Any]] = {}  # iterations -> device log table, pow-fix rows
    per_agent = [{nm: {"moves": 0.0, "total_time_ms": 0.0, "total_simulations": 0.0, "moves_with_simulations": 0.0,
                       "move_times_ms": []} for nm in set(seats[i].values())} for i in range(n)]
    tot = np.zeros((n, 2), np.int64)  # turn_count, passes so far
    results: List[Optional[Tuple[Any, int, int, bool]]] = [None] * n
    active = np.ones(n, bool)
    prof.update(setup_s=time.perf_counter() - t0, advance_s=0.0, mcts_s=0.0, fast_s=0.0, wait_s=0.0, host_s=0.0,
                rounds=0, uncertified_heuristic=0, device_driver=1)
    forced = np.full(n, -1, np.int32)
    caller = torch.cuda.current_stream(dev)
    stream = caller
    if opts.high_priority:
        # the per-step kernels (bk_arena_step, FastMCTS, gathers) on a high-priority stream:
        # when a search block frees a CU they are dispatched before queued search blocks
        stream = torch.cuda.Stream(dev, priority=-1)
        stream.wait_stream(caller)
        torch.cuda.set_stream(stream)
    # MCTS searches run on their own streams and handles (opts.search_streams) and are
    # not waited for: a game whose search is in flight sits at its stop seat
    # (BK_FORCE_SKIP: arena_step does not touch it) while the other games play on and
    # launch their own searches; its move is placed in the first step after the search
    # ends.  FastMCTS seats are decided on the device in the step that stops at them
    # (fast_on_device), so the next step places their move.  opts.pipeline False: one
    # search at a time on the main stream, waited for at once, FastMCTS host-staged.
    pipeline = opts.pipeline
    n_slots = opts.search_streams if pipeline else 1
    job_games = opts.job_games if pipeline else 1 << 30
    engines = [BlokusGPU(device) for _ in range(n_slots)] if pipeline else [gpu]
    jstreams = [torch.cuda.Stream(dev) for _ in range(n_slots)] if pipeline else [stream]
    reserve = opts.reserve_cus if pipeline else 0
    if reserve > 0:  # search streams may not use `reserve` CUs, spread over the chip (bk_stream_create)
        n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
        step = max(1, n_cu // reserve)
        mask = np.zeros((n_cu + 31) // 32, np.uint32)
        for cu in range(n_cu):
            if cu % step != 0 or cu // step >= reserve:
                mask[cu // 32] |= np.uint32(1 << (cu % 32))
        jstreams = [torch.cuda.ExternalStream(e.handle.stream_create(mask), device=dev) for e in engines]
    free_slots = list(range(n_slots))
    jobs: List[Dict[str, Any]] = []
    # opts.capture_dir (diagnostics): keep every search launch's inputs; a launch that
    # returns a failed search is saved there and replayed alone (_capture_failed_job)
    capture_dir = opts.capture_dir or ""
    fast_eng = BlokusGPU(device) if pipeline else gpu
    inflight = np.zeros(n, bool)
    # per-search hand-back: each slot's launches write their out records and done flags
    # into mapped host memory the loop polls (bk_mcts_set_done); the agents' MT / TT rows
    # are updated in place, so a handed-back game may search again while its launch's
    # other searches still run.  (A TT past 500,000 entries is reset between searches,
    # mcts_agent.py:338-339: only possible at > 11,000 iterations -- those runs keep the
    # launch-end path.)
    early = bool(pipeline and opts.handback and not capture_dir and am and cap <= 500000)
    hb_done: Dict[int, Any] = {}

    def mcts_launch_early(slot, games, aid, iters, roll, c, use_tt, policy):
        eng, js = engines[slot], jstreams[slot]
        k = len(games)
        if slot not in hb_done:
            hb_done[slot] = N.HostBuffer(8 * n, np.uint64)
        done_a = hb_done[slot].array
        done_a[:k] = 0  # (the slot's previous launch has ended)
        eng.handle.set_done(hb_done[slot].ptr)
        if int(aid.max()) >= am or int(aid.min()) < 0:
            raise RuntimeError(f"MCTS agent rows out of range: {aid.min()}..{aid.max()} of {am}")
        ga_d = up(np.stack([games, aid]).astype(np.int64))
        gi_d, aid_d = ga_d[0], ga_d[1]
        roots_d = states_d.index_select(0, gi_d).contiguous()
        sets_g = sets_d.index_select(0, gi_d).contiguous()
        players = roots_d[:, 241] & 3
        zi_d = aid_d.to(torch.int32)
        if iters not in log_tables:
            log_tables[iters] = up(mcts_log_table(iters))
        ready = torch.cuda.Event()
        ready.record(stream)
        js.wait_event(ready)
        with torch.cuda.stream(js):
            nodes = torch.empty((k, mcts_node_cap(iters) * N.MCTS_NODE_DTYPE.itemsize), dtype=torch.uint8, device=dev)
            o_d = torch.zeros((k, N.MCTS_OUT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
            eng.mcts_device(roots_d, sets_g, players, None, zob_d, zi_d, mtm_d, log_tables[iters], nodes, o_d,
                            iterations=iters, tt_keys=ttk_d if use_tt else None, tt_vals=ttv_d if use_tt else None,
                            tt_count=ttc_d if use_tt else None, max_rollout_moves=roll, exploration=c,
                            rollout_policy=policy, asynchronous=True, state_rows=True)
            done = torch.cuda.Event()
            done.record(js)
        for t in (ga_d, roots_d, sets_g, players, zi_d):
            t.record_stream(js)
        inflight[games] = True
        jobs.append({"slot": slot, "games": games, "aid": aid, "done": done, "t0": time.perf_counter(),
                     "nodes": nodes, "o_d": o_d, "cap": None, "seq": tl["mcts_jobs_launched"],
                     "key": (iters, roll, c, use_tt, policy), "inflight_at_launch": len(jobs), "early": True,
                     "flags": done_a[:k], "left": np.ones(k, bool)})
        tl["mcts_jobs_launched"] += 1

    def handback(job, ks, words=None):
        """Moves of the job's searches ks (their result words, bk_mcts_set_done): the
        games play on."""
        w = job["flags"][ks] if words is None else words
        status = (w >> np.uint64(56)) & np.uint64(0x7F)
        if (status & ~np.uint64(N.MCTS_EUNCERT)).any():
            jobs.remove(job)
            mcts_finish(job)  # waits for the launch and raises with its failure record
            return
        games, aid = job["games"][ks], job["aid"][ks]
        prof["uncertified_heuristic"] += int(np.count_nonzero(status & np.uint64(N.MCTS_EUNCERT)))
        its = ((w >> np.uint64(32)) & np.uint64(0xFFFFFF)).astype(np.int64)
        best = (w & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
        last_iters[aid] = its
        for i, a, mv, it in zip(games.tolist(), aid.tolist(), best.tolist(), its.tolist()):
            forced[i] = int(mv)
            e = per_agent[i][mcts[a]["name"]]
            e["total_simulations"] += float(it)
            e["moves_with_simulations"] += 1
        inflight[games] = False
        job["left"][ks] = False
        tl["handback_games"] += len(ks)
        tl["handback_s"] += (time.perf_counter() - job["t0"]) * len(ks)

    def mcts_launch(games, pls, aid, iters, roll, c, use_tt, policy):
        slot = free_slots.pop(0)
        if early:
            mcts_launch_early(slot, games, aid, iters, roll, c, use_tt, policy)
            return
        eng, js = engines[slot], jstreams[slot]
        ga_d = up(np.stack([games, aid]).astype(np.int64))  # one copy in; nothing comes back
        gi_d, aid_d = ga_d[0], ga_d[1]
        roots_d = states_d.index_select(0, gi_d).contiguous()
        sets_g = sets_d.index_select(0, gi_d).contiguous()
        players = roots_d[:, 241] & 3  # bk_state.current_player: the searching seat
        rh_d = None  # ZobristHash.hash_board on the device (bk_mcts, k_root_hash)
        zi_d = aid_d.to(torch.int32)
        mt_g = mtm_d.index_select(0, aid_d).contiguous()
        if iters not in log_tables:
            log_tables[iters] = up(mcts_log_table(iters))
        tt = (ttk_d.index_select(0, aid_d), ttv_d.index_select(0, aid_d), ttc_d.index_select(0, aid_d)) \
            if use_tt else (None, None, None)
        ready = torch.cuda.Event()
        ready.record(stream)
        js.wait_event(ready)
        with torch.cuda.stream(js):
            nodes = torch.empty((len(games), mcts_node_cap(iters) * N.MCTS_NODE_DTYPE.itemsize),
                                dtype=torch.uint8, device=dev)
            o_d = torch.zeros((len(games), N.MCTS_OUT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
            cap_in = None
            if capture_dir:  # the launch's inputs as the kernel sees them (it advances mt / tt in place)
                cap_in = {"roots": roots_d.clone(), "sets": sets_g.clone(), "players": players.clone(),
                          "zidx": zi_d.clone(), "mt": mt_g.clone()}
                if use_tt:
                    cap_in.update(ttk=tt[0].clone(), ttv=tt[1].clone(), ttc=tt[2].clone())
            eng.mcts_device(roots_d, sets_g, players, rh_d, zob_d, zi_d, mt_g, log_tables[iters], nodes, o_d,
                            iterations=iters, tt_keys=tt[0], tt_vals=tt[1], tt_count=tt[2],
                            max_rollout_moves=roll, exploration=c, rollout_policy=policy, asynchronous=pipeline)
            mtm_d.index_copy_(0, aid_d, mt_g)
            if use_tt:
                ttk_d.index_copy_(0, aid_d, tt[0])
                ttv_d.index_copy_(0, aid_d, tt[1])
                ttc_d.index_copy_(0, aid_d, tt[2])
            done = torch.cuda.Event()
            done.record(js)
        for t in (ga_d, roots_d, sets_g, players, zi_d, mt_g) + (tt if use_tt else ()):
            t.record_stream(js)
        inflight[games] = True
        # nodes stays referenced until the job is finished: the launch is asynchronous
        jobs.append({"slot": slot, "games": games, "aid": aid, "o_d": o_d, "tc": tt[2], "done": done,
                     "t0": time.perf_counter(), "nodes": nodes, "cap": cap_in, "seq": tl["mcts_jobs_launched"],
                     "key": (iters, roll, c, use_tt, policy), "inflight_at_launch": len(jobs)})
        tl["mcts_jobs_launched"] += 1
        if not pipeline:
            mcts_finish(jobs.pop(0))

    def mcts_finish(job):
        job["done"].synchronize()
        tl["mcts_jobs"] += 1
        tl["mcts_job_s"] += time.perf_counter() - job["t0"]
        tl["mcts_job_games"] += len(job["games"])
        eng = engines[job["slot"]]
        sync_err = None
        try:
            eng.synchronize()  # sticky launch errors, a failure record (BK_ECHECK)
        except RuntimeError as e:
            sync_err = e
        games, aid = job["games"], job["aid"]
        o = job["o_d"].cpu().numpy().view(N.MCTS_OUT_DTYPE).reshape(len(games))
        bad = o["status"] & ~np.uint32(N.MCTS_EUNCERT)
        if bad.any() or sync_err is not None:
            rec = eng.mcts_failure()  # what the failing search saw (bk_debug_mcts_failure)
            if rec is not None:
                rec.update(games=[int(idx[games[rec["game_in_launch"]]])] if rec["game_in_launch"] < len(games) else [],
                           slot=job["slot"], inflight_at_launch=job["inflight_at_launch"], job_seq=job["seq"])
            where = ""
            if capture_dir:
                where = " (inputs and replays in " + _capture_failed_job(capture_dir, job, o, bad, zob_d,
                                                                      log_tables, rec) + ")"
            raise RuntimeError(f"bk_mcts: {int(np.count_nonzero(bad))} searches stopped early, status bits "
                               f"{int(np.bitwise_or.reduce(bad)) if bad.any() else 0}; failure record {rec}; "
                               f"synchronize: {sync_err}{where}")
        its = o["iterations_run"].astype(np.int64)
        kms, kplies = eng.last_kernel_ms(), int(o["rollout_plies"].astype(np.int64).sum())
        if len(games):  # a launch lasts as long as its longest search: its work against the mean
            pl = o["rollout_plies"].astype(np.float64)
            tl["job_plies_max_over_mean"] += float(pl.max() / max(pl.mean(), 1.0))
        for t in (SEARCH_TOTALS, SEARCH_TOTALS["by_kernel"].setdefault(
                eng.last_kernel(), {"launches": 0, "kernel_ms": 0.0, "sims": 0, "rollout_plies": 0})):
            t["launches"] += 1
            t["kernel_ms"] += kms
            t["sims"] += int(its.sum())
            t["rollout_plies"] += kplies
        if job.get("early"):
            rest = np.flatnonzero(job["left"])
            if len(rest):  # (the launch has ended: its out records are complete)
                oo = o[rest]
                handback(job, rest, (oo["best_move"].astype(np.int64) & 0xFFFFFFFF).astype(np.uint64) |
                         (oo["iterations_run"].astype(np.uint64) << np.uint64(32)) |
                         (oo["status"].astype(np.uint64) << np.uint64(56)) | np.uint64(1 << 63))
            free_slots.append(job["slot"])
            return
        prof["uncertified_heuristic"] += int(np.count_nonzero(o["status"] & N.MCTS_EUNCERT))
        last_iters[aid] = its
        for i, a, mv, it in zip(games.tolist(), aid.tolist(), o["best_move"].tolist(), its.tolist()):
            forced[i] = int(mv)
            e = per_agent[i][mcts[a]["name"]]
            e["total_simulations"] += float(it)
            e["moves_with_simulations"] += 1
        if job["tc"] is not None and int(job["tc"].max().item()) > 500000:  # mcts_agent.py:338-339
            full = aid[(job["tc"].cpu().numpy() > 500000)]
            ttk_d[up(full)] = 0
            ttv_d[up(full)] = float("nan")
            ttc_d[up(full)] = 0
        inflight[games] = False
        free_slots.append(job["slot"])
    mtf_d = up(mtf.view(np.int32)) if (pipeline and len(fast)) else None
    fast_dev: List[Tuple[Any, Any]] = []  # this step's (games, forced values) computed on the device

    def fast_on_device(games, aid, nl, counts, ce):
        """FastMCTSAgent.think for these stopped games on the main stream, inputs from the
        step's stop infos on the device; the chosen list index becomes the game's forced
        move on the device (FastMCTSAgent: quick move below 5 iterations, else the best
        child, else index 0), so the next step places it with no host round trip."""
        k = len(games)
        if int(np.max(nl)) > N.FASTMCTS_MAX_CHILDREN:  # k_fastmcts would leave the output unset
            g = int(games[int(np.argmax(nl))])
            raise RuntimeError(f"game {idx[g]}: a FastMCTS root with {int(np.max(nl))} legal moves, more than "
                               f"bk_fastmcts supports ({N.FASTMCTS_MAX_CHILDREN})")
        need = max(counts) + 1
        if need not in fast_tabs:
            lt = _log_table(need)
            fo, fe = N.pow_half_fix(lt, rows=need)
            fast_tabs[need] = (up(lt), up(fo), up(fe if len(fe) else np.zeros(1, np.int32)))
        lt_d, fo_d, fe_d = fast_tabs[need]
        off = np.zeros(k + 1, np.int32)
        np.cumsum(nl.astype(np.int32), out=off[1:])
        meta = up(np.concatenate([off, np.asarray(counts, np.int32), games.astype(np.int32),
                                  aid.astype(np.int32)]))
        off_d, it_d = meta[:k + 1], meta[k + 1:2 * k + 1]
        g_d, a_d = meta[2 * k + 1:3 * k + 1].long(), meta[3 * k + 1:].long()
        st = stop_d.index_select(0, g_d)  # bk_stop_info rows: n_legal, quick_index, quick_reward
        base = st[:, 8:16].contiguous().view(torch.float64).reshape(k)
        quick_i = st[:, 4:8].contiguous().view(torch.int32).reshape(k)
        mt_g = mtf_d.index_select(0, a_d).contiguous()
        o = torch.zeros((k, N.FASTMCTS_OUT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        fast_eng.fastmcts_device(off_d, it_d, base, mt_g, lt_d, fo_d, fe_d, ce, o)
        mtf_d.index_copy_(0, a_d, mt_g)
        w = o[:, :12].contiguous().view(torch.int32)  # best_index, iterations, n_children
        j = torch.where(w[:, 1] < 5, quick_i, torch.where(w[:, 2] > 0, w[:, 0], torch.zeros_like(w[:, 0])))
        fast_dev.append((g_d, (j | N.FORCE_INDEX).to(torch.int32)))
        for i, a, it in zip(games.tolist(), aid.tolist(), counts):
            forced[i] = N.FORCE_INDEX  # placeholder: the device value replaces it
            e = per_agent[i][fast[a]["name"]]
            e["total_simulations"] += it
            e["moves_with_simulations"] += 1

    def fast_launch(games, aid, nl, counts, quick, ce):  # opts.pipeline False: host-staged, waited for
        mt = np.ascontiguousarray(mtf[aid])
        r = gpu.fastmcts(nl.tolist(), counts, quick.tolist(), mt, _log_table(max(counts) + 1), ce)
        mtf[aid] = mt
        for i, a, it_run, bi, nch, it in zip(games.tolist(), aid.tolist(), r["iterations"].tolist(),
                                              r["best_index"].tolist(), r["n_children"].tolist(), counts):
            j = int(stops_q[i]) if it_run < 5 else (int(bi) if nch > 0 else 0)
            forced[i] = N.FORCE_INDEX | j
            e = per_agent[i][fast[a]["name"]]
            e["total_simulations"] += it
            e["moves_with_simulations"] += 1

    def drain():
        moved = False
        for j in list(jobs):
            if j.get("early"):
                new = np.flatnonzero((j["flags"] >> np.uint64(63)).astype(bool) & j["left"])
                if len(new):
                    handback(j, new)
                    moved = True
            if j in jobs and j["done"].query():
                jobs.remove(j)
                mcts_finish(j)
                moved = True
        return moved

    stops_q = np.zeros(n, np.int64)  # the FastMCTS seats' quick_index (stop info)
    # host-side timeline: jobs' launch -> completion seen, games inside a search per step
    tl = {"mcts_jobs": 0, "mcts_job_s": 0.0, "mcts_job_games": 0, "search_games_per_step": 0, "mcts_jobs_launched": 0,
          "job_plies_max_over_mean": 0.0, "handback_games": 0, "handback_s": 0.0}
    try:
        while active.any():
            prof["rounds"] += 1
            tl["search_games_per_step"] += sum(len(j["games"]) for j in jobs)
            if progress is not None:
                progress(prof["rounds"], int(active.sum()), prof)
            ta = time.perf_counter()
            gpu.arena_step(states_d, sets_d, masks_d, rng_d, quick_d, forced_d, out_d, stop_d,
                           max_turns=run_config.max_turns)
            # one copy back per step: results, stop infos, the player to move
            step_h = torch.cat([out_d, stop_d, states_d[:, 240:244]], dim=1).cpu().numpy()
            res = np.ascontiguousarray(step_h[:, :32]).view(N.RESULT_DTYPE).reshape(n)
            stops = np.ascontiguousarray(step_h[:, 32:32 + N.STOP_DTYPE.itemsize]).view(N.STOP_DTYPE).reshape(n)
            to_move = step_h[:, 32 + N.STOP_DTYPE.itemsize + 1].astype(np.int64) & 3  # bk_state byte 241
            prof["advance_s"] += time.perf_counter() - ta
            status = res["status"].astype(np.int64)
            forced[:] = -1
            act = np.flatnonzero(active & ~inflight)
            tot[act, 0] += res["turns"][act]
            tot[act, 1] += res["passes"][act]
            prof["uncertified_heuristic"] += int(np.count_nonzero(status[act] & N.STATUS_UNCERT))
            bad = status[act] & ~(N.STATUS_CAP | N.STATUS_STOP | N.STATUS_UNCERT)
            if bad.any():
                j = int(act[np.flatnonzero(bad)[0]])
                raise RuntimeError(f"game {idx[j]}: kernel status {int(status[j])}")
            stop = act[(status[act] & N.STATUS_STOP) != 0]
            fin = act[(status[act] & N.STATUS_STOP) == 0]
            for i in fin.tolist():
                r = res[i].copy()
                turns, passes, truncated = int(tot[i, 0]), int(tot[i, 1]), False
                if status[i] & N.STATUS_CAP:  # cut by max_turns: over or not (arena_runner.py:702)
                    st_i = states_d[i:i + 1].cpu().numpy().view(N.STATE_DTYPE)
                    if int(gpu.has_moves(st_i)[0]) != 0:
                        truncated = True
                    else:
                        turns -= int(r["reserved"][0])
                        passes -= int(r["reserved"][0])
                results[i] = (r, turns, passes, truncated)
                active[i] = False
            if len(stop):
                pl = (np.zeros(len(stop), np.int64))
                pl[:] = to_move[stop]
                kind = seat_kind[stop, pl]
                ag = seat_agent[stop, pl]
                nleg = stops["n_legal"][stop].astype(np.int64)
                # ---- MCTS seats (select_action answers a single legal move without a search)
                sel = np.flatnonzero(kind == 1)
                if len(sel):
                    tm = time.perf_counter()
                    one = sel[nleg[sel] == 1]
                    for k in one.tolist():
                        i, a = int(stop[k]), int(ag[k])
                        forced[i] = N.FORCE_INDEX
                        e = per_agent[i][mcts[a]["name"]]
                        e["total_simulations"] += float(last_iters[a])  # the agent's stale iterations_run
                        e["moves_with_simulations"] += 1
                    multi = sel[nleg[sel] > 1]
                    groups: Dict[Tuple, List[int]] = {}
                    for k in multi.tolist():
                        a = mcts[int(ag[k])]
                        groups.setdefault((a["iters"], a["roll"], a["c"], a["tt"], a["policy"]), []).append(k)
                    for key, ks in groups.items():
                        # launches of at most job_games searches: a launch ends with its
                        # slowest search, so smaller ones hand finished games back sooner
                        for c0 in range(0, len(ks), job_games):
                            kc = np.array(ks[c0:c0 + job_games])
                            if not free_slots:
                                mcts_finish(jobs.pop(0))
                            mcts_launch(stop[kc], pl[kc], ag[kc], *key)
                    prof["mcts_s"] += time.perf_counter() - tm
                # ---- FastMCTS seats (think: a single legal move draws nothing)
                sel = np.flatnonzero(kind == 2)
                if len(sel):
                    tf = time.perf_counter()
                    for k in sel[nleg[sel] == 1].tolist():
                        forced[int(stop[k])] = N.FORCE_INDEX
                    multi = sel[nleg[sel] > 1]
                    groups = {}
                    for k in multi.tolist():
                        groups.setdefault(fast[int(ag[k])]["c"], []).append(k)
                    for ce, ks in groups.items():
                        ks = np.array(ks)
                        games = stop[ks]
                        aid = ag[ks]
                        counts = [fast[int(a)]["iters"] for a in aid]
                        if pipeline:
                            fast_on_device(games, aid, nleg[ks], counts, ce)
                        else:
                            stops_q[games] = stops["quick_index"][games]
                            fast_launch(games, aid, nleg[ks], counts, stops["quick_reward"][games], ce)
                    prof["fast_s"] += time.perf_counter() - tf
            tm = time.perf_counter()
            drain()
            while jobs and not (forced >= 0).any():  # nothing to place: wait for a search
                if not drain():
                    time.sleep(50e-6)
            prof["wait_s"] += time.perf_counter() - tm
            send = np.where(inflight, np.int32(N.FORCE_SKIP), forced)  # in-flight games: not touched
            forced_d.copy_(torch.from_numpy(send))
            for g_d, v_d in fast_dev:  # FastMCTS choices made on the device this step
                forced_d.index_copy_(0, g_d, v_d)
            fast_dev.clear()
        assert not jobs and not inflight.any()
        prof["timeline"] = {"mcts_jobs": tl["mcts_jobs"],
                            "mcts_job_ms_mean": 1e3 * tl["mcts_job_s"] / max(1, tl["mcts_jobs"]),
                            "mcts_games_per_job": tl["mcts_job_games"] / max(1, tl["mcts_jobs"]),
                            "job_plies_max_over_mean": tl["job_plies_max_over_mean"] / max(1, tl["mcts_jobs"]),
                            "handback": early,
                            "handback_ms_mean": 1e3 * tl["handback_s"] / max(1, tl["handback_games"]),
                            "games_in_search_per_step": tl["search_games_per_step"] / max(1, prof["rounds"])}
        stream.synchronize()
    finally:
        if stream is not caller:
            stream.synchronize()
            torch.cuda.set_stream(caller)
        for j in jobs:  # (an exception left launches running: they still write the buffers)
            j["done"].synchronize()
        for e in engines:
            e.handle.set_done(None)
        for b in hb_done.values():
            b.close()
    dt = time.perf_counter() - t0
    prof["total_s"] = dt
    prof["host_s"] = dt - prof["setup_s"] - prof["advance_s"] - prof["mcts_s"] - prof["fast_s"] - prof["wait_s"]
    if prof["uncertified_heuristic"]:
        warnings.warn(f"run_games_batched: {prof['uncertified_heuristic']} HeuristicAgent draw(s) fell within 2^-40 "
                      "of a probability boundary (choice not certified equal to the reference's on every host)",
                      RuntimeWarning, stacklevel=2)
    prof["t_end"] = time.perf_counter()
    final = states_d.cpu().numpy().view(N.STATE_DTYPE).reshape(n)
    out = []
    gc_on = gc.isenabled()  # (the records are new objects only: no collection can free any)
    if gc_on:
        gc.disable()
    try:
        _device_records(out, idx, results, per_agent, final, seats, gseeds, run_config, run_id, dt, n)
    finally:
        if gc_on:
            gc.enable()
    return out


def _device_records(out, idx, results, per_agent, final, seats, gseeds, run_config, run_id, dt, n):
    """The per-game records of _run_games_device (arena_runner.py's record fields)."""
    used, moves_made = final["used"].astype(np.int64).tolist(), final["move_count"].tolist()
    for i, gi in enumerate(idx):
        r, turns, passes, truncated = results[i]
        scores = {p + 1: int(v) for p, v in enumerate(r["scores"].tolist())}
        winners = [p for p, sc in scores.items() if sc == max(scores.values())]
        pa = per_agent[i]
        for p in range(4):
            pa[seats[i][str(p + 1)]]["moves"] += float(bin(used[i][p]).count("1"))
        total_moves = max(sum(e["moves"] for e in pa.values()), 1.0)
        for e in pa.values():
            e["total_time_ms"] = dt / n * (e["moves"] / total_moves) * 1000.0
        _finish_stats(pa)
        out.append(_record(run_id=run_id, game_index=gi, game_seed=gseeds[i], run_config=run_config, seats=seats[i],
                           scores=scores, winner_ids=winners, is_tie=len(winners) > 1,
                           moves_made=int(moves_made[i]), turn_count=turns, passes=passes, invalid=0,
                           duration=dt / n, truncated=truncated, per_agent=pa, error=None))


@dataclass(frozen=True)
class ArenaOptions:
    """How run_games_batched drives the games (never what they play: every setting gives
    the same records).  Explicit arguments, so nothing in a caller's environment changes
    the pipeline; the one environment read is the BK_ARENA_CAPTURE diagnostics switch,
    the default of capture_dir.
    * device_driver: positions, tables and agent streams resident in HBM for the whole
      run (bk_arena_step); False: the round-3 host-staged rounds (bk_arena_advance).
    * pipeline: MCTS searches in flight on `search_streams` streams while the other games
      play on; False: one search at a time, waited for at once.
    * search_streams: 1..16.  16 is the most any test has validated (tests/
      test_gpu_config4_queues.py); round 4's BK_MCTS_ELOG failures came at 24.
    * job_games: at most this many searches per bk_mcts launch.
    * reserve_cus: search streams may not use this many CUs (bk_stream_create; slower).
    * high_priority: the per-step kernels on a high-priority stream.
    * serial_worker: host-staged driver's searches on the calling thread (profiling).
    * capture_dir: keep each search launch's inputs; save and replay a failed one.
    * handback: with pipeline, each search's move goes back to its game as soon as that
      search is done (bk_mcts_set_done result words in mapped host memory, agent state
      rows updated in place: BK_MCTS_STATE_ROWS), not when its launch's longest search
      (2.3x the mean at config 4) ends.  Off by default: measured slower -- the games'
      searches then overlap more and each runs ~4x longer (1,160 vs 1,219 games/s at
      1,024 games, profiles/r06/sweeps/r06ai).  Ignored with capture_dir."""
    device_driver: bool = True
    pipeline: bool = True
    handback: bool = False
    search_streams: int = 8
    job_games: int = 1_000_000
    reserve_cus: int = 0
    high_priority: bool = True
    serial_worker: bool = False
    capture_dir: Optional[str] = None

    def __post_init__(self):
        if not 1 <= int(self.search_streams) <= MAX_SEARCH_STREAMS:
            raise ValueError(f"search_streams must be in 1..{MAX_SEARCH_STREAMS}")
        if int(self.job_games) < 1 or int(self.reserve_cus) < 0:
            raise ValueError("job_games must be >= 1 and reserve_cus >= 0")


MAX_SEARCH_STREAMS = 16


def run_games_batched(run_config: RunConfig, game_indices: Sequence[int], *, run_id: str = "gpu",
                      device: int = 0, progress=None, options: Optional[ArenaOptions] = None,
                      **option_kw) -> List[Dict[str, Any]]:
    """Mixed seatings (Random / Heuristic / MCTS / FastMCTS, config 4) in lockstep batches:
    every game's random and heuristic turns run inside bk_arena_advance (one launch
    advances all games to their next search-seat turn, each seat drawing from its own
    agent stream), then all MCTS seats to move search in one bk_mcts launch
    (MCTSAgent.search_packed) and all FastMCTS seats in one bk_fastmcts launch
    (FastMCTSAgent.think_many), their moves are placed, and the loop repeats.  Records
    equal run_single_game's (arena_runner.py:578-777): same agents, seeds, streams and
    move order.  Per-move times are launch shares.  progress(round, games_left, profile),
    if given, is called at the start of every round.  options (or the same fields as
    keywords, e.g. search_streams=4): ArenaOptions."""
    from .. import _native as N
    from ..engine.move_generator import frontier_ranks, order_moves, order_moves_many
    from ..engine.pieces import ORIENT_CELLS, ORIENT_LIST
    from ..gpu import BlokusGPU, empty_state
    idx = list(game_indices)
    n = len(idx)
    if n == 0:
        return []
    cfgs = {a.name: a for a in run_config.agents}
    if options is None:
        option_kw.setdefault("capture_dir", os.environ.get("BK_ARENA_CAPTURE") or None)
        options = ArenaOptions(**option_kw)
    elif option_kw:
        raise TypeError("pass ArenaOptions or its fields as keywords, not both")
    if options.device_driver:
        t_in = time.perf_counter()
        seats_d, gseeds_d = [], []
        for gi in idx:
            gs = game_seed_from_run_seed(run_config.seed, gi)
            st = seat_assignment_for_game(run_config.agent_names, gi, gs, run_config.seat_policy)
            if not _batchable(run_config, st):
                raise ValueError(f"game {gi}: seating {st} cannot be batched; use run_single_game")
            seats_d.append(st)
            gseeds_d.append(gs)
        t_seats = time.perf_counter()
        gc0 = sum(g["collections"] for g in gc.get_stats())
        # no collections during the agent setup: over the caller's heap (torch, earlier
        # records) they cost ~0.02 s per 1,024 games and free nothing the setup made
        # (profiles/r05/sweeps/r05an)
        gc_on = gc.isenabled()
        if gc_on:
            gc.disable()
        try:
            ag = _device_agents(run_config, seats_d, idx)
        finally:
            if gc_on:
                gc.enable()
        if ag is not None:
            agents_s = time.perf_counter() - t_in
            setup_gc = sum(g["collections"] for g in gc.get_stats()) - gc0
            out = _run_games_device(run_config, idx, seats_d, gseeds_d, ag, run_id=run_id, device=device,
                                    progress=progress, opts=options)
            # host time around the device loop: seats + agents before it, records after it
            LAST_BATCH_PROFILE.update(agents_s=agents_s, seats_s=t_seats - t_in, agents_gc=setup_gc,
                                      records_s=time.perf_counter() - LAST_BATCH_PROFILE["t_end"],
                                      call_s=time.perf_counter() - t_in)
            del LAST_BATCH_PROFILE["t_end"]
            return out
    gpu = BlokusGPU(device)
    t0 = time.perf_counter()
    states = np.repeat(empty_state(), n)
    sets = N.fset_new(n)
    masks = np.zeros(n, np.uint8)
    rng = np.zeros((n, 16), np.uint32)
    seats, gseeds, agents, per_agent = [], [], [], []
    for i, gi in enumerate(idx):
        gs = game_seed_from_run_seed(run_config.seed, gi)
        st = seat_assignment_for_game(run_config.agent_names, gi, gs, run_config.seat_policy)
        if not _batchable(run_config, st):
            raise ValueError(f"game {gi}: seating {st} cannot be batched; use run_single_game")
        seats.append(st)
        gseeds.append(gs)
        built = {}
        for p in range(4):
            name = st[str(p + 1)]
            c = cfgs[name]
            kind = c.type.lower()
            seed = agent_seed(run_config.seed, gi, name)
            if kind in ("random", "heuristic"):
                rng[i, 4 * p:4 * p + 4] = N.mt_cursors([seed])[0]
                if kind == "heuristic":
                    masks[i] |= 1 << p
            else:
                masks[i] |= 16 << p
                if name not in built:
                    built[name] = build_agent(c, seed)
        agents.append(built)
        per_agent.append({name: {"moves": 0.0, "total_time_ms": 0.0, "total_simulations": 0.0,
                                 "moves_with_simulations": 0.0, "move_times_ms": []} for name in set(st.values())})
    results: List[Optional[Dict[str, Any]]] = [None] * n
    active = np.arange(n)
    prof = LAST_BATCH_PROFILE
    prof.clear()
    # uncertified_heuristic: advance launches whose game had a HeuristicAgent draw within
    # 2^-40 of a cumulative-probability boundary (bk_result status bit 4), plus MCTS searches
    # with such a rollout draw (BK_MCTS_EUNCERT): the choice is the exact-arithmetic one,
    # but a host's rounding could pick the neighbour (HeuristicAgent)
    prof.update(setup_s=time.perf_counter() - t0, advance_s=0.0, mcts_s=0.0, fast_s=0.0, host_s=0.0, rounds=0,
                uncertified_heuristic=0)
    worker = _InlineWorker() if options.serial_worker else _mcts_worker()
    while len(active):
        prof["rounds"] += 1
        if progress is not None:
            progress(prof["rounds"], len(active), prof)
        ta = time.perf_counter()
        sub_st, sub_fs, sub_rng = states[active].copy(), sets[active].copy(), rng[active].copy()
        before = sub_st["reserved"].copy()
        res = gpu.arena_advance(sub_st, sub_fs, masks[active], sub_rng, max_turns=run_config.max_turns)
        prof["advance_s"] += time.perf_counter() - ta
        states[active], sets[active], rng[active] = sub_st, sub_fs, sub_rng
        stopped = []
        status = res["status"].astype(np.int64)
        prof["uncertified_heuristic"] += int(np.count_nonzero(status & N.STATUS_UNCERT))
        bad = status & ~(N.STATUS_CAP | N.STATUS_STOP | N.STATUS_UNCERT)
        if bad.any():
            j = int(np.flatnonzero(bad)[0])
            raise RuntimeError(f"game {idx[int(active[j])]}: kernel status {int(status[j])}")
        stop = (status & N.STATUS_STOP) != 0
        stopped = active[stop].tolist()
        # finished games (the rest): record results, turns and passes as whole arrays
        fin = np.flatnonzero(~stop)
        f_turns = (before[fin, 0].astype(np.int64) + res["turns"][fin].astype(np.int64)).tolist()
        f_passes = (before[fin, 1].astype(np.int64) + res["passes"][fin].astype(np.int64)).tolist()
        f_cap = ((status[fin] & N.STATUS_CAP) != 0).tolist()
        for j, turns, passes, cap in zip(fin.tolist(), f_turns, f_passes, f_cap):
            i = int(active[j])
            r = res[j]
            truncated = False
            if cap:  # cut by max_turns: over or not (arena_runner.py:702)
                if int(gpu.has_moves(states[i:i + 1])[0]) != 0:
                    truncated = True
                else:
                    turns -= int(r["reserved"][0])
                    passes -= int(r["reserved"][0])
            results[i] = (r.copy(), turns, passes, truncated)
        if stopped:
            stopped = np.array(stopped)
            pl = (states["current_player"][stopped] & 3).astype(np.uint8)
            cnt, rows = gpu.movegen(states[stopped], pl)
            chosen: Dict[int, Optional[int]] = {}
            mcts_job = None
            by_kind: Dict[str, List[Tuple[int, Any, int, list]]] = {"mcts": [], "fast": []}
            fast_k = []
            for k, i in enumerate(stopped):
                p = int(pl[k])
                adapter = agents[i][seats[i][str(p + 1)]]
                kind = "mcts" if isinstance(getattr(adapter, "agent", None), MCTSAgent) else "fast"
                if kind == "mcts":  # the search needs the count only (and the move if it is the only one)
                    if int(cnt[k]) == 1:
                        g, rr, cc = order_moves(rows[k], None)
                        legal = [int(g[0]) * 400 + int(rr[0]) * 20 + int(cc[0])]
                    else:
                        legal = [None] * int(cnt[k])
                else:  # FastMCTS: the reference's list order (frontier sets), ordered below at once
                    fast_k.append(k)
                    legal = None
                by_kind[kind].append((i, adapter, p, legal))
            if fast_k:
                fk = np.array(fast_k)
                ordered = iter(order_moves_many(rows[fk], ranks=frontier_ranks(sets[stopped[fk]], pl[fk])))
                by_kind["fast"] = [(i, a, p, next(ordered)) for i, a, p, _ in by_kind["fast"]]
            if by_kind["mcts"]:
                todo = [(i, a, p, lg) for i, a, p, lg in by_kind["mcts"] if len(lg) > 1]
                for i, a, p, lg in by_kind["mcts"]:
                    if len(lg) == 1:
                        chosen[i] = lg[0]
                        # select_action returns the only move without a search (mcts_agent.py
                        # :319-320), and the arena reads the agent's stats as they are: the
                        # previous search's iterations_run (0 before any) counts again
                        e = per_agent[i][seats[i][str(p + 1)]]
                        e["total_simulations"] += a.agent.stats["iterations_run"]
                        e["moves_with_simulations"] += 1
                if todo:
                    # the MCTS searches run on a worker thread (its own engine and stream)
                    # while this thread prepares and launches the FastMCTS seats; the two
                    # sets of games are disjoint and nothing below reads them until joined
                    ti = np.array([t[0] for t in todo])
                    mcts_job = (todo, worker.submit(_timed_search, [t[1].agent for t in todo], states[ti], sets[ti],
                                                    [t[2] for t in todo]))
            if by_kind["fast"]:
                ags, lists, iters = [], [], []
                for i, a, p, lg in by_kind["fast"]:
                    fa = a.agent if isinstance(a, _FastMCTSAdapter) else a.agent._agent
                    budget = (int(cfgs[seats[i][str(p + 1)]].thinking_time_ms or max(int(fa.time_limit * 1000), 1))
                              if isinstance(a, _FastMCTSAdapter)
                              else int(cfgs[seats[i][str(p + 1)]].thinking_time_ms or 1))
                    if not a.deterministic_time_budget:
                        raise ValueError("run_games_batched: FastMCTS seats need deterministic_time_budget")
                    ags.append(fa)
                    lists.append(lg)
                    iters.append(max(1, int(round(a.iterations_per_ms * budget))))
                tf = time.perf_counter()
                picks = FastMCTSAgent.think_arrays(ags, lists, iters)
                prof["fast_s"] += time.perf_counter() - tf
                for (i, a, p, lg), j, it in zip(by_kind["fast"], picks, iters):
                    g, rr, cc = lg
                    chosen[i] = int(g[j]) * 400 + int(rr[j]) * 20 + int(cc[j]) if j >= 0 else None
                    e = per_agent[i][seats[i][str(p + 1)]]
                    if len(g) > 1:
                        e["total_simulations"] += it
                        e["moves_with_simulations"] += 1
            if mcts_job is not None:
                todo, fut = mcts_job
                tw = time.perf_counter()
                mv, dt_m = fut.result()
                prof["mcts_s"] += dt_m  # the searches' own time (overlaps the FastMCTS phase)
                prof["mcts_wait_s"] = prof.get("mcts_wait_s", 0.0) + time.perf_counter() - tw
                prof["uncertified_heuristic"] += sum(int(t[1].agent.stats.get("last_search_uncertified", False))
                                                     for t in todo)
                for (i, a, p, lg), m in zip(todo, mv):
                    chosen[i] = m
                    e = per_agent[i][seats[i][str(p + 1)]]
                    e["total_simulations"] += a.agent.stats["iterations_run"]
                    e["moves_with_simulations"] += 1
            # place the search moves (Board.place_piece, engine/board.py:515-555), all games
            # of the round at once; the frontier tables per game (CPython set order)
            th = time.perf_counter()
            sp = (states["current_player"][stopped] & 3).astype(np.int64)
            mv = np.array([-1 if chosen.get(i) is None else int(chosen[i]) for i in stopped], np.int64)
            states["reserved"][stopped, 0] += 1  # turn_count
            passed = mv < 0  # agent returned no move: the reference passes (arena_runner.py:683-687)
            states["reserved"][stopped[passed], 1] += 1
            pm, pp, mm = stopped[~passed], sp[~passed], mv[~passed]
            if len(pm):
                masks_, pieces_ = _move_tables()
                states["planes"][pm, pp, :] |= masks_[mm]
                states["used"][pm, pp] |= (np.uint32(1) << pieces_[mm // 400].astype(np.uint32))
                states["first_move"][pm] &= (~(np.uint8(1) << pp.astype(np.uint8))).astype(np.uint8)
                states["move_count"][pm] += 1
                for i, p, m in zip(pm.tolist(), pp.tolist(), mm.tolist()):
                    g, a = divmod(m, 400)
                    N.fset_place(sets[i:i + 1], states[i:i + 1], p,
                                 [(a // 20 + dr) * 20 + a % 20 + dc for dr, dc in ORIENT_CELLS[g]])
            states["current_player"][stopped] = ((sp + 1) & 3).astype(np.uint8)
            prof["place_s"] = prof.get("place_s", 0.0) + time.perf_counter() - th
        active = np.array([i for i in active if results[i] is None], dtype=np.int64)
    dt = time.perf_counter() - t0
    prof["total_s"] = dt
    # the MCTS searches run on the worker thread while this thread runs the FastMCTS phase:
    # this thread's timeline is setup, advance, FastMCTS, the wait for the searches
    # (mcts_wait_s) and host work (host_s, everything else); mcts_s is the searches' own
    # time, overlapping the FastMCTS phase, and is not subtracted
    prof["host_s"] = (dt - prof["setup_s"] - prof["advance_s"] - prof["fast_s"] - prof.get("mcts_wait_s", 0.0))
    if prof["uncertified_heuristic"]:
        warnings.warn(f"run_games_batched: {prof['uncertified_heuristic']} HeuristicAgent draw(s) fell within 2^-40 "
                      "of a probability boundary (choice not certified equal to the reference's on every host)",
                      RuntimeWarning, stacklevel=2)
    out = []
    for i, gi in enumerate(idx):
        r, turns, passes, truncated = results[i]
        scores = {p + 1: int(r["scores"][p]) for p in range(4)}
        winners = [p for p, sc in scores.items() if sc == max(scores.values())]
        pa = per_agent[i]
        for p in range(4):
            pa[seats[i][str(p + 1)]]["moves"] += float(bin(int(states["used"][i, p])).count("1"))
        total_moves = max(sum(e["moves"] for e in pa.values()), 1.0)
        for e in pa.values():
            e["total_time_ms"] = dt / n * (e["moves"] / total_moves) * 1000.0
        _finish_stats(pa)
        out.append(_record(run_id=run_id, game_index=gi, game_seed=gseeds[i], run_config=run_config, seats=seats[i],
                           scores=scores, winner_ids=winners, is_tie=len(winners) > 1,
                           moves_made=int(states["move_count"][i]), turn_count=turns, passes=passes, invalid=0,
                           duration=dt / n, truncated=truncated, per_agent=pa, error=None))
    return out


def _write_json(path: Path, payload: Mapping[str, Any]) -> None:
    with path.open("w", encoding="utf-8") as fh:
        json.dump(payload, fh, indent=2, sort_keys=True)
        fh.write("\n")


def run_experiment(run_config: RunConfig, *, verbose: bool = False, device: int = 0, rank: int = 0,
                   world: int = 1, dist=None, batched: bool = True) -> Dict[str, Any]:
    """run_config.json + games.jsonl + summary.json (:914-996).  With ``world`` > 1 each
    rank plays games index == rank (mod world) on its GPU and rank 0 gathers the records
    and writes the run (one gather of JSON records, games are independent)."""
    from ..shard import shard_indices
    mine = shard_indices(run_config.num_games, rank, world).tolist()
    if _all_random(run_config):
        records = run_games_gpu(run_config, mine, run_id="pending", device=device)
    elif batched and all(_batchable(run_config, seat_assignment_for_game(
            run_config.agent_names, gi, game_seed_from_run_seed(run_config.seed, gi), run_config.seat_policy))
            for gi in mine):
        records = run_games_batched(run_config, mine, run_id="pending", device=device)
    else:
        agent_configs = {a.name: a for a in run_config.agents}
        records = []
        for gi in mine:
            gs = game_seed_from_run_seed(run_config.seed, gi)
            seats = seat_assignment_for_game(run_config.agent_names, gi, gs, run_config.seat_policy)
            records.append(run_single_game(run_id="pending", game_index=gi, game_seed=gs, run_config=run_config,
                                           seat_assignment=seats, agent_configs=agent_configs))
            if verbose:
                print(f"[{gi + 1}/{run_config.num_games}] seed={gs} winners={records[-1]['winner_agents']}")
    if world > 1:
        gathered: List[Any] = [None] * world
        dist.all_gather_object(gathered, records)
        records = [r for part in gathered for r in part]
    records.sort(key=lambda r: r["game_index"])
    if rank != 0:
        return {"run_id": None, "games": len(records)}
    root = Path(run_config.output_root)
    root.mkdir(parents=True, exist_ok=True)
    stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
    import hashlib
    run_id = f"{stamp}_{hashlib.sha256(json.dumps(run_config.to_dict(), sort_keys=True).encode()).hexdigest()[:8]}"
    run_dir = root / run_id
    k = 1
    while run_dir.exists():
        run_dir = root / f"{run_id}_{k:02d}"
        k += 1
    run_id = run_dir.name
    run_dir.mkdir(parents=True)
    payload = run_config.to_dict()
    payload.update(run_id=run_id, created_at=datetime.now().isoformat(timespec="seconds"))
    _write_json(run_dir / "run_config.json", payload)
    with (run_dir / "games.jsonl").open("w", encoding="utf-8") as fh:
        for r in records:
            r["run_id"] = run_id
            r["game_id"] = f"{run_id}_g{r['game_index']:04d}"
            fh.write(json.dumps(r, sort_keys=True) + "\n")
    summary = compute_summary(records, run_id=run_id, run_seed=run_config.seed, seat_policy=run_config.seat_policy,
                              agent_names=run_config.agent_names,
                              thinking_time_ms_by_agent={a.name: a.thinking_time_ms for a in run_config.agents},
                              run_config=payload)
    _write_json(run_dir / "summary.json", summary)
    return {"run_id": run_id, "run_dir": str(run_dir), "summary": summary}
