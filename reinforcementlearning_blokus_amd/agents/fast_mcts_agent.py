"""FastMCTSAgent with the simulate loop on the GPU (reference: agents/fast_mcts_agent.py).

The reference's search (fast_mcts_agent.py:153-256) is a bandit over the root's legal
moves: expansion pops the last untried move (:62), children never get untried moves of
their own, so after the root is fully expanded every iteration picks the UCB1-best root
child (:45-56).  The rollout (:243-267) looks up the root's cached legal list, so its
reward is one deterministic number per search (``_quick_move_evaluation``'s move: piece
size + centre bonus) plus ``self.rng.random() * 0.1``.

Here the per-iteration loop runs inside the HIP kernel ``bk_fastmcts`` -- one wave per
root, visit/reward arrays in LDS, CPython's Mersenne Twister (``random.Random``) and
its 53-bit ``random()`` reproduced on the device from ``self.rng.getstate()``, and the
advanced state handed back with ``setstate``.  The host only does what the reference
does once per think() call (cache lookup, quick evaluation, result dicts), so for the
same seed and iteration count the chosen move, visits and Q values are the
reference's (pinned by tests/golden/fastmcts.json).

Differences, by design:
* Iteration count.  The reference stops at ``self.iterations`` or the wall-clock
  budget, whichever comes first.  The kernel runs a fixed count: ``self.iterations``,
  capped to what the measured kernel rate fits in the budget.  With a generous budget
  the count is exactly ``self.iterations`` and results are deterministic.
* ``think_batch`` searches many roots in one launch (one wave per root).
"""
from __future__ import annotations

import math
import random
import time
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from ..engine.board import Board, Player
from ..engine.move_generator import Move, get_shared_generator
from ..gpu import BlokusGPU

_MT_WORDS = 625
_MAX_CHILDREN = 2048


def compute_policy_entropy(visits: List[int]) -> float:
    """Shannon entropy of the visit distribution (fast_mcts_agent.py:15-25)."""
    total = sum(visits)
    if total <= 0:
        return 0.0
    entropy = 0.0
    for v in visits:
        if v > 0:
            p = v / total
            entropy -= p * math.log(p)
    return entropy


_LOG_TABLE = np.zeros(1, dtype=np.float64)


def _log_table(n: int) -> np.ndarray:
    """math.log(k) for k < n (k = 0 is never read).  CPython's own values, so the UCB
    term matches the reference bit for bit."""
    global _LOG_TABLE
    if len(_LOG_TABLE) < n:
        m = max(n, 2 * len(_LOG_TABLE))
        _LOG_TABLE = np.array([0.0] + [math.log(k) for k in range(1, m)], dtype=np.float64)
    return _LOG_TABLE


def _advance_words(words: np.ndarray, n_words: int) -> np.ndarray:
    """State (625 words: key + position) after drawing n_words 32-bit outputs.  numpy's
    MT19937 runs the same recurrence as CPython's random module."""
    if n_words == 0:
        return words.copy()
    bg = np.random.MT19937()
    bg.state = {"bit_generator": "MT19937", "state": {"key": words[:624].copy(), "pos": int(words[624])}}
    full, rest = divmod(n_words, 1 << 20)
    for _ in range(full):
        bg.random_raw(1 << 20)
    if rest:
        bg.random_raw(rest)
    st = bg.state["state"]
    out = np.empty(_MT_WORDS, dtype=np.uint32)
    out[:624] = st["key"]
    out[624] = st["pos"]
    return out


def _move_dict(m: Move, visits: int, q: float) -> Dict[str, Any]:
    return {"piece_id": m.piece_id, "orientation": m.orientation, "anchor_row": m.anchor_row,
            "anchor_col": m.anchor_col, "visits": int(visits), "q_value": round(float(q), 4)}


class FastMCTSAgent:
    """GPU-backed drop-in for agents/fast_mcts_agent.py:75 FastMCTSAgent."""

    # kernel time model used to fit the iteration count into a wall-clock budget
    _US_PER_ITER_INIT = 2.0

    def __init__(self, iterations: int = 30, time_limit: float = 0.5, exploration_constant: float = 1.414,
                 seed: Optional[int] = None, enable_diagnostics: bool = False,
                 diagnostics_sample_interval: int = 100, device: int = 0):
        self.iterations = iterations
        self.time_limit = time_limit
        self.exploration_constant = exploration_constant
        self.rng = random.Random(seed)
        self.move_generator = get_shared_generator()
        self.enable_diagnostics = enable_diagnostics
        self.diagnostics_sample_interval = diagnostics_sample_interval
        self.device = device
        self._legal_moves_cache: Dict[str, List[Move]] = {}
        self._gpu = None
        self._us_per_iter = self._US_PER_ITER_INIT

    # ------------------------------------------------------------------ engine
    def _engine(self):
        if self._gpu is None:
            from ..gpu import BlokusGPU
            self._gpu = BlokusGPU(self.device)
        return self._gpu

    def _rng_words(self) -> np.ndarray:
        version, words, _gauss = self.rng.getstate()
        if version != 3 or len(words) != _MT_WORDS:
            raise RuntimeError("unexpected random.Random state layout")
        return np.array(words, dtype=np.uint32)

    def _set_rng_words(self, words: np.ndarray) -> None:
        self.rng.setstate((3, tuple(np.asarray(words, dtype=np.uint32).tolist()), None))

    # ------------------------------------------------------------------ reference helpers
    def _get_cached_legal_moves(self, board: Board, player: Player) -> List[Move]:
        """Keyed by player and move count only, as the reference (:307-315) -- stale
        across different boards with equal move counts, exactly like it."""
        key = f"{player.name}_{board.move_count}"
        if key not in self._legal_moves_cache:
            self._legal_moves_cache[key] = self.move_generator.get_legal_moves(board, player)
        return self._legal_moves_cache[key]

    def _quick_move_evaluation(self, legal_moves: List[Move]) -> Optional[Move]:
        """Largest three piece ids, then nearest the centre (:283-296); stable sorts."""
        if not legal_moves:
            return None
        by_size = sorted(legal_moves, key=lambda m: m.piece_id, reverse=True)
        top = by_size[:min(3, len(by_size))]
        centre = sorted(top, key=lambda m: abs(m.anchor_row - 9.5) + abs(m.anchor_col - 9.5))
        return centre[0] if centre else legal_moves[0]

    def _quick_heuristic_selection(self, board: Board, player: Player, legal_moves: List[Move]) -> Move:
        return self._quick_move_evaluation(legal_moves) or legal_moves[0]

    def _base_reward(self, board: Board, player: Player) -> float:
        """Deterministic part of _fast_rollout (:243-267); NaN = empty cached list
        (reward 0.0, no random draw)."""
        legal = self._get_cached_legal_moves(board, player)
        if not legal:
            return math.nan
        move = self._quick_move_evaluation(legal)
        if move is None:
            return math.nan
        reward = move.piece_id * 0.1
        center_distance = abs(move.anchor_row - 9.5) + abs(move.anchor_col - 9.5)
        reward += (20 - center_distance) * 0.05
        return reward

    # ------------------------------------------------------------------ search
    def select_action(self, board: Board, player: Player, legal_moves: List[Move]) -> Optional[Move]:
        return self.think(board, player, legal_moves, int(self.time_limit * 1000))["move"]

    def _iteration_cap(self, budget_s: float, n_roots: int) -> int:
        """self.iterations, or fewer if the measured kernel rate says the budget is too
        short for them (the reference's wall-clock stop, :153)."""
        fit = int(budget_s * 1e6 / max(self._us_per_iter, 1e-3))
        return max(1, min(self.iterations, fit))

    def think(self, board: Board, player: Player, legal_moves: List[Move], time_budget_ms: int) -> Dict[str, Any]:
        """Search one root; same result dict as the reference (:112-231)."""
        return self.think_batch([board], [player], [legal_moves], time_budget_ms)[0]

    def think_batch(self, boards: Sequence[Board], players: Sequence[Player],
                    legal_lists: Sequence[List[Move]], time_budget_ms: int) -> List[Dict[str, Any]]:
        """Search several roots in one kernel launch.  Roots draw from this agent's
        random stream one after another, in list order, as sequential think() calls
        would."""
        start = time.perf_counter()
        budget_s = max(time_budget_ms, 1) / 1000.0
        results: List[Optional[Dict[str, Any]]] = [None] * len(boards)
        todo = []
        for i, (board, player, legal) in enumerate(zip(boards, players, legal_lists)):
            if not legal:
                results[i] = {"move": None, "stats": {"timeBudgetMs": time_budget_ms, "timeSpentMs": 0,
                                                      "nodesEvaluated": 0, "maxDepthReached": 0, "topMoves": []}}
            elif len(legal) == 1:
                m = legal[0]
                results[i] = {"move": m, "stats": {
                    "timeBudgetMs": time_budget_ms, "timeSpentMs": int((time.perf_counter() - start) * 1000),
                    "nodesEvaluated": 1, "maxDepthReached": 1, "topMoves": [_move_dict(m, 1, 0.0)]}}
            else:
                if len(legal) > _MAX_CHILDREN:
                    raise ValueError(f"{len(legal)} legal moves exceed the kernel's {_MAX_CHILDREN}")
                todo.append(i)
        if not todo:
            return results  # type: ignore[return-value]
        iters = self._iteration_cap(budget_s, len(todo))
        if self.enable_diagnostics:
            for i in todo:
                results[i] = self._search_diag(boards[i], players[i], legal_lists[i], iters, time_budget_ms, start)
            return results  # type: ignore[return-value]
        # One launch for all roots.  Sequential think() calls would draw from one
        # random stream, root after root; each search of `iters` iterations takes
        # exactly `iters` random() calls (none with an empty cached list), so every
        # root's starting state is the previous one advanced by 2*iters words.
        bases = [self._base_reward(boards[i], players[i]) for i in todo]
        mt = np.empty((len(todo), _MT_WORDS), dtype=np.uint32)
        mt[0] = self._rng_words()
        for k in range(1, len(todo)):
            mt[k] = _advance_words(mt[k - 1], 0 if math.isnan(bases[k - 1]) else 2 * iters)
        out = self._launch([len(legal_lists[i]) for i in todo], [iters] * len(todo), bases, mt,
                           exact_ucb=iters >= self.iterations)
        self._set_rng_words(mt[-1])
        for k, i in enumerate(todo):
            results[i] = self._finish(out[k], boards[i], players[i], legal_lists[i], time_budget_ms, start)
        return results  # type: ignore[return-value]

    @staticmethod
    def think_many(agents: Sequence["FastMCTSAgent"], players: Sequence[Player], legal_lists: Sequence[List[Move]],
                   move_counts: Sequence[int], iterations: Sequence[int]) -> List[Optional[Move]]:
        """think(board, player, legal, budget >= 10^7 ms) of several agents, each on its
        own root, in ONE bk_fastmcts launch: agent k runs iterations[k] iterations from its
        own random stream, exactly as its think() would (the arena's deterministic budget,
        arena_runner.py:352-369).  move_counts[k] = board.move_count (key of the
        reference's cached legal list, :304-312).  Returns each agent's move."""
        assert len({id(a) for a in agents}) == len(agents), "one search per agent per launch"
        moves: List[Optional[Move]] = [None] * len(agents)
        todo = []
        for k, (a, p, legal) in enumerate(zip(agents, players, legal_lists)):
            if len(legal) == 1:
                moves[k] = legal[0]
            elif len(legal) > 1:
                if len(legal) > _MAX_CHILDREN:
                    raise ValueError(f"{len(legal)} legal moves exceed the kernel's {_MAX_CHILDREN}")
                todo.append(k)
        if not todo:
            return moves
        bases = []
        for k in todo:
            a, p, legal = agents[k], players[k], legal_lists[k]
            cache = a._legal_moves_cache.setdefault(f"{p.name}_{int(move_counts[k])}", legal)
            q = a._quick_move_evaluation(cache) if cache else None
            bases.append(math.nan if q is None else
                         q.piece_id * 0.1 + (20 - (abs(q.anchor_row - 9.5) + abs(q.anchor_col - 9.5))) * 0.05)
        base_of = dict(zip(todo, bases))
        groups: Dict[float, List[int]] = {}  # one launch per exploration constant
        for k in todo:
            groups.setdefault(float(agents[k].exploration_constant), []).append(k)
        for c, ks in groups.items():
            mt = np.stack([agents[k]._rng_words() for k in ks])
            counts = [max(1, int(iterations[k])) for k in ks]
            eng = BlokusGPU.shared(agents[ks[0]].device)  # one handle for all batched launches
            out = eng.fastmcts([len(legal_lists[k]) for k in ks], counts, [base_of[k] for k in ks],
                               mt, _log_table(max(counts) + 1), c)
            for j, k in enumerate(ks):
                agents[k]._set_rng_words(mt[j])
                res, legal = out[j], legal_lists[k]
                if int(res["iterations"]) < 5:
                    moves[k] = agents[k]._quick_heuristic_selection(None, players[k], legal)
                else:
                    moves[k] = legal[int(res["best_index"])] if int(res["n_children"]) > 0 else legal[0]
        return moves

    @staticmethod
    def think_arrays(agents: Sequence["FastMCTSAgent"], legal_arrays, iterations: Sequence[int]) -> List[int]:
        """think_many on legal lists given as arrays: legal_arrays[k] = (g, r, c) int arrays
        in the reference's list order (order_moves), no Move objects.  For callers whose
        agents never see one (player, move_count) twice (one agent per game, as in the
        arena), where the reference's cached legal list is always the current one.
        Returns the index of each agent's move in its list (-1: no legal move)."""
        from ..engine.pieces import ORIENT_LIST
        pid_of = np.array([p for p, _ in ORIENT_LIST], dtype=np.int64)
        out = [-1] * len(agents)
        todo, bases = [], []
        for k, (g, r, c) in enumerate(legal_arrays):
            n = len(g)
            if n == 1:
                out[k] = 0
            elif n > 1:
                if n > _MAX_CHILDREN:
                    raise ValueError(f"{n} legal moves exceed the kernel's {_MAX_CHILDREN}")
                todo.append(k)
                # _quick_move_evaluation (:283-296): stable sort by piece id desc, top 3,
                # stable sort by centre distance
                top = np.argsort(-pid_of[g], kind="stable")[:3]
                dist = [abs(int(r[j]) - 9.5) + abs(int(c[j]) - 9.5) for j in top]
                q = int(top[min(range(len(top)), key=lambda t: dist[t])])
                reward = int(pid_of[g[q]]) * 0.1
                reward += (20 - (abs(int(r[q]) - 9.5) + abs(int(c[q]) - 9.5))) * 0.05
                bases.append(reward)
        groups: Dict[float, List[int]] = {}
        for k in todo:
            groups.setdefault(float(agents[k].exploration_constant), []).append(k)
        base_of = dict(zip(todo, bases))
        for ce, ks in groups.items():
            mt = np.stack([agents[k]._rng_words() for k in ks])
            counts = [max(1, int(iterations[k])) for k in ks]
            eng = BlokusGPU.shared(agents[ks[0]].device)  # one handle for all batched launches
            res = eng.fastmcts([len(legal_arrays[k][0]) for k in ks], counts, [base_of[k] for k in ks], mt,
                               _log_table(max(counts) + 1), ce)
            for j, k in enumerate(ks):
                agents[k]._set_rng_words(mt[j])
                g, r, c = legal_arrays[k]
                if int(res[j]["iterations"]) < 5:  # _quick_heuristic_selection
                    top = np.argsort(-pid_of[g], kind="stable")[:3]
                    dist = [abs(int(r[t]) - 9.5) + abs(int(c[t]) - 9.5) for t in top]
                    out[k] = int(top[min(range(len(top)), key=lambda t: dist[t])])
                else:
                    out[k] = int(res[j]["best_index"]) if int(res[j]["n_children"]) > 0 else 0
        return out

    def _launch(self, n_legal, counts, bases, mt, want_visits=False, exact_ucb=True):
        # exact_ucb=False: the time budget cut the iteration count (a wall-clock search,
        # not reproducible by the reference either), so do not stall on building pow
        # corrections for it (gpu.fastmcts)
        t0 = time.perf_counter()
        r = self._engine().fastmcts(n_legal, counts, bases, mt, _log_table(max(counts) + 1),
                                    self.exploration_constant, want_visits=want_visits, exact_ucb=exact_ucb)
        work = max(counts)  # roots run side by side, one wave each
        if work >= 64:
            self._us_per_iter = 0.5 * self._us_per_iter + 0.5 * (time.perf_counter() - t0) * 1e6 / work
        return r

    def _finish(self, res, board: Board, player: Player, legal: List[Move], time_budget_ms: int,
                start: float, diag_max_depth: Optional[int] = None) -> Dict[str, Any]:
        iteration = int(res["iterations"])
        top = [_move_dict(legal[int(res["top_index"][t])], res["top_visits"][t], res["top_q"][t])
               for t in range(int(res["n_top"]))]
        spent = int((time.perf_counter() - start) * 1000)
        if iteration < 5:
            return {"move": self._quick_heuristic_selection(board, player, legal),
                    "stats": {"timeBudgetMs": time_budget_ms, "timeSpentMs": spent,
                              "nodesEvaluated": max(iteration, 1), "maxDepthReached": 2, "topMoves": top}}
        best = legal[int(res["best_index"])] if int(res["n_children"]) > 0 else None
        stats = {"timeBudgetMs": time_budget_ms, "timeSpentMs": spent, "nodesEvaluated": max(iteration, 1),
                 "maxDepthReached": diag_max_depth if diag_max_depth is not None else 2, "topMoves": top,
                 "diagnostics": None}
        return {"move": best if best else legal[0], "stats": stats}

    def _search_diag(self, board: Board, player: Player, legal: List[Move], iters: int, time_budget_ms: int,
                     start: float) -> Dict[str, Any]:
        """think() with enable_diagnostics (:160-231).  The bandit is deterministic
        given (random state, iteration count), so each in-loop sample of the reference
        (after iteration+1 iterations, iteration % interval == 0, iteration > 0) is one
        more root in the same launch with the shorter count."""
        base = self._base_reward(board, player)
        interval = max(int(self.diagnostics_sample_interval), 1)
        sample_at = list(range(interval, iters, interval))
        counts = [iters] + [s + 1 for s in sample_at]
        n_legal = len(legal)
        mt = np.repeat(self._rng_words()[None, :], len(counts), axis=0)
        out, vis = self._launch([n_legal] * len(counts), counts, [base] * len(counts), mt, want_visits=True)
        self._set_rng_words(mt[0])
        res = out[0]
        n_children = int(res["n_children"])
        depth = 1 if n_children else 0
        result = self._finish(res, board, player, legal, time_budget_ms, start, diag_max_depth=depth)
        if int(res["iterations"]) < 5:
            return result

        def child_visits(k: int, nch: int) -> List[int]:
            # child j was expanded from legal[n_legal - 1 - j] (untried_moves.pop())
            return [int(x) for x in vis[k * n_legal:(k + 1) * n_legal][::-1][:nch]]

        trace = []
        for k, s in enumerate(sample_at, start=1):
            r = out[k]
            if int(r["n_top"]) == 0:
                continue
            bm = legal[int(r["top_index"][0])]
            trace.append({"sim": s, "bestActionId": f"{bm.piece_id}-{bm.orientation}-{bm.anchor_row}-{bm.anchor_col}",
                          "bestQMean": float(r["top_q"][0]),
                          "entropy": float(compute_policy_entropy(child_visits(k, int(r["n_children"]))))})
        stats = result["stats"]
        sims = max(int(res["iterations"]), 1)
        spent = stats["timeSpentMs"]
        stats["diagnostics"] = {
            "version": "v1", "timeBudgetMs": int(time_budget_ms), "timeSpentMs": int(spent), "simulations": sims,
            "simsPerSec": int(sims / (spent / 1000.0)) if spent > 0 else 0,
            "rootLegalMoves": n_legal, "rootChildrenExpanded": n_children, "rootPolicy": stats["topMoves"],
            "policyEntropy": float(compute_policy_entropy(child_visits(0, n_children))),
            "maxDepthReached": depth, "nodesExpanded": n_children,
            "nodesByDepth": [{"depth": 0, "nodes": 1}] + ([{"depth": 1, "nodes": n_children}] if n_children else []),
            "bestMoveTrace": trace}
        return result

    def get_action_info(self) -> Dict[str, Any]:
        return {"name": "FastMCTSAgent", "type": "mcts",
                "description": "FastMCTS with the simulate loop in a HIP kernel",
                "parameters": {"iterations": self.iterations, "time_limit": self.time_limit,
                               "exploration_constant": self.exploration_constant}}

    def reset(self):
        self._legal_moves_cache.clear()

    def set_seed(self, seed: int):
        self.rng = random.Random(seed)
