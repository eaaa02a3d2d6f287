"""UCT MCTS with GPU rollouts (reference: mcts/mcts_agent.py).

Tree policy, expansion (``untried_moves.pop()``: last legal move first), UCB1 with
numpy log/sqrt, best = most visited child (first on ties) and the Zobrist
transposition cache follow mcts/mcts_agent.py:19-191, :304-437, :572-582.

Rollouts (mcts/mcts_agent.py:470-554, <= max_rollout_moves plies, stop at the first
player without a move, reward = final - initial Board.get_score of the root player)
have three GPU backends:

* ``rollout_backend="search"`` (the default, for the reference's default HeuristicAgent
  rollout agent and for a RandomAgent): the WHOLE search -- selection, expansion, TT
  lookups, rollouts, backpropagation -- runs in one bk_mcts launch (k_mcts / k_mcts_h),
  bit-identical to the reference: frontier-order legal lists, the agent's numpy MT19937
  stream (read from and written back to ``rollout_agent.rng``), HeuristicAgent choices
  certified exact per draw, the Zobrist TT kept in device-layout tables across calls.
  ``search_batch`` runs many agents' searches in one launch.
* ``rollout_backend="exact"`` (a rollout_agent with ``select_action``): the tree and
  the ply loop run on the host, every legal-move list comes from the GPU in the
  reference's frontier order and the agent draws from its own stream -- bit-identical
  to the reference for RandomAgent, usable with any agent.
  Used for rollout agents the kernels do not implement (e.g. re-weighted heuristics).
* ``rollout_backend="kernel"`` (opt-in): the whole playout runs inside the persistent
  HIP rollout kernel (bk_rollout, BK_SEM_ROLLOUT, Philox stream, naive move order) with
  UNIFORM random moves: statistically a random playout, not the reference's numbers,
  and not its heuristic policy.
The learned-evaluator options of the reference are out of scope and rejected.
"""
from __future__ import annotations

import contextlib
import math
import time
import warnings
from typing import Any, Dict, List, Optional

import numpy as np

from ..engine.board import Board, Player, Position, _PLAYERS, pack_state
from ..engine.move_generator import Move, get_shared_generator, int_to_move
from ..engine.pieces import PieceGenerator
from .zobrist import TranspositionTable, ZobristHash


def _search_on_device(gpu, ags, rts, sts, pl, rh, zob, zidx, mt, iters, max_roll, c, use_tt, tl_us, policy):
    """One bk_mcts launch for search_packed with every buffer in HBM (BK_MEM_DEVICE).
    The agents' TTs stay on the device between calls (TTPool rows, gathered into the
    launch's [n, cap] block and scattered back); only the roots, streams and per-search
    outputs cross PCIe.  mt (uint32[n, 625]) is advanced in place.  Returns dict(out,
    rewards, hit_flags) as host arrays."""
    import torch

    from .. import _native as N
    from ..gpu import TT_LOCK, TTPool, mcts_log_table, mcts_node_cap
    n = len(ags)
    dev = f"cuda:{gpu.device}"
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    lts = gpu.__dict__.setdefault("_log_tables", {})
    if iters not in lts:
        lts[iters] = up(mcts_log_table(iters))
    cap_nodes = mcts_node_cap(iters)
    d_mt = up(mt.view(np.int32))
    d_out = torch.zeros((n, N.MCTS_OUT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    d_rew = torch.empty((n, iters), dtype=torch.float64, device=dev)
    d_flags = torch.empty((n, iters), dtype=torch.uint8, device=dev)
    tk = tv = tc = rows = pool = None
    # TT_LOCK from the rows' lease / gather to their scatter (synchronized by the count
    # copy): another thread's search or pool growth cannot interleave (gpu.TT_LOCK)
    with (TT_LOCK if use_tt else contextlib.nullcontext()):
        if use_tt:
            cap = max([a._gpu_tt.cap for a in ags if a._gpu_tt is not None] or [1 << 12])
            need = max([int(a._gpu_tt.count[0]) for a in ags if a._gpu_tt is not None] or [0]) + iters + 2
            while 2 * need > cap:
                cap *= 2
            pool = TTPool.get(gpu.device, cap)
            for a in ags:
                row = a._gpu_tt
                if row is None:
                    a._gpu_tt = pool.lease()
                elif row.pool is not pool:  # grown: re-insert into a row of the larger pool
                    nr = pool.lease()
                    nr.load(*row.items(0))
                    row.release()
                    a._gpu_tt = nr
            rows = torch.tensor([a._gpu_tt.row for a in ags], dtype=torch.int64, device=dev)
            tk, tv, tc = (pool.keys.index_select(0, rows), pool.vals.index_select(0, rows),
                          pool.count.index_select(0, rows))
        gpu.mcts_device(up(rts.view(np.uint8).reshape(n, 256)), up(sts.view(np.uint8).reshape(n, -1)), up(pl),
                        up(rh.view(np.int64)), up(zob.view(np.int64)), up(zidx), d_mt, lts[iters],
                        torch.empty((n, cap_nodes * N.MCTS_NODE_DTYPE.itemsize), dtype=torch.uint8, device=dev),
                        d_out, iterations=iters, tt_keys=tk, tt_vals=tv, tt_count=tc, rewards=d_rew,
                        hit_flags=d_flags, max_rollout_moves=max_roll, exploration=c, rollout_policy=policy,
                        time_limit_us=tl_us)
        if use_tt:
            pool.keys.index_copy_(0, rows, tk)
            pool.vals.index_copy_(0, rows, tv)
            pool.count.index_copy_(0, rows, tc)
            for a, cnt in zip(ags, tc.cpu().numpy()):  # synchronizes this stream
                a._gpu_tt.count[0] = cnt
    mt[:] = d_mt.cpu().numpy().view(np.uint32)
    out = d_out.cpu().numpy().view(N.MCTS_OUT_DTYPE).reshape(n)
    # only the iterations some search ran cross PCIe (a timed search's bound is far above)
    live = max(1, int(out["iterations_run"].max())) if n else 1
    return {"out": out, "rewards": d_rew[:, :live].cpu().numpy(), "hit_flags": d_flags[:, :live].cpu().numpy()}

_MT_VIEWS_OK: Optional[bool] = None


def _mt_view(rng) -> Optional[np.ndarray]:
    """uint32[625] view of a numpy RandomState's MT19937 key[624] + pos (the bit
    generator's C state), so search_packed moves 500 agents' rollout streams without 500
    get_state / set_state round trips (~50 us each); the Gaussian cache stays untouched,
    as set_state((.., key, pos, has_gauss, gauss)) with the old has_gauss leaves it.
    None if this numpy's layout does not match get_state (checked once)."""
    global _MT_VIEWS_OK
    import ctypes

    def view(r):
        addr = r._bit_generator.ctypes.state_address
        return np.ctypeslib.as_array(ctypes.cast(addr, ctypes.POINTER(ctypes.c_uint32)), shape=(625,))

    if _MT_VIEWS_OK is None:
        try:
            probe = np.random.RandomState(20260301)
            probe.random_sample(700)  # past a twist
            v, st = view(probe), probe.get_state()
            ok = np.array_equal(v[:624], st[1]) and int(v[624]) == st[2]
            v[:624] = np.arange(624, dtype=np.uint32)
            v[624] = 7
            st = probe.get_state()
            _MT_VIEWS_OK = bool(ok and np.array_equal(st[1], np.arange(624)) and st[2] == 7)
        except Exception:  # noqa: BLE001 -- any other numpy: fall back to get_state
            _MT_VIEWS_OK = False
    if not _MT_VIEWS_OK or type(rng) is not np.random.RandomState:
        return None
    return view(rng)


def _search_policy(agent) -> Optional[int]:
    """bk_mcts rollout policy replaying this rollout agent on the GPU, or None:
    RandomAgent, or HeuristicAgent with the reference's default weights (the kernel's
    scoring constants, agents/heuristic_agent.py:33-37)."""
    from .. import _native as N
    from ..agents.heuristic_agent import HeuristicAgent
    from ..agents.random_agent import RandomAgent
    if isinstance(agent, RandomAgent):
        return N.MCTS_ROLLOUT_RANDOM
    if isinstance(agent, HeuristicAgent) and agent._weights() == (1.0, 2.0, -1.5, 0.5):
        return N.MCTS_ROLLOUT_HEURISTIC
    return None


def _positions(move: Move) -> List[Position]:
    shape = get_shared_generator().piece_orientations_cache[move.piece_id][move.orientation]
    return [Position(move.anchor_row + int(r), move.anchor_col + int(c)) for r, c in zip(*np.nonzero(shape))]


# search_packed's running totals (bench / arena profiling): launches, their kernel time
# (HIP events around bk_mcts), simulations and rollout plies, overall and per kernel
# (bk_mcts picks the kernel by batch size; "by_kernel": {name: the same four totals})
SEARCH_TOTALS: Dict[str, Any] = {"launches": 0, "kernel_ms": 0.0, "sims": 0, "rollout_plies": 0, "by_kernel": {}}


def reset_search_totals() -> None:
    SEARCH_TOTALS.update(launches=0, kernel_ms=0.0, sims=0, rollout_plies=0, by_kernel={})

# Timed searches (time_limit): iteration bound per second of limit, and overall.  One
# search runs ~100-1,000 iterations/s on the GPU (a lane of a persistent wave), so the
# bound is not reached in practice; if it is, stats say so and a warning is issued.
TIMED_MAX_ITERS_PER_S = 20000
TIMED_MAX_ITERS = 1 << 18


class MCTSNode:
    def __init__(self, board: Board, player: Player, move: Optional[Move] = None,
                 parent: Optional["MCTSNode"] = None):
        self.board = board.copy()
        self.player = player
        self.move = move
        self.parent = parent
        self.children: List["MCTSNode"] = []
        self.visits = 0
        self.total_reward = 0.0
        self.prior_bias = 0.0
        self.untried_moves: List[Move] = get_shared_generator().get_legal_moves(self.board, self.player)

    def is_fully_expanded(self) -> bool:
        return not self.untried_moves

    def is_terminal(self) -> bool:
        return not self.untried_moves and not self.children

    def ucb1_value(self, exploration_constant: float = 1.414, progressive_bias_weight: float = 0.0) -> float:
        if self.visits == 0:
            return float("inf")
        exploit = self.total_reward / self.visits
        explore = exploration_constant * np.sqrt(np.log(self.parent.visits) / self.visits)
        return exploit + explore + progressive_bias_weight * (self.prior_bias / (1.0 + self.visits))

    def select_child(self, exploration_constant: float = 1.414, progressive_bias_weight: float = 0.0) -> "MCTSNode":
        return max(self.children, key=lambda ch: ch.ucb1_value(exploration_constant, progressive_bias_weight))

    def expand(self) -> Optional["MCTSNode"]:
        if not self.untried_moves:
            return None
        move = self.untried_moves.pop()
        nb = self.board.copy()
        if not nb.place_piece(_positions(move), self.player, move.piece_id, validate=False):
            return None
        child = MCTSNode(nb, _PLAYERS[(_PLAYERS.index(self.player) + 1) % 4], move, self)
        self.children.append(child)
        return child

    def update(self, reward: float):
        self.visits += 1
        self.total_reward += reward

    def get_best_move(self) -> Optional[Move]:
        return max(self.children, key=lambda ch: ch.visits).move if self.children else None


class MCTSAgent:
    def __init__(self, iterations: int = 1000, time_limit: Optional[float] = None,
                 exploration_constant: float = 1.414, rollout_agent=None, use_transposition_table: bool = True,
                 seed: Optional[int] = None, learned_model_path: Optional[str] = None,
                 leaf_evaluation_enabled: bool = False, progressive_bias_enabled: bool = False,
                 progressive_bias_weight: float = 0.25, potential_shaping_enabled: bool = False,
                 potential_shaping_gamma: float = 1.0, potential_shaping_weight: float = 1.0,
                 potential_mode: str = "prob", max_rollout_moves: int = 50,
                 rollout_backend: Optional[str] = None, device: int = 0):
        if potential_mode not in {"prob", "logit"}:
            raise ValueError("potential_mode must be either 'prob' or 'logit'.")
        if int(max_rollout_moves) <= 0:
            raise ValueError("max_rollout_moves must be > 0.")
        if leaf_evaluation_enabled or progressive_bias_enabled or potential_shaping_enabled or learned_model_path:
            raise ValueError("learned evaluation is not supported by the GPU MCTS (out of scope)")
        self.iterations = iterations
        self.time_limit = time_limit
        self.exploration_constant = exploration_constant
        self.use_transposition_table = use_transposition_table
        self.max_rollout_moves = int(max_rollout_moves)
        self.progressive_bias_enabled = False
        self.progressive_bias_weight = float(progressive_bias_weight)
        self.move_generator = get_shared_generator()
        self.piece_generator = PieceGenerator()
        self.zobrist_hash = ZobristHash(seed=seed)
        from ..agents.heuristic_agent import HeuristicAgent
        from ..agents.random_agent import RandomAgent
        if rollout_agent is None and rollout_backend != "kernel":
            rollout_agent = HeuristicAgent(seed=seed)  # the reference's default policy
        self.rollout_agent = rollout_agent
        if rollout_backend is None:
            rollout_backend = "search" if _search_policy(rollout_agent) is not None else "exact"
        self.rollout_backend = rollout_backend
        if self.rollout_backend not in ("search", "exact", "kernel"):
            raise ValueError("rollout_backend must be 'search', 'exact' or 'kernel'")
        if self.rollout_backend == "exact" and rollout_agent is None:
            raise ValueError("rollout_backend='exact' needs a rollout_agent")
        if self.rollout_backend == "search" and _search_policy(rollout_agent) is None:
            raise ValueError("rollout_backend='search' needs a RandomAgent or a default-weight HeuristicAgent "
                             "rollout_agent (its numpy stream is replayed on the GPU)")
        self.seed = 0 if seed is None else int(seed)
        self._kernel_calls = 0
        self.device = device
        self._gpu = None
        self.transposition_table = TranspositionTable() if use_transposition_table else None
        self._gpu_tt = None  # "search" backend: the TT as a device-layout open-addressing table
        self.stats = self._fresh_stats()

    @staticmethod
    def _fresh_stats():
        return {"iterations_run": 0, "time_elapsed": 0.0, "transposition_hits": 0, "rollout_rewards": [],
                "uncertified_searches": 0, "last_search_uncertified": False,
                "leaf_eval_calls": 0, "progressive_bias_updates": 0, "potential_shaping_terms": [],
                "evaluator_errors": 0}

    def select_action(self, board: Board, player: Player, legal_moves: List[Move]) -> Optional[Move]:
        if not legal_moves:
            return None
        if len(legal_moves) == 1:
            return legal_moves[0]
        if self.rollout_backend == "search":
            return MCTSAgent.search_batch([self], [board], [player], [legal_moves])[0]
        t0 = time.time()
        root = MCTSNode(board, player)
        if self.time_limit:
            i = 0
            while time.time() - t0 < self.time_limit:
                self._mcts_iteration(root)
                i += 1
            self.stats["iterations_run"] = i
        else:
            for i in range(self.iterations):
                self._mcts_iteration(root)
                self.stats["iterations_run"] = i + 1
        self.stats["time_elapsed"] = time.time() - t0
        best = root.get_best_move()
        if self.transposition_table and len(self.transposition_table.table) > 500000:
            self.transposition_table.clear()
        return best

    @staticmethod
    def search_batch(agents: List["MCTSAgent"], boards: List[Board], players: List[Player],
                     legal_moves: Optional[List[List[Move]]] = None) -> List[Optional[Move]]:
        """select_action for several "search"-backend agents in ONE bk_mcts launch (one
        search per agent; an agent appears at most once).  Each result equals the
        agent's own select_action on that position: the search reads and advances the
        agent's rollout stream and TT, and updates its stats, exactly as the
        reference's select_action (mcts/mcts_agent.py:304-341) does.  Positions with
        < 2 legal moves are answered without a search (:313-318); ``legal_moves[i]`` is
        the caller's legal list for position i (generated here when omitted)."""
        assert len(agents) == len(boards) == len(players)
        gen = get_shared_generator()
        legal = [legal_moves[i] if legal_moves is not None else gen.get_legal_moves(b, p)
                 for i, (b, p) in enumerate(zip(boards, players))]
        todo = [i for i in range(len(agents)) if len(legal[i]) > 1]
        out: List[Optional[Move]] = [lm[0] if len(lm) == 1 else None for lm in legal]
        if todo:
            roots = np.concatenate([pack_state(boards[i]) for i in todo])
            sets = np.concatenate([boards[i].frontier_tables for i in todo])
            moves = MCTSAgent.search_packed([agents[i] for i in todo], roots, sets,
                                            [players[i].value - 1 for i in todo])
            for i, mv in zip(todo, moves):
                out[i] = int_to_move(mv) if mv is not None else None
        return out

    @staticmethod
    def search_packed(agents: List["MCTSAgent"], roots: np.ndarray, sets: np.ndarray, players) -> List[Optional[int]]:
        """The searches of search_batch on packed positions (STATE_DTYPE roots, their
        FSET_DTYPE frontier tables, players 0..3), each with >= 2 legal moves; one
        bk_mcts launch per parameter group.  Returns move ints (g * 400 + cell)."""
        from .. import _native as N
        from ..gpu import BlokusGPU
        from .zobrist import flat_keys, hash_states
        assert len({id(a) for a in agents}) == len(agents), "one search per agent per launch"
        out: List[Optional[int]] = [None] * len(agents)
        groups = {}  # agents sharing (iterations, rollout cap, c, TT on/off, time limit) share a launch
        for i, a in enumerate(agents):
            if a.rollout_backend != "search":
                raise ValueError("search_batch needs rollout_backend='search' agents")
            # time_limit (seconds, mcts_agent.py:325-333, :349-356): iterate until it runs
            # out, ignoring `iterations`, as _run_mcts_with_time_limit does.  The kernel stops
            # each search at the first iteration boundary past the limit; the launch still
            # needs an iteration bound to size the node pool / log table / reward buffers,
            # so a timed search gets time_limit x TIMED_MAX_ITERS_PER_S (far above what one
            # search reaches on the GPU); stats["iteration_bound_reached"] reports a search
            # that hit the bound before its time ran out
            tl_us = int(round(float(a.time_limit) * 1e6)) if a.time_limit else 0
            iters = int(a.iterations)
            if tl_us:
                iters = int(min(TIMED_MAX_ITERS, max(16, math.ceil(float(a.time_limit) * TIMED_MAX_ITERS_PER_S))))
            policy = _search_policy(a.rollout_agent)
            if policy is None:
                raise ValueError("search_batch: the rollout agent cannot be replayed on the GPU")
            key = (iters, a.max_rollout_moves, float(a.exploration_constant), a.use_transposition_table,
                   tl_us, policy)
            groups.setdefault(key, []).append(i)
        for (iters, max_roll, c, use_tt, tl_us, policy), idx in groups.items():
            ags = [agents[i] for i in idx]
            gpu = BlokusGPU.shared(ags[0].device)
            rts = np.ascontiguousarray(roots[idx])
            sts = np.ascontiguousarray(sets[idx])
            pl = np.array([players[i] for i in idx], np.uint8)
            rts["current_player"] = pl
            tabs, zidx = [], []
            for a in ags:
                tabs.append(flat_keys(a.zobrist_hash))
                zidx.append(len(tabs) - 1)
            zob = np.stack(tabs)
            rh = hash_states(rts, zob)  # one table per search
            views = [_mt_view(a.rollout_agent.rng) for a in ags]
            if all(v is not None for v in views):
                mt = np.stack(views)  # a copy: the kernel advances it, written back below
                rng_states = None
            else:
                mt = np.zeros((len(idx), 625), np.uint32)
                rng_states = [a.rollout_agent.rng.get_state() for a in ags]
                for j, st in enumerate(rng_states):
                    mt[j, :624] = st[1]
                    mt[j, 624] = st[2]
            t0 = time.time()
            r = _search_on_device(gpu, ags, rts, sts, pl, rh, zob, np.array(zidx, np.int32), mt, iters, max_roll, c,
                                  use_tt, tl_us, policy)
            dt = time.time() - t0
            kms, ksims = gpu.last_kernel_ms(), int(r["out"]["iterations_run"].sum())
            kplies = int(r["out"]["rollout_plies"].astype(np.int64).sum())
            for tot in (SEARCH_TOTALS, SEARCH_TOTALS["by_kernel"].setdefault(
                    gpu.last_kernel(), {"launches": 0, "kernel_ms": 0.0, "sims": 0, "rollout_plies": 0})):
                tot["launches"] += 1
                tot["kernel_ms"] += kms
                tot["sims"] += ksims
                tot["rollout_plies"] += kplies
            # the non-hit rewards of every search as Python lists in one pass (NaN marks a
            # TT hit or an iteration past the search's end: rewards are finite)
            its = np.arange(r["rewards"].shape[1])[None, :]
            live = (r["hit_flags"] == 0) & (its < r["out"]["iterations_run"][:, None])
            rew_rows = np.where(live, r["rewards"], np.nan).tolist()
            ro = r["out"]  # per-search fields as Python ints (structured-scalar access is slow)
            f_it, f_hits, f_roll = ro["iterations_run"].tolist(), ro["tt_hits"].tolist(), ro["rollouts"].tolist()
            f_status, f_best = ro["status"].tolist(), ro["best_move"].tolist()
            for j, (i, a) in enumerate(zip(idx, ags)):
                if rng_states is None:
                    views[j][:] = mt[j]
                else:
                    st = rng_states[j]
                    a.rollout_agent.rng.set_state((st[0], mt[j, :624].copy(), int(mt[j, 624]), st[3], st[4]))
                n_it = f_it[j]
                a.stats["iterations_run"] = n_it
                # HeuristicAgent rollouts: a draw within 2^-40 of a probability boundary
                # (BK_MCTS_EUNCERT; the kernel flags the search, it does not count draws)
                unc = bool(f_status[j] & N.MCTS_EUNCERT)
                a.stats["last_search_uncertified"] = unc
                a.stats["uncertified_searches"] = a.stats.get("uncertified_searches", 0) + int(unc)
                if tl_us:
                    a.stats["iteration_bound"] = iters
                    a.stats["iteration_bound_reached"] = n_it >= iters
                    if a.stats["iteration_bound_reached"]:
                        warnings.warn(f"MCTSAgent: a {a.time_limit} s search stopped at its {iters}-iteration "
                                      "bound before the time ran out", RuntimeWarning, stacklevel=2)
                a.stats["time_elapsed"] = dt
                a.stats["transposition_hits"] += f_hits[j]
                a.stats["rollout_rewards"].extend([x for x in rew_rows[j] if x == x])
                if use_tt:
                    t = a.transposition_table
                    t.access_count += f_hits[j] + f_roll[j]
                    t.hit_count += f_hits[j]
                    t.gpu_size = int(a._gpu_tt.count[0])
                    if t.gpu_size > 500000:  # mcts_agent.py:338-339
                        t.clear()
                        a._gpu_tt.release()
                        a._gpu_tt = None
                out[i] = f_best[j] if f_best[j] >= 0 else None
        return out

    def _get_move_positions(self, move: Move) -> List[Position]:
        return _positions(move)

    def _mcts_iteration(self, root: MCTSNode):
        node = self._selection(root)
        if not node.is_fully_expanded() and not node.is_terminal():
            node = node.expand()
            if node is None:
                return
        self._backpropagation(node, self._simulation(node))

    def _selection(self, node: MCTSNode) -> MCTSNode:
        while not node.is_terminal():
            if not node.is_fully_expanded():
                return node
            node = node.select_child(self.exploration_constant, 0.0)
        return node

    def _simulation(self, node: MCTSNode) -> float:
        if self.transposition_table:
            h = self.zobrist_hash.hash_board(node.board)
            hit = self.transposition_table.get(h)
            if hit:
                self.stats["transposition_hits"] += 1
                return hit["reward"]
        reward = self._rollout(node.board, node.player)
        if self.transposition_table:
            self.transposition_table.put(h, {"reward": reward})
        self.stats["rollout_rewards"].append(reward)
        return reward

    def _rollout(self, board: Board, player: Player) -> float:
        if self.rollout_backend == "kernel":
            return self._rollout_kernel(board, player)
        sim = board.copy()
        cur = player
        start = sim.get_score(player)
        for _ in range(self.max_rollout_moves):
            legal = self.move_generator.get_legal_moves(sim, cur)
            if not legal:
                break
            mv = self.rollout_agent.select_action(sim, cur, legal)
            if mv is None or not sim.place_piece(_positions(mv), cur, mv.piece_id, validate=False):
                break
            cur = _PLAYERS[(_PLAYERS.index(cur) + 1) % 4]
        reward = sim.get_score(player) - start
        if sim.is_game_over():  # never set inside a rollout (reference dead code kept for parity)
            w = sim.get_winner()
            reward += 100 if w == player else 10 if w is None else 0
        return reward

    def _rollout_kernel(self, board: Board, player: Player) -> float:
        from .. import _native as N
        from ..gpu import BlokusGPU
        if self._gpu is None:
            self._gpu = BlokusGPU(self.device)
        st = pack_state(board)
        st["current_player"] = player.value - 1
        self._kernel_calls += 1
        res = self._gpu.rollout(st, 1, semantics=N.SEM_ROLLOUT, rng=N.RNG_PHILOX,
                                seed=(self.seed << 20) + self._kernel_calls, max_plies=self.max_rollout_moves)
        return float(res["reward"][0])

    def _backpropagation(self, node: MCTSNode, reward: float):
        while node is not None:
            node.update(reward)
            node = node.parent

    def get_action_info(self) -> Dict[str, Any]:
        info = {"name": "MCTSAgent", "type": "mcts", "description": "UCT MCTS with GPU random rollouts",
                "parameters": {"iterations": self.iterations, "time_limit": self.time_limit,
                               "exploration_constant": self.exploration_constant,
                               "use_transposition_table": self.use_transposition_table,
                               "max_rollout_moves": self.max_rollout_moves,
                               "rollout_backend": self.rollout_backend},
                "stats": self.stats.copy()}
        if self.transposition_table:
            info["transposition_stats"] = self.transposition_table.get_stats()
        return info

    def reset(self):
        self.stats = self._fresh_stats()
        if self.transposition_table:
            self.transposition_table.clear()
        if self._gpu_tt is not None:
            self._gpu_tt.release()
        self._gpu_tt = None

    def set_seed(self, seed: int):
        self.zobrist_hash = ZobristHash(seed=seed)
        self.seed = int(seed)
        if self.rollout_agent is not None:
            self.rollout_agent.set_seed(seed)
