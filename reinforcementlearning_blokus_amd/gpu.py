"""Batched GPU entry points (thin Python layer over the C-ABI).

Inputs may be numpy arrays (host; the library stages them) or torch tensors already
on the GPU (device pointers, launched on torch's current stream).  There is no CPU
implementation behind any of these functions.
"""
from __future__ import annotations

import threading
import warnings

import numpy as np

from . import _native as N

STATE_DTYPE = N.STATE_DTYPE
RESULT_DTYPE = N.RESULT_DTYPE


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _as_host(x, dtype):
    a = np.ascontiguousarray(x)
    if dtype is not None and a.dtype != dtype:
        a = a.view(dtype) if a.dtype.itemsize == 1 and dtype.itemsize != 1 else a.astype(dtype)
    return a


class BlokusGPU:
    """Owns one bk_handle (one HIP stream + scratch) on `device`."""

    _shared = threading.local()

    def __init__(self, device: int = 0):
        self.handle = N.Handle(device)
        self.device = device

    @classmethod
    def shared(cls, device: int = 0) -> "BlokusGPU":
        """One engine per (thread, device) for batched callers (MCTSAgent.search_packed):
        the agents of an arena share its handle and scratch instead of each allocating its
        own.  Per thread, because a call binds the handle to the caller's current torch
        stream (agents run in worker threads in the reference's web API)."""
        engines = cls._shared.__dict__.setdefault("engines", {})
        if device not in engines:
            engines[device] = cls(device)
        return engines[device]

    # ------------------------------------------------------------------ helpers
    def _stream_from_torch(self):
        import torch
        self.handle.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def last_kernel_ms(self) -> float:
        return self.handle.last_kernel_ms()

    def last_kernel(self) -> str:
        return self.handle.last_kernel()

    def synchronize(self):
        """Wait for this handle's launches; raises if a device-path launch tripped its
        iteration guard or read a bad root_index, or a search broke a tree invariant
        (bk_synchronize; mcts_failure() then has the record)."""
        self.handle.synchronize()

    def mcts_failure(self):
        """The record of the first bk_mcts search on this handle whose tree broke an
        invariant (a node visited more often than the iterations allow, or root visits !=
        iterations run), or None (bk_debug_mcts_failure)."""
        return self.handle.mcts_failure()

    def tune(self, **overrides):
        """Set tuning / test overrides of this handle by their environment-variable names
        without the BK_ prefix (tune(MCTS_COOP=1, COOP_BAL=None); None = automatic).  The
        library reads the environment once per handle, at creation (bk_set_tuning)."""
        for k, v in overrides.items():
            self.handle.set_tuning("BK_" + k, v)

    def _check_playout_tensors(self, roots, n_playouts, root_index, compat_seeds, out, rng):
        import torch
        _check_device_tensor(roots, "roots", torch.uint8, (roots.shape[0], 256), self.device)
        if root_index is not None:
            _check_device_tensor(root_index, "root_index", torch.int32, (root_index.shape[0],), self.device)
            if root_index.shape[0] < n_playouts:
                raise ValueError(f"root_index: {root_index.shape[0]} entries for {n_playouts} playouts")
        if rng == N.RNG_NUMPY_MT:
            if compat_seeds is None:
                raise ValueError("compat rng needs compat_seeds")
            if compat_seeds.dtype not in (torch.int32, torch.uint32):
                raise ValueError(f"compat_seeds: expected int32/uint32, got {compat_seeds.dtype}")
            _check_device_tensor(compat_seeds, "compat_seeds", compat_seeds.dtype, (compat_seeds.shape[0], 4),
                                 self.device)
            if compat_seeds.shape[0] < n_playouts:
                raise ValueError("compat_seeds: fewer rows than playouts")
        if out is not None:
            _check_device_tensor(out, "out", torch.uint8, (out.shape[0], 32), self.device)
            if out.shape[0] < n_playouts:
                raise ValueError("out: fewer rows than playouts")

    # ------------------------------------------------------------------ movegen
    def movegen(self, states, players, rows: bool = True):
        """Legal-move masks + counts for (state, player) pairs.

        states: n bk_state records (numpy STATE_DTYPE / uint8[n,256], or a torch uint8
        cuda tensor [n,256]); players: n uint8 in 0..3.
        Returns (counts[n] uint32, rows[n,91,20] uint32 or None); rows[i,g,r] bit c =
        anchor (r, c) legal for global orientation g (move_generator.py:130 set).
        """
        if _is_torch(states):
            import torch
            n = states.shape[0]
            _check_device_tensor(states, "states", torch.uint8, (n, 256), self.device)
            _check_device_tensor(players, "players", torch.uint8, (n,), self.device)
            cnt = torch.empty(n, dtype=torch.int32, device=states.device)
            out = torch.empty((n, N.N_ORIENTS, 20), dtype=torch.int32, device=states.device) if rows else None
            self._stream_from_torch()
            self.handle.movegen(states.data_ptr(), players.data_ptr(), n, out.data_ptr() if rows else 0,
                                cnt.data_ptr(), N.MEM_DEVICE)
            return cnt, out
        st = np.ascontiguousarray(states).view(np.uint8).reshape(-1, 256)
        pl = np.ascontiguousarray(players, dtype=np.uint8)
        n = st.shape[0]
        assert pl.shape[0] == n
        cnt = np.zeros(n, dtype=np.uint32)
        out = np.zeros((n, N.N_ORIENTS, 20), dtype=np.uint32) if rows else None
        self.handle.set_stream(None)
        self.handle.movegen(st.ctypes.data, pl.ctypes.data, n, out.ctypes.data if rows else 0, cnt.ctypes.data,
                            N.MEM_HOST)
        return cnt, out

    def movegen_mask(self, states, players, masks: bool = True):
        """movegen with the legal sets as 400-bit masks (bk_movegen_mask): returns
        (counts[n] uint32, masks[n,91,7] uint64 or None); bit r*20+c of masks[i,g] =
        anchor (r, c) legal for global orientation g (engine/move_generator.py:130 set,
        Board.player_bits numbering).  Inputs as movegen; torch in -> torch out."""
        if _is_torch(states):
            import torch
            n = states.shape[0]
            _check_device_tensor(states, "states", torch.uint8, (n, 256), self.device)
            _check_device_tensor(players, "players", torch.uint8, (n,), self.device)
            cnt = torch.empty(n, dtype=torch.int32, device=states.device)
            out = torch.empty((n, N.N_ORIENTS, 7), dtype=torch.int64, device=states.device) if masks else None
            self._stream_from_torch()
            self.handle.movegen_mask(states.data_ptr(), players.data_ptr(), n, out.data_ptr() if masks else 0,
                                     cnt.data_ptr(), N.MEM_DEVICE)
            return cnt, out
        st = np.ascontiguousarray(states).view(np.uint8).reshape(-1, 256)
        pl = np.ascontiguousarray(players, dtype=np.uint8)
        n = st.shape[0]
        assert pl.shape[0] == n
        cnt = np.zeros(n, dtype=np.uint32)
        out = np.zeros((n, N.N_ORIENTS, 7), dtype=np.uint64) if masks else None
        self.handle.set_stream(None)
        self.handle.movegen_mask(st.ctypes.data, pl.ctypes.data, n, out.ctypes.data if masks else 0, cnt.ctypes.data,
                                 N.MEM_HOST)
        return cnt, out

    def has_moves(self, states):
        """uint8 mask per state: bit p set iff player p has a legal move (move_generator.py:961)."""
        if _is_torch(states):
            import torch
            n = states.shape[0]
            _check_device_tensor(states, "states", torch.uint8, (n, 256), self.device)
            out = torch.empty(n, dtype=torch.uint8, device=states.device)
            self._stream_from_torch()
            self.handle.has_moves(states.data_ptr(), n, out.data_ptr(), N.MEM_DEVICE)
            return out
        st = np.ascontiguousarray(states).view(np.uint8).reshape(-1, 256)
        out = np.zeros(st.shape[0], dtype=np.uint8)
        self.handle.set_stream(None)
        self.handle.has_moves(st.ctypes.data, st.shape[0], out.ctypes.data, N.MEM_HOST)
        return out

    # ------------------------------------------------------------------ rollouts
    def rollout(self, roots, n_playouts: int, *, semantics: int = N.SEM_ARENA, rng: int = N.RNG_PHILOX,
                seed: int = 0, max_plies: int | None = None, compat_seeds=None, root_index=None,
                order: int = N.ORDER_NAIVE, seats_share_stream: bool = False, out=None, stream_base: int = 0):
        """Random playouts from roots (see bk_rollout in include/blokus_hip.h).

        Host numpy in -> numpy RESULT_DTYPE out; torch cuda in -> torch uint8 [n,32] out.
        stream_base: playout i draws from Philox stream (seed, stream_base + i).
        """
        if max_plies is None:
            max_plies = 2500 if semantics == N.SEM_ARENA else 50
        cfg = N.BkRolloutCfg(semantics, order, rng, max_plies, seed & (2**64 - 1), int(seats_share_stream), 0,
                             _stream_base(stream_base, n_playouts))
        if _is_torch(roots):
            import torch
            dev = roots.device
            if out is None:
                out = torch.empty((n_playouts, 32), dtype=torch.uint8, device=dev)
            self._check_playout_tensors(roots, n_playouts, root_index, compat_seeds, out, rng)
            self._stream_from_torch()
            self.handle.rollout(roots.data_ptr(), roots.shape[0],
                                root_index.data_ptr() if root_index is not None else 0, n_playouts, cfg,
                                compat_seeds.data_ptr() if compat_seeds is not None else 0, out.data_ptr(),
                                N.MEM_DEVICE)
            return out
        st = np.ascontiguousarray(roots).view(np.uint8).reshape(-1, 256)
        res = np.zeros(n_playouts, dtype=RESULT_DTYPE)
        idx = _host_root_index(root_index, n_playouts)
        seeds = np.ascontiguousarray(compat_seeds, dtype=np.uint32).reshape(-1, 4) if compat_seeds is not None else None
        if seeds is not None:
            assert seeds.shape[0] >= n_playouts
        self.handle.set_stream(None)
        self.handle.rollout(st.ctypes.data, st.shape[0], idx.ctypes.data if idx is not None else 0, n_playouts, cfg,
                            seeds.ctypes.data if seeds is not None else 0, res.ctypes.data, N.MEM_HOST)
        return res

    # ------------------------------------------------------------------ frontier order
    def rollout_frontier(self, roots, root_sets, n_playouts: int, *, semantics: int = N.SEM_ARENA,
                         rng: int = N.RNG_NUMPY_MT, seed: int = 0, max_plies: int | None = None,
                         compat_seeds=None, root_index=None, seats_share_stream: bool = False, out=None,
                         with_results: bool = False, with_states: bool = False, heuristic_seats: int = 0,
                         stream_base: int = 0):
        """Playouts in the reference's FRONTIER list order (bk_rollout_frontier): with the
        numpy-MT compat stream these are the reference's default-config games.
        root_sets: FSET_DTYPE records (one per root).  Host numpy in/out.  SEM_ADVANCE
        returns (states, tables[, results]); SEM_ARENA with with_states returns
        (states, tables, results): the final positions as well.  heuristic_seats: bit p =
        seat p plays HeuristicAgent (its draws from the seat's compat stream)."""
        if max_plies is None:
            max_plies = 2500 if semantics == N.SEM_ARENA else 50
        cfg = N.BkRolloutCfg(semantics, N.ORDER_FRONTIER, rng, max_plies, seed & (2**64 - 1),
                             int(seats_share_stream), int(heuristic_seats), _stream_base(stream_base, n_playouts))
        if _is_torch(roots):  # device tensors: roots uint8 [n,256], root_sets uint8 [n,2080]
            import torch
            assert semantics != N.SEM_ADVANCE, "device path: playout results only"
            if out is None:
                out = torch.empty((n_playouts, 32), dtype=torch.uint8, device=roots.device)
            self._check_playout_tensors(roots, n_playouts, root_index, compat_seeds, out, rng)
            _check_device_tensor(root_sets, "root_sets", torch.uint8, (roots.shape[0], N.FSET_DTYPE.itemsize),
                                 self.device)
            self._stream_from_torch()
            self.handle.rollout_frontier(roots.data_ptr(), root_sets.data_ptr(), roots.shape[0],
                                         root_index.data_ptr() if root_index is not None else 0, n_playouts, cfg,
                                         compat_seeds.data_ptr() if compat_seeds is not None else 0,
                                         out.data_ptr(), 0, 0, N.MEM_DEVICE)
            return out
        st = np.ascontiguousarray(roots).view(np.uint8).reshape(-1, 256)
        fs = np.ascontiguousarray(root_sets, dtype=N.FSET_DTYPE)
        assert fs.shape[0] == st.shape[0]
        idx = _host_root_index(root_index, n_playouts)
        seeds = np.ascontiguousarray(compat_seeds, dtype=np.uint32).reshape(-1, 4) if compat_seeds is not None else None
        if seeds is not None:
            assert seeds.shape[0] >= n_playouts
        self.handle.set_stream(None)
        if semantics == N.SEM_ADVANCE or (semantics == N.SEM_ARENA and with_states):  # (states, tables[, results])
            with_results = with_results or semantics == N.SEM_ARENA
            out_st = np.zeros(n_playouts, dtype=STATE_DTYPE)
            out_fs = np.zeros(n_playouts, dtype=N.FSET_DTYPE)
            res = np.zeros(n_playouts, dtype=RESULT_DTYPE) if with_results else None
            self.handle.rollout_frontier(st.ctypes.data, fs.ctypes.data, st.shape[0],
                                         idx.ctypes.data if idx is not None else 0, n_playouts, cfg,
                                         seeds.ctypes.data if seeds is not None else 0,
                                         res.ctypes.data if res is not None else 0, out_st.ctypes.data,
                                         out_fs.ctypes.data, N.MEM_HOST)
            return (out_st, out_fs, res) if with_results else (out_st, out_fs)
        res = np.zeros(n_playouts, dtype=RESULT_DTYPE)
        self.handle.rollout_frontier(st.ctypes.data, fs.ctypes.data, st.shape[0],
                                     idx.ctypes.data if idx is not None else 0, n_playouts, cfg,
                                     seeds.ctypes.data if seeds is not None else 0, res.ctypes.data, 0, 0,
                                     N.MEM_HOST)
        return res

    # ------------------------------------------------------------------ arena with search seats
    def arena_advance(self, states, sets, seat_masks, rng_state, *, max_turns: int = 2500):
        """bk_arena_advance on host arrays, in place: states (STATE_DTYPE[n]), sets
        (FSET_DTYPE[n]), rng_state uint32[n, 16]; seat_masks uint8[n] (bits 0-3 heuristic
        seats, 4-7 stop seats).  Returns RESULT_DTYPE[n]."""
        n = len(states)
        assert states.dtype == STATE_DTYPE and sets.dtype == N.FSET_DTYPE and len(sets) == n
        assert states.flags.c_contiguous and sets.flags.c_contiguous
        masks = np.ascontiguousarray(seat_masks, dtype=np.uint8)
        assert masks.shape == (n,) and rng_state.dtype == np.uint32 and rng_state.shape == (n, 16)
        assert rng_state.flags.c_contiguous
        cfg = N.BkRolloutCfg(N.SEM_ARENA, N.ORDER_FRONTIER, N.RNG_NUMPY_MT, int(max_turns), 0, 0, 0)
        out = np.zeros(n, dtype=RESULT_DTYPE)
        if n == 0:
            return out
        self.handle.set_stream(None)
        self.handle.arena_advance(states.ctypes.data, sets.ctypes.data, n, cfg, masks.ctypes.data,
                                  rng_state.ctypes.data, out.ctypes.data, N.MEM_HOST)
        return out

    def arena_step(self, states, sets, seat_masks, rng_state, quick_masks, forced, out, stop_out, *,
                   max_turns: int = 2500):
        """bk_arena_step on device tensors, in place (BK_MEM_DEVICE, torch's current
        stream): states uint8[n,256], sets uint8[n,2080], seat_masks / quick_masks uint8[n],
        forced int32[n], rng_state int32[n,16], out uint8[n,32], stop_out uint8[n,16]
        (STOP_DTYPE).  No position or table crosses PCIe (config 4's device driver)."""
        import torch
        n = states.shape[0]
        for t, name, dt, shape in ((states, "states", torch.uint8, (n, 256)),
                                   (sets, "sets", torch.uint8, (n, N.FSET_DTYPE.itemsize)),
                                   (seat_masks, "seat_masks", torch.uint8, (n,)),
                                   (quick_masks, "quick_masks", torch.uint8, (n,)),
                                   (forced, "forced", torch.int32, (n,)), (rng_state, "rng_state", torch.int32, (n, 16)),
                                   (out, "out", torch.uint8, (n, 32)),
                                   (stop_out, "stop_out", torch.uint8, (n, N.STOP_DTYPE.itemsize))):
            _check_device_tensor(t, name, dt, shape, self.device)
        cfg = N.BkRolloutCfg(N.SEM_ARENA, N.ORDER_FRONTIER, N.RNG_NUMPY_MT, int(max_turns), 0, 0, 0)
        if n == 0:
            return
        self._stream_from_torch()
        self.handle.arena_step(states.data_ptr(), sets.data_ptr(), n, cfg, seat_masks.data_ptr(),
                               quick_masks.data_ptr(), forced.data_ptr(), rng_state.data_ptr(), out.data_ptr(),
                               stop_out.data_ptr(), N.MEM_DEVICE)

    # ------------------------------------------------------------------ positions
    def advance(self, roots, n: int, plies: int, *, seed: int = 0, root_index=None, stream_base: int = 0):
        """Play `plies` uniformly random moves (naive order, Philox stream) from each root
        and return the reached states (BK_SEM_ADVANCE).  Batched analogue of
        tests/utils_game_states.py:12 generate_random_valid_state (different RNG)."""
        cfg = N.BkRolloutCfg(N.SEM_ADVANCE, N.ORDER_NAIVE, N.RNG_PHILOX, plies, seed & (2**64 - 1), 0, 0,
                             _stream_base(stream_base, n))
        if _is_torch(roots):
            import torch
            out = torch.empty((n, 256), dtype=torch.uint8, device=roots.device)
            self._check_playout_tensors(roots, n, root_index, None, None, N.RNG_PHILOX)
            self._stream_from_torch()
            self.handle.advance(roots.data_ptr(), roots.shape[0],
                                root_index.data_ptr() if root_index is not None else 0, n, cfg, 0,
                                out.data_ptr(), N.MEM_DEVICE)
            return out
        st = np.ascontiguousarray(roots).view(np.uint8).reshape(-1, 256)
        out = np.zeros(n, dtype=STATE_DTYPE)
        idx = _host_root_index(root_index, n)
        self.handle.set_stream(None)
        self.handle.advance(st.ctypes.data, st.shape[0], idx.ctypes.data if idx is not None else 0, n, cfg, 0,
                            out.ctypes.data, N.MEM_HOST)
        return out

    # ------------------------------------------------------------------ FastMCTS
    def fastmcts(self, n_legal, iterations, base, mt_state, log_table, exploration: float,
                 want_visits: bool = False, exact_ucb: bool = True):
        """Run FastMCTSAgent's bandit loop for a batch of roots (bk_fastmcts).

        n_legal[i]: root legal-move count; iterations[i]; base[i]: deterministic part of
        the rollout reward (NaN = empty cached list); mt_state: uint32[n,625] CPython
        random states, advanced in place; log_table[k] = math.log(k).  exact_ucb: build
        the pow-correction rows the iteration counts need (bk_pow_half_fix), else use
        whatever rows are cached (wall-clock-bounded searches).
        Returns a FASTMCTS_OUT_DTYPE record array (and, with want_visits, the flat int32
        visit counts per legal index)."""
        n = len(n_legal)
        off = np.zeros(n + 1, dtype=np.int32)
        np.cumsum(np.asarray(n_legal, dtype=np.int32), out=off[1:])
        it = np.ascontiguousarray(iterations, dtype=np.int32)
        b = np.ascontiguousarray(base, dtype=np.float64)
        assert mt_state.dtype == np.uint32 and mt_state.shape == (n, 625) and mt_state.flags.c_contiguous
        lt = np.ascontiguousarray(log_table, dtype=np.float64)
        need = int(it.max(initial=0))
        fo, fe = N.pow_half_fix(lt, rows=need, cached_only=not exact_ucb)
        if exact_ucb and len(fo) - 1 < need:
            # parent visits >= the table's rows use plain sqrt: the UCB of a child can be one
            # ulp off CPython's (2*log(N)/v) ** 0.5 there, so a near-tie may pick another child
            warnings.warn(f"FastMCTS: {need} iterations exceed the {len(fo) - 1} pow-correction rows "
                          "(_native.POW_FIX_ROWS); UCB1 is bit-exact only below that", RuntimeWarning,
                          stacklevel=2)
        out = np.zeros(n, dtype=N.FASTMCTS_OUT_DTYPE)
        vis = np.zeros(max(int(off[-1]), 1), dtype=np.int32) if want_visits else None
        self.handle.set_stream(None)
        self.handle.fastmcts(n, off.ctypes.data, it.ctypes.data, b.ctypes.data, mt_state.ctypes.data,
                             lt.ctypes.data, len(lt), fo.ctypes.data, fe.ctypes.data if len(fe) else 0, len(fo) - 1,
                             exploration, out.ctypes.data, vis.ctypes.data if vis is not None else 0, N.MEM_HOST)
        return (out, vis[: int(off[-1])]) if want_visits else out

    def fastmcts_device(self, legal_offset, iterations, base, mt_state, log_table, pow_fix_offsets, pow_fix_entries,
                        exploration: float, out):
        """bk_fastmcts on torch CUDA tensors (BK_MEM_DEVICE, torch's current stream, not
        waited for): legal_offset int32[n+1] (0, cumulative legal counts), iterations
        int32[n], base float64[n], mt_state int32[n,625] (advanced in place), log_table
        float64, pow-fix offsets / entries int32 (N.pow_half_fix of the same log_table),
        out uint8[n, FASTMCTS_OUT_DTYPE.itemsize].  The caller validates the counts
        (iterations < len(log_table)); the config-4 driver's FastMCTS seats."""
        import torch
        n = iterations.shape[0]
        for t, name, dt, shape in ((legal_offset, "legal_offset", torch.int32, (n + 1,)),
                                   (iterations, "iterations", torch.int32, (n,)), (base, "base", torch.float64, (n,)),
                                   (mt_state, "mt_state", torch.int32, (n, 625)),
                                   (out, "out", torch.uint8, (n, N.FASTMCTS_OUT_DTYPE.itemsize))):
            _check_device_tensor(t, name, dt, shape, self.device)
        _check_device_tensor(log_table, "log_table", torch.float64, (log_table.shape[0],), self.device)
        rows = pow_fix_offsets.shape[0] - 1
        if n == 0:
            return
        self._stream_from_torch()
        self.handle.fastmcts(n, legal_offset.data_ptr(), iterations.data_ptr(), base.data_ptr(), mt_state.data_ptr(),
                             log_table.data_ptr(), log_table.shape[0], pow_fix_offsets.data_ptr(),
                             pow_fix_entries.data_ptr() if pow_fix_entries.numel() else 0, rows, exploration,
                             out.data_ptr(), 0, N.MEM_DEVICE)

    def fastmcts_select(self, visits, totals, root_visits: int, log_table, exploration: float) -> int:
        """Diagnostic: k_fastmcts's UCB1 argmax (FastMCTSNode.select_child,
        fast_mcts_agent.py:45-56) over children with these visits / total rewards."""
        v = np.ascontiguousarray(visits, dtype=np.uint32)
        t = np.ascontiguousarray(totals, dtype=np.float64)
        assert len(v) == len(t) and len(v) > 0
        lt = np.ascontiguousarray(log_table, dtype=np.float64)
        fo, fe = N.pow_half_fix(lt)
        self.handle.set_stream(None)
        return self.handle.debug_fastmcts_select(len(v), v.ctypes.data, t.ctypes.data, int(root_visits), lt.ctypes.data,
                                                 len(lt), fo.ctypes.data, fe.ctypes.data if len(fe) else 0,
                                                 len(fo) - 1, exploration)

    # ------------------------------------------------------------------ MCTSAgent
    def mcts(self, roots, root_sets, players, root_hash, *, iterations: int, zobrist, mt_state,
             zobrist_index=None, tt: "MctsTT" = None, max_rollout_moves: int = 50, exploration: float = 1.414,
             log_table=None, node_cap: int = 0, time_limit_us: int = 0, want_rewards: bool = True,
             want_nodes: bool = False, chunk: int = 0, rollout_policy: int = N.MCTS_ROLLOUT_RANDOM):
        """MCTSAgent.select_action searches for a batch of positions, whole on the GPU
        (bk_mcts; mcts/mcts_agent.py:304-582 with RandomAgent rollouts).

        roots / root_sets / players / root_hash: per game (STATE_DTYPE, FSET_DTYPE, the
        searching player 0..3, ZobristHash.hash_board).  zobrist: uint64[n_tables, 2088]
        key tables (cells x 5, turn x 4, player x piece), zobrist_index[g] picks one.
        mt_state: uint32[n, 625] numpy MT19937 states (key then pos), advanced in place.
        tt: an MctsTT (one table per game, kept across calls) or None (no TT).
        node_cap: node slots per search (default 4 * iterations + 1, which the kernel's
        child-block growth never exceeds).  chunk > 0: run the searches in launches of
        `chunk` iterations (cfg.iter_stop / cfg.resume), same result as one launch.
        rollout_policy: MCTS_ROLLOUT_RANDOM (RandomAgent) or MCTS_ROLLOUT_HEURISTIC
        (HeuristicAgent, MCTSAgent's default); mt_state is that agent's stream.
        Returns dict(out=MCTS_OUT_DTYPE[n], rewards, hit_flags, nodes)."""
        n = len(roots)
        roots = np.ascontiguousarray(roots, dtype=STATE_DTYPE)
        root_sets = np.ascontiguousarray(root_sets, dtype=N.FSET_DTYPE)
        pl = np.ascontiguousarray(players, dtype=np.uint8)
        rh = np.ascontiguousarray(np.asarray(root_hash, dtype=np.uint64))
        zob = np.ascontiguousarray(np.asarray(zobrist, dtype=np.uint64).reshape(-1, N.MCTS_ZOBRIST_WORDS))
        zi = np.zeros(n, np.int32) if zobrist_index is None else np.ascontiguousarray(zobrist_index, dtype=np.int32)
        assert mt_state.dtype == np.uint32 and mt_state.shape == (n, 625) and mt_state.flags.c_contiguous
        assert len(root_sets) == n and len(pl) == n and len(rh) == n and len(zi) == n
        assert not (chunk and time_limit_us), "chunked searches run a fixed iteration count"
        if log_table is None:
            log_table = mcts_log_table(iterations)
        lt = np.ascontiguousarray(log_table, dtype=np.float64)
        if tt is not None:
            tt.reserve(iterations + 1)
            assert tt.keys.shape[0] == n
        cap = int(node_cap) or mcts_node_cap(iterations)
        mt0 = mt_state.copy()
        tt0 = tt.snapshot() if tt is not None else None
        stops = mcts_chunks(iterations, chunk)
        while True:
            out = np.zeros(n, dtype=N.MCTS_OUT_DTYPE)
            rewards = np.zeros((n, max(iterations, 1))) if want_rewards else None
            flags = np.zeros((n, max(iterations, 1)), np.uint8) if want_rewards else None
            nodes = np.zeros((n, cap), dtype=N.MCTS_NODE_DTYPE) if (want_nodes or len(stops) > 1) else None
            ptr = lambda x: x.ctypes.data if x is not None else 0  # noqa: E731
            self.handle.set_stream(None)
            for j, stop in enumerate(stops):
                cfg = N.BkMctsCfg(iterations, max_rollout_moves, float(exploration), int(tt is not None), cap,
                                  tt.cap if tt is not None else 0, int(time_limit_us), stop, int(j > 0),
                                  int(rollout_policy), 0)
                self.handle.mcts(roots.ctypes.data, root_sets.ctypes.data, pl.ctypes.data, rh.ctypes.data, n, cfg,
                                 zob.ctypes.data, len(zob), zi.ctypes.data, mt_state.ctypes.data,
                                 ptr(tt.keys) if tt is not None else 0, ptr(tt.vals) if tt is not None else 0,
                                 ptr(tt.count) if tt is not None else 0, lt.ctypes.data, len(lt), ptr(nodes),
                                 ptr(rewards), ptr(flags), out.ctypes.data, N.MEM_HOST)
            st = out["status"]
            if (st & N.MCTS_EPOOL).any() and not (st & ~np.uint32(N.MCTS_EPOOL)).any():
                mt_state[:] = mt0  # roll back and retry with a bigger pool (only for a caller-set cap)
                if tt is not None:
                    tt.restore(tt0)
                cap = cap * 2 + 1
                continue
            fatal = st & ~np.uint32(N.MCTS_EUNCERT)
            if fatal.any():
                raise RuntimeError(f"bk_mcts: search stopped early, status bits {sorted(set(st[st != 0].tolist()))}")
            return {"out": out, "rewards": rewards, "hit_flags": flags, "nodes": nodes, "node_cap": cap,
                    "uncertified": int((st & np.uint32(N.MCTS_EUNCERT) != 0).sum())}

    def mcts_device(self, roots, root_sets, players, root_hash, zobrist, zobrist_index, mt_state, log_table, nodes,
                    out, *, iterations: int, tt_keys=None, tt_vals=None, tt_count=None, rewards=None,
                    hit_flags=None, max_rollout_moves: int = 50, exploration: float = 1.414, chunk: int = 0,
                    on_chunk=None, stop_after: int | None = None, rollout_policy: int = N.MCTS_ROLLOUT_RANDOM,
                    resume_from: int | None = None, time_limit_us: int = 0, asynchronous: bool = False,
                    state_rows: bool = False, out_ptr: int | None = None):
        """bk_mcts with every buffer a torch CUDA tensor on this device (zero copy,
        BK_MEM_DEVICE, torch's current stream): the config-5 path, where the trees
        (nodes[n, node_cap]), TTs and RNG states of 65,536 searches stay in HBM.
        Layouts as in mcts(): roots uint8[n,256], root_sets uint8[n,2080], players
        uint8[n], root_hash (None: computed on the device) / zobrist int64, zobrist_index
        int32[n], mt_state int32[n,625],
        log_table float64, nodes uint8[n, node_cap*24], out uint8[n,32], tt_keys int64 /
        tt_vals float64 [n, tt_cap] (NaN = empty) + tt_count int32[n] (all or none),
        rewards float64 / hit_flags uint8 [n, iterations] (optional).  chunk > 0 splits
        the searches into launches of `chunk` iterations; on_chunk(done_iterations) is
        called after each; stop_after: run only the first stop_after iterations (they
        can be resumed by no caller here: a warm-up).  time_limit_us: stop each search at
        the first iteration boundary past it (no chunking).  Raises if any search reports
        a nonzero status.  asynchronous: one launch, enqueued on torch's current stream
        and not waited for (BK_MCTS_ASYNC); the caller checks the statuses in `out` and
        calls synchronize() once the stream has passed it.  state_rows (BK_MCTS_STATE_ROWS):
        mt_state / tt_* are the agents' rows [agents, ...], search g using row
        zobrist_index[g] (BK_MCTS_STATE_ROWS).  out_ptr: write the out records there instead
        (memory the device can write; `out` is then ignored)."""
        import torch
        n = roots.shape[0]
        use_tt = tt_keys is not None
        node_cap = nodes.shape[1] // N.MCTS_NODE_DTYPE.itemsize
        rows = mt_state.shape[0] if state_rows else n  # agent rows, or one per search
        if state_rows and rows < zobrist.shape[0]:  # zobrist_index < n_zobrist: every row it names exists
            raise ValueError(f"state_rows: {rows} mt_state rows for {zobrist.shape[0]} zobrist rows")
        tensors = dict(roots=(roots, torch.uint8, (n, 256)), root_sets=(root_sets, torch.uint8, (n, N.FSET_DTYPE.itemsize)),
                       players=(players, torch.uint8, (n,)),
                       zobrist_index=(zobrist_index, torch.int32, (n,)), mt_state=(mt_state, torch.int32, (rows, 625)),
                       nodes=(nodes, torch.uint8, (n, node_cap * N.MCTS_NODE_DTYPE.itemsize)))
        if out_ptr is None:
            tensors.update(out=(out, torch.uint8, (n, N.MCTS_OUT_DTYPE.itemsize)))
        else:
            assert asynchronous and not (chunk or stop_after or resume_from), "out_ptr: one asynchronous launch"
        if root_hash is not None:  # None: ZobristHash.hash_board computed on the device (k_root_hash)
            tensors.update(root_hash=(root_hash, torch.int64, (n,)))
        if use_tt:
            cap = tt_keys.shape[1]
            tensors.update(tt_keys=(tt_keys, torch.int64, (rows, cap)), tt_vals=(tt_vals, torch.float64, (rows, cap)),
                           tt_count=(tt_count, torch.int32, (rows,)))
        if rewards is not None:
            tensors.update(rewards=(rewards, torch.float64, (n, iterations)),
                           hit_flags=(hit_flags, torch.uint8, (n, iterations)))
        for name, (t, dt, shape) in tensors.items():
            _check_device_tensor(t, name, dt, shape, self.device)
        _check_device_tensor(zobrist, "zobrist", torch.int64, (zobrist.shape[0], N.MCTS_ZOBRIST_WORDS), self.device)
        _check_device_tensor(log_table, "log_table", torch.float64, (log_table.shape[0],), self.device)
        self._stream_from_torch()
        d = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        assert not ((chunk or stop_after or resume_from) and time_limit_us), "timed searches run in one launch"
        stops = mcts_chunks(iterations, chunk)
        if stop_after is not None and 0 < stop_after < iterations:
            stops = [x for x in stops if 0 < x < stop_after] + [stop_after]
        if resume_from is not None:  # continue searches a stop_after call left at resume_from
            stops = [x for x in stops if x == 0 or x > resume_from]
        for j, stop in enumerate(stops):
            resume = int(j > 0 or resume_from is not None)
            cfg = N.BkMctsCfg(iterations, max_rollout_moves, float(exploration), int(use_tt), node_cap,
                              tt_keys.shape[1] if use_tt else 0, int(time_limit_us), stop, resume,
                              int(rollout_policy), (N.MCTS_ASYNC if asynchronous else 0) |
                              (N.MCTS_STATE_ROWS if state_rows else 0))
            self.handle.mcts(d(roots), d(root_sets), d(players), d(root_hash), n, cfg, d(zobrist), zobrist.shape[0],
                             d(zobrist_index), d(mt_state), d(tt_keys), d(tt_vals), d(tt_count), d(log_table),
                             log_table.shape[0], d(nodes), d(rewards), d(hit_flags),
                             out_ptr if out_ptr is not None else d(out), N.MEM_DEVICE)
            if on_chunk is not None:
                on_chunk(stop or iterations)
        if asynchronous:
            assert len(stops) == 1, "an asynchronous search is one launch"
            return
        st = out.view(torch.int32)[:, 6] & ~N.MCTS_EUNCERT
        bad = int((st != 0).sum().item())
        if bad:
            raise RuntimeError(f"bk_mcts: {bad} searches stopped early, status bits "
                               f"{sorted(set(st[st != 0].tolist()))[:8]}")


def _stream_base(base: int, n: int) -> int:
    """Philox stream id of a launch's playout 0 (stream ids are uint32 in the kernel)."""
    if base < 0 or base + max(n, 0) > 2**32:
        raise ValueError(f"stream_base {base} + {n} playouts exceeds the uint32 stream ids")
    return int(base)


def _host_root_index(root_index, n_playouts):
    if root_index is None:
        return None
    idx = np.ascontiguousarray(root_index, dtype=np.int32)
    if idx.ndim != 1 or idx.shape[0] < n_playouts:
        raise ValueError(f"root_index: need {n_playouts} entries, got shape {idx.shape}")
    return idx


def _check_device_tensor(t, name, dtype, shape, device):
    """The C-ABI reads raw device pointers: insist on the exact dtype, shape,
    contiguity and device so a mismatch fails here instead of in the kernel."""
    if not t.is_cuda or t.device.index != device:
        raise ValueError(f"{name}: expected a tensor on cuda:{device}, got {t.device}")
    if t.dtype != dtype or tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected {dtype} {tuple(shape)}, got {t.dtype} {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")


def mcts_node_cap(iterations: int) -> int:
    """Node slots one search of `iterations` can need (bk_mcts child-block growth)."""
    return 4 * int(iterations) + 1


def mcts_chunks(iterations: int, chunk: int):
    """cfg.iter_stop per launch: [0] (one launch) or chunk, 2*chunk, ..., iterations."""
    if not chunk or chunk >= iterations:
        return [0]
    return list(range(chunk, iterations, chunk)) + [iterations]


def mcts_log_table(iterations: int) -> np.ndarray:
    """log_table[v] = np.log(v): the exact doubles numpy's log gives UCB1
    (mcts_agent.py:86); index 0 is unused."""
    t = np.zeros(iterations + 2)
    t[1:] = np.log(np.arange(1, iterations + 2, dtype=np.float64))
    return t


class MctsTT:
    """Per-game Zobrist transposition tables for bk_mcts (mcts/zobrist.py:155-220 as
    open addressing: slot = key & (cap - 1), linear probing, NaN value = empty)."""

    def __init__(self, n_games: int, cap: int = 1 << 12):
        assert cap >= 2 and cap & (cap - 1) == 0
        self.keys = np.zeros((n_games, cap), np.uint64)
        self.vals = np.full((n_games, cap), np.nan)
        self.count = np.zeros(n_games, np.int32)

    @property
    def cap(self) -> int:
        return self.keys.shape[1]

    def snapshot(self):
        return self.keys.copy(), self.vals.copy(), self.count.copy()

    def restore(self, snap):
        self.keys, self.vals, self.count = (x.copy() for x in snap)

    def clear(self, g=None):
        sl = slice(None) if g is None else g
        self.keys[sl] = 0
        self.vals[sl] = np.nan
        self.count[sl] = 0

    def items(self, g: int):
        live = ~np.isnan(self.vals[g])
        return self.keys[g][live], self.vals[g][live]

    def load(self, g: int, keys, vals):
        """Replace table g's contents with the given (key, reward) entries."""
        keys = np.asarray(keys, np.uint64)
        while 2 * (len(keys) + 1) > self.cap:
            self.reserve(self.cap)
        self.clear(g)
        _insert(self.keys[g], self.vals[g], keys, np.asarray(vals, np.float64))
        self.count[g] = len(keys)

    def reserve(self, extra: int):
        """Grow (rehash) so every table stays at most half full after `extra` inserts."""
        need = int(self.count.max(initial=0)) + int(extra) + 1
        cap = self.cap
        while need * 2 > cap:
            cap *= 2
        if cap == self.cap:
            return
        n = self.keys.shape[0]
        keys = np.zeros((n, cap), np.uint64)
        vals = np.full((n, cap), np.nan)
        for g in range(n):
            _insert(keys[g], vals[g], *self.items(g))
        self.keys, self.vals = keys, vals


# One lock for every TTPool: agents search from several threads (web-API executor,
# the arena's MCTS worker), and a pool's lease / growth / release and a search's
# gather -> launch -> scatter of its rows must not interleave with another thread's
# (a growth reassigns the pool's tensors).  mcts_agent._search_on_device holds it from
# the row gather until the scattered rows are synchronized.
TT_LOCK = threading.RLock()


class TTPool:
    """Device-resident transposition tables of one capacity (the MctsTT layout in HBM:
    keys int64 / vals float64 [rows, cap], NaN = empty, count int32 [rows]).  An agent
    leases one row (TTRow) and keeps it across select_action calls, so a search never
    moves its table between host and device (mcts/mcts_agent.py:304-341 keeps the TT
    across moves; mcts/zobrist.py:155-220).  One pool per (device, cap): get(); a pool
    whose rows are all released is dropped (its HBM freed).  Thread safety: TT_LOCK."""

    _pools: dict = {}

    def __init__(self, device: int, cap: int, rows: int = 64):
        import torch
        assert cap >= 2 and cap & (cap - 1) == 0
        self.device, self.cap = device, cap
        dev = f"cuda:{device}"
        self.keys = torch.zeros((rows, cap), dtype=torch.int64, device=dev)
        self.vals = torch.full((rows, cap), float("nan"), dtype=torch.float64, device=dev)
        self.count = torch.zeros(rows, dtype=torch.int32, device=dev)
        self.free = list(range(rows - 1, -1, -1))

    @classmethod
    def get(cls, device: int, cap: int) -> "TTPool":
        with TT_LOCK:
            key = (device, cap)
            if key not in cls._pools:
                cls._pools[key] = TTPool(device, cap)
            return cls._pools[key]

    def lease(self) -> "TTRow":
        import torch
        with TT_LOCK:
            if not self.free:  # double the rows (new rows empty)
                n = self.keys.shape[0]
                # the old tensors may still be read by this thread's queued work: the
                # copies are ordered after it on this stream, and the old storage is
                # freed by the caching allocator only after that stream's use
                self.keys = torch.cat([self.keys, torch.zeros_like(self.keys)])
                self.vals = torch.cat([self.vals, torch.full_like(self.vals, float("nan"))])
                self.count = torch.cat([self.count, torch.zeros_like(self.count)])
                self.free = list(range(2 * n - 1, n - 1, -1))
            return TTRow(self, self.free.pop())

    def release(self, row: int):
        import torch
        with TT_LOCK:
            self.keys[row] = 0
            self.vals[row] = float("nan")
            self.count[row] = 0
            self.free.append(row)
            torch.cuda.current_stream(self.keys.device).synchronize()  # visible to every thread's stream
            if len(self.free) == self.keys.shape[0] and TTPool._pools.get((self.device, self.cap)) is self:
                del TTPool._pools[(self.device, self.cap)]  # no row leased: free the pool's HBM


class TTRow:
    """One agent's table: a row of a TTPool.  count mirrors the device count after
    each search; items(0) / cap match MctsTT's single-table accessors."""

    def __init__(self, pool: TTPool, row: int):
        import weakref
        self.pool, self.row, self.count = pool, row, np.zeros(1, np.int32)
        self._fin = weakref.finalize(self, pool.release, row)
        self._fin.atexit = False  # no device work while the interpreter shuts down

    @property
    def cap(self) -> int:
        return self.pool.cap

    def items(self, g: int = 0):
        assert g == 0
        keys = self.pool.keys[self.row].cpu().numpy().view(np.uint64)
        vals = self.pool.vals[self.row].cpu().numpy()
        live = ~np.isnan(vals)
        return keys[live], vals[live]

    def load(self, keys, vals):
        """Replace the row's contents with the given (key, reward) entries."""
        import torch
        tk = np.zeros(self.cap, np.uint64)
        tv = np.full(self.cap, np.nan)
        _insert(tk, tv, np.asarray(keys, np.uint64), np.asarray(vals, np.float64))
        dev = self.pool.keys.device
        self.pool.keys[self.row] = torch.from_numpy(tk.view(np.int64)).to(dev)
        self.pool.vals[self.row] = torch.from_numpy(tv).to(dev)
        self.pool.count[self.row] = len(keys)
        self.count[0] = len(keys)

    def release(self):
        self._fin()


def _insert(tkeys: np.ndarray, tvals: np.ndarray, k: np.ndarray, v: np.ndarray) -> None:
    """Linear-probing inserts of distinct keys into one table row (NaN = empty slot):
    each round places one key per free slot, the others probe on."""
    cap = len(tkeys)
    slot = (k & np.uint64(cap - 1)).astype(np.int64)
    todo = np.arange(len(k))
    while len(todo):
        cand = slot[todo]
        free = np.isnan(tvals[cand])
        _, first = np.unique(cand, return_index=True)
        win = np.zeros(len(todo), bool)
        win[first] = True
        win &= free
        tkeys[cand[win]] = k[todo[win]]
        tvals[cand[win]] = v[todo[win]]
        rest = todo[~win]
        slot[rest] = (slot[rest] + 1) % cap
        todo = rest


def empty_state() -> np.ndarray:
    """The initial position (engine/board.py:54-78): nobody has moved, RED to play."""
    s = np.zeros(1, dtype=STATE_DTYPE)
    s["first_move"] = 0xF
    return s


def winners(results) -> np.ndarray:
    """winner_ids as a 4-bit mask per playout (GameResult.winner_ids)."""
    return np.asarray(results["winner_mask"])
