"""ctypes binding of the HIP C-ABI (include/blokus_hip.h).

The shared library is built in-tree (``_lib/libblokus_hip.so``) by
``reinforcementlearning_blokus_amd.build.build_native()`` / ``__graft_entry__.build()``.
There is no CPU fallback: if the library or a GPU is missing, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# BK_LIB_PATH: load an alternative in-tree build (kernel tuning experiments)
LIB_PATH = os.environ.get("BK_LIB_PATH") or os.path.join(_HERE, "_lib", "libblokus_hip.so")

OK, EINVAL, EHIP, ENOMEM, EOVERFLOW, ECHECK = 0, -1, -2, -3, -4, -5
STATUS_CAP, STATUS_UNCERT, STATUS_STOP, STATUS_BADFORCE = 8, 16, 32, 64  # bk_result.status bits
FORCE_INDEX = 0x40000000  # bk_arena_step forced[i]: the k-th entry of the legal list (BK_FORCE_INDEX | k)
FORCE_SKIP = -2  # bk_arena_step forced[i]: leave game i untouched (its search is in flight)
MEM_HOST, MEM_DEVICE = 0, 1
SEM_ARENA, SEM_ROLLOUT, SEM_ADVANCE = 0, 1, 2
ORDER_NAIVE, ORDER_FRONTIER = 0, 1
RNG_PHILOX, RNG_NUMPY_MT = 0, 1
N_ORIENTS = 91
STREAM_OWN = (1 << 64) - 1  # BK_STREAM_OWN

# every symbol include/blokus_hip.h declares
EXPORTS = (
    "bk_abi_version", "bk_tables_version", "bk_create", "bk_destroy", "bk_set_stream", "bk_stream_create",
    "bk_synchronize", "bk_last_error", "bk_orient_info", "bk_movegen", "bk_movegen_mask", "bk_has_moves",
    "bk_rollout", "bk_advance", "bk_fastmcts", "bk_last_kernel_ms", "bk_last_kernel",
    "bk_fset_init", "bk_fset_place", "bk_fset_copy", "bk_fset_list", "bk_rollout_frontier",
    "bk_mcts", "bk_debug_sections", "bk_pow_half_fix", "bk_debug_fastmcts_select", "bk_arena_advance",
    "bk_arena_step", "bk_mt_cursor_init", "bk_set_tuning", "bk_get_tuning", "bk_debug_fset_op",
    "bk_debug_mcts_failure", "bk_mcts_set_done", "bk_host_alloc", "bk_host_free",
)
# bk_debug_mcts_failure record (include/blokus_hip.h BK_DIAG_*)
DIAG_WORDS = 64
DIAG_KERNELS = ("k_mcts", "k_mcts_pair", "k_mcts_h", "k_mcts_coop", "k_mcts_coop_h")
# bk_set_tuning keys (include/blokus_hip.h BK_TUNE_*), by the environment variable name
# bk_create reads each from once
TUNE_KEYS = {name: i for i, name in enumerate((
    "BK_MG_GROUPS", "BK_MG_STAGE", "BK_MG_PARTS", "BK_MG_PART_WAVES", "BK_DEBUG_MAX_ITERS", "BK_HANDOUT",
    "BK_MCTS_COOP", "BK_COOP_BLOCKS_PER_CU", "BK_MCTS_SPREAD", "BK_TREE_BATCH", "BK_COOP_WALK", "BK_COOP_BAL",
    "BK_MCTS_PAIR"))}
FSET_SLOTS = 256
# bk_fset: the 4 players' CPython frontier-set tables (include/blokus_hip.h)
FSET_DTYPE = np.dtype([("key", "<i2", (4, FSET_SLOTS)), ("mask", "<u2", (4,)), ("fill", "<u2", (4,)),
                       ("used", "<u2", (4,)), ("reserved", "<u2", (4,))])
assert FSET_DTYPE.itemsize == 2080
FASTMCTS_TOP = 10
FASTMCTS_MAX_CHILDREN = 2048


class NativeUnavailable(RuntimeError):
    """The HIP library is not built / cannot be loaded / no GPU.  Never silently bypassed."""


class BkState(C.Structure):
    _fields_ = [("planes", (C.c_uint64 * 7) * 4), ("used", C.c_uint32 * 4), ("first_move", C.c_uint8),
                ("current_player", C.c_uint8), ("out_mask", C.c_uint8), ("flags", C.c_uint8),
                ("move_count", C.c_uint16), ("reserved16", C.c_uint16), ("reserved", C.c_uint32 * 2)]


class BkResult(C.Structure):
    _fields_ = [("scores", C.c_int16 * 4), ("winner_mask", C.c_uint8), ("status", C.c_uint8),
                ("plies", C.c_uint16), ("passes", C.c_uint16), ("turns", C.c_uint16),
                ("reward", C.c_int32), ("draws", C.c_uint32), ("reserved", C.c_uint32 * 2)]


class BkRolloutCfg(C.Structure):
    _fields_ = [("semantics", C.c_int32), ("order", C.c_int32), ("rng", C.c_int32), ("max_plies", C.c_int32),
                ("seed", C.c_uint64), ("seats_share_stream", C.c_int32), ("heuristic_seats", C.c_int32),
                ("stream_base", C.c_uint32), ("reserved", C.c_int32)]


class BkFastMctsOut(C.Structure):
    _fields_ = [("best_index", C.c_int32), ("iterations", C.c_int32), ("n_children", C.c_int32),
                ("n_top", C.c_int32), ("top_index", C.c_int32 * 10), ("top_visits", C.c_int32 * 10),
                ("top_q", C.c_double * 10)]


assert C.sizeof(BkFastMctsOut) == 176
FASTMCTS_OUT_DTYPE = np.dtype([("best_index", "<i4"), ("iterations", "<i4"), ("n_children", "<i4"),
                               ("n_top", "<i4"), ("top_index", "<i4", (10,)), ("top_visits", "<i4", (10,)),
                               ("top_q", "<f8", (10,))])
assert FASTMCTS_OUT_DTYPE.itemsize == 176
assert C.sizeof(BkState) == 256 and C.sizeof(BkResult) == 32 and C.sizeof(BkRolloutCfg) == 40


class BkMctsCfg(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("max_rollout_moves", C.c_int32), ("exploration", C.c_double),
                ("use_tt", C.c_int32), ("node_cap", C.c_int32), ("tt_cap", C.c_int32),
                ("time_limit_us", C.c_int32), ("iter_stop", C.c_int32), ("resume", C.c_int32),
                ("rollout_policy", C.c_int32), ("flags", C.c_int32)]
MCTS_ASYNC = 1  # bk_mcts_cfg.flags: enqueue only (device buffers)
MCTS_STATE_ROWS = 2  # bk_mcts_cfg.flags: mt / tt rows indexed by zobrist_index (agent rows, in place)


assert C.sizeof(BkMctsCfg) == 48
MCTS_NODE_DTYPE = np.dtype([("total", "<f8"), ("visits", "<u4"), ("child0", "<i4"), ("move", "<u2"),
                            ("n_exp", "<u2"), ("n_legal", "<u2"), ("flags", "<u2")])
assert MCTS_NODE_DTYPE.itemsize == 24
MCTS_OUT_DTYPE = np.dtype([("best_move", "<i4"), ("iterations_run", "<i4"), ("tt_hits", "<i4"),
                           ("rollouts", "<i4"), ("nodes_used", "<i4"), ("root_children", "<i4"),
                           ("status", "<u4"), ("rollout_plies", "<i4")])
assert MCTS_OUT_DTYPE.itemsize == 32
MCTS_ZOBRIST_WORDS = 2088
MCTS_MAX_DEPTH = 63
MCTS_EPOOL, MCTS_EFSET, MCTS_ETT, MCTS_EPATH, MCTS_ELOG, MCTS_EINTERNAL, MCTS_EUNCERT = 1, 2, 4, 8, 16, 32, 64
MCTS_ROLLOUT_RANDOM, MCTS_ROLLOUT_HEURISTIC = 0, 1

# numpy views of the same records

STATE_DTYPE = np.dtype([("planes", "<u8", (4, 7)), ("used", "<u4", (4,)), ("first_move", "u1"),
                        ("current_player", "u1"), ("out_mask", "u1"), ("flags", "u1"),
                        ("move_count", "<u2"), ("reserved16", "<u2"), ("reserved", "<u4", (2,))])
STOP_DTYPE = np.dtype([("n_legal", "<i4"), ("quick_index", "<i4"), ("quick_reward", "<f8")])  # bk_stop_info
RESULT_DTYPE = np.dtype([("scores", "<i2", (4,)), ("winner_mask", "u1"), ("status", "u1"),
                         ("plies", "<u2"), ("passes", "<u2"), ("turns", "<u2"), ("reward", "<i4"),
                         ("draws", "<u4"), ("reserved", "<u4", (2,))])
assert STATE_DTYPE.itemsize == 256 and RESULT_DTYPE.itemsize == 32

ABI_VERSION = 7  # include/blokus_hip.h BK_ABI_VERSION
_lib = None
_lock = threading.Lock()


def load():
    """Load libblokus_hip.so and declare the C signatures.  Raises NativeUnavailable."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        # One HIP runtime per process.  torch bundles its own libamdhip64 (+ HSA runtime)
        # with the same soname as /opt/rocm's (libamdhip64.so.7).  Loaded after torch,
        # this library binds torch's copy; loaded before, torch later pulls in a second
        # runtime that finds no GPU ("No HIP GPUs are available"), measured with
        # tools/runtime_order_probe.py.  A plain import touches no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        try:
            L = C.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - environment specific
            raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        L.bk_abi_version.restype, L.bk_abi_version.argtypes = C.c_int, []
        if L.bk_abi_version() != ABI_VERSION:
            raise NativeUnavailable(f"{LIB_PATH} has ABI {L.bk_abi_version()}, this package needs {ABI_VERSION}: "
                                    "rebuild it (__graft_entry__.build())")
        P, vp = C.POINTER, C.c_void_p
        sigs = {
            "bk_abi_version": (C.c_int, []),
            "bk_tables_version": (C.c_int, []),
            "bk_create": (C.c_int, [C.c_int, C.c_uint32, P(vp)]),
            "bk_destroy": (C.c_int, [vp]),
            "bk_set_stream": (C.c_int, [vp, vp]),
            "bk_stream_create": (C.c_int, [vp, vp, C.c_int32, C.POINTER(C.c_void_p)]),
            "bk_synchronize": (C.c_int, [vp]),
            "bk_last_error": (C.c_int, [vp, C.c_char_p, C.c_size_t]),
            "bk_orient_info": (C.c_int, [C.c_int, P(C.c_int32), P(C.c_int32), P(C.c_int32), P(C.c_int32)]),
            "bk_movegen": (C.c_int, [vp, vp, vp, C.c_int32, vp, vp, C.c_int]),
            "bk_movegen_mask": (C.c_int, [vp, vp, vp, C.c_int32, vp, vp, C.c_int]),
            "bk_has_moves": (C.c_int, [vp, vp, C.c_int32, vp, C.c_int]),
            "bk_rollout": (C.c_int, [vp, vp, C.c_int32, vp, C.c_int32, P(BkRolloutCfg), vp, vp, C.c_int]),
            "bk_advance": (C.c_int, [vp, vp, C.c_int32, vp, C.c_int32, P(BkRolloutCfg), vp, vp, C.c_int]),
            "bk_fastmcts": (C.c_int, [vp, C.c_int32, vp, vp, vp, vp, vp, C.c_int32, vp, vp, C.c_int32, C.c_double,
                                      vp, vp, C.c_int]),
            "bk_pow_half_fix": (C.c_int, [vp, C.c_int32, vp, vp, C.c_int32, P(C.c_int32)]),
            "bk_arena_advance": (C.c_int, [vp, vp, vp, C.c_int32, P(BkRolloutCfg), vp, vp, vp, C.c_int]),
            "bk_arena_step": (C.c_int, [vp, vp, vp, C.c_int32, P(BkRolloutCfg), vp, vp, vp, vp, vp, vp, C.c_int]),
            "bk_mt_cursor_init": (C.c_int, [C.c_uint32, vp]),
            "bk_debug_fastmcts_select": (C.c_int, [vp, C.c_int32, vp, vp, C.c_uint32, vp, C.c_int32, vp, vp,
                                                   C.c_int32, C.c_double, P(C.c_int32)]),
            "bk_last_kernel_ms": (C.c_int, [vp, P(C.c_float)]),
            "bk_last_kernel": (C.c_char_p, [vp]),
            "bk_fset_init": (C.c_int, [vp]),
            "bk_fset_place": (C.c_int, [vp, vp, C.c_int32, vp, C.c_int32]),
            "bk_fset_copy": (C.c_int, [vp, vp]),
            "bk_fset_list": (C.c_int, [vp, C.c_int32, vp, C.c_int32]),
            "bk_rollout_frontier": (C.c_int, [vp, vp, vp, C.c_int32, vp, C.c_int32, P(BkRolloutCfg), vp, vp, vp,
                                              vp, C.c_int]),
            "bk_mcts": (C.c_int, [vp, vp, vp, vp, vp, C.c_int32, P(BkMctsCfg), vp, C.c_int32, vp, vp, vp, vp,
                                  vp, vp, C.c_int32, vp, vp, vp, vp, C.c_int]),
            "bk_debug_sections": (C.c_int, [vp, vp, C.c_int32, C.c_int32]),
            "bk_set_tuning": (C.c_int, [vp, C.c_int32, C.c_int64]),
            "bk_debug_fset_op": (C.c_int, [vp, C.c_int32, C.c_int32, C.c_int32]),
            "bk_debug_mcts_failure": (C.c_int, [vp, vp, C.c_int32]),
            "bk_get_tuning": (C.c_int, [vp, C.c_int32, P(C.c_int64)]),
            "bk_mcts_set_done": (C.c_int, [vp, vp]),
            "bk_host_alloc": (C.c_void_p, [C.c_size_t]),
            "bk_host_free": (C.c_int, [vp]),
        }
        for name, (res, args) in sigs.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
        return L


class HostBuffer:
    """Pinned, device-mapped, coherent host memory (bk_host_alloc): the device writes it
    at the same address while the host reads it through `array` (a numpy view)."""

    def __init__(self, nbytes: int, dtype=np.uint8):
        L = load()
        self._L = L
        self.nbytes = int(nbytes)
        self.ptr = L.bk_host_alloc(self.nbytes)
        if not self.ptr:
            raise MemoryError(f"bk_host_alloc({self.nbytes}) failed")
        raw = (C.c_uint8 * self.nbytes).from_address(self.ptr)
        self.array = np.frombuffer(raw, dtype=np.uint8).view(dtype)

    def close(self):
        if self.ptr:
            self.array = None
            self._L.bk_host_free(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


def orient_table():
    """[(piece_id, orientation, [(dr, dc), ...])] for g = 0..90 (host-side table query)."""
    L = load()
    out = []
    for g in range(N_ORIENTS):
        pid, o, n = C.c_int32(), C.c_int32(), C.c_int32()
        offs = (C.c_int32 * 10)()
        if L.bk_orient_info(g, C.byref(pid), C.byref(o), C.byref(n), offs) != OK:
            raise NativeUnavailable("bk_orient_info failed")
        out.append((pid.value, o.value, [(offs[2 * k], offs[2 * k + 1]) for k in range(n.value)]))
    return out


# FastMCTS UCB bit-exact for searches of up to 65,536 iterations (a 65,537-row table takes
# ~7 s to build once per process and 7 MB; an arena seat at thinking_time_ms=1000 and the
# default iterations_per_ms=20 needs 20,001 rows).  Beyond it gpu.fastmcts warns.
POW_FIX_ROWS = 65537
_POW_FIX = {"lt": np.zeros(0), "off": np.zeros(1, np.int32), "ent": np.zeros(0, np.int32)}


def pow_half_fix(log_table: np.ndarray, rows: int | None = None, cached_only: bool = False):
    """(offsets int32[rows+1], entries int32[k]) of bk_pow_half_fix: the (N, v), N < rows,
    where CPython's (2*log(N)/v) ** 0.5 (libm pow) differs from sqrt by one ulp.
    rows defaults to min(len(log_table), POW_FIX_ROWS).  Host only (no GPU).  The largest
    table built so far is kept; a smaller request is its prefix.  cached_only: never
    build, return at most what is cached (for wall-clock-bounded searches, whose
    iteration count -- hence reference parity -- depends on timing anyway)."""
    lt = np.ascontiguousarray(log_table, dtype=np.float64)
    rows = min(len(lt), POW_FIX_ROWS) if rows is None else min(int(rows), len(lt), POW_FIX_ROWS)
    c = _POW_FIX
    have = len(c["off"]) - 1
    if have < rows and cached_only:
        rows = have
    if have >= rows and np.array_equal(c["lt"][:rows], lt[:rows]):
        off = c["off"][: rows + 1]
        return off, c["ent"][: int(off[-1])]
    L = load()
    off = np.zeros(rows + 1, np.int32)
    cap = max(64, rows * 8)
    while True:
        ent = np.zeros(cap, np.int32)
        k = C.c_int32()
        rc = L.bk_pow_half_fix(lt.ctypes.data, rows, off.ctypes.data, ent.ctypes.data, cap, C.byref(k))
        if rc == EOVERFLOW:
            cap = int(k.value)
            continue
        if rc != OK:
            raise RuntimeError(f"bk_pow_half_fix failed ({rc})")
        break
    ent = ent[: k.value].copy()
    if rows >= have:
        c.update(lt=lt[:rows].copy(), off=off, ent=ent)
    return off, ent


def mt_cursors(seeds) -> np.ndarray:
    """uint32[len(seeds), 4]: bk_mt_cursor_init of each numpy RandomState seed."""
    L = load()
    seeds = np.asarray(seeds, dtype=np.uint32).reshape(-1)
    out = np.zeros((len(seeds), 4), np.uint32)
    for i, sd in enumerate(seeds.tolist()):
        L.bk_mt_cursor_init(sd, out[i].ctypes.data)
    return out


def fset_new(n: int = 1) -> np.ndarray:
    """n bk_fset records initialised as Board() does (each set = {start corner})."""
    L = load()
    out = np.zeros(n, dtype=FSET_DTYPE)
    for i in range(n):
        if L.bk_fset_init(out[i:i + 1].ctypes.data) != OK:
            raise RuntimeError("bk_fset_init failed")
    return out


def fset_place(fs: np.ndarray, after_state: np.ndarray, player: int, cells) -> None:
    """Frontier update of place_piece (engine/board.py:315-367) on record fs (1 element),
    given the packed board after the move and the placed cells (r*20+c, in order)."""
    L = load()
    c = np.ascontiguousarray(cells, dtype=np.int32)
    rc = L.bk_fset_place(fs.ctypes.data, after_state.ctypes.data, int(player), c.ctypes.data, len(c))
    if rc != OK:
        raise RuntimeError(f"bk_fset_place failed ({rc})")


def fset_copy(dst: np.ndarray, src: np.ndarray) -> None:
    if load().bk_fset_copy(dst.ctypes.data, src.ctypes.data) != OK:
        raise RuntimeError("bk_fset_copy failed")


def fset_list(fs: np.ndarray, player: int) -> list:
    """Iteration order of player's frontier set (cells r*20+c)."""
    buf = np.zeros(FSET_SLOTS, dtype=np.int32)
    n = load().bk_fset_list(fs.ctypes.data, int(player), buf.ctypes.data, FSET_SLOTS)
    if n < 0:
        raise RuntimeError("bk_fset_list failed")
    return buf[:n].tolist()


class Handle:
    """One bk_handle: a HIP stream + scratch on one device.  Use one per host thread."""

    def __init__(self, device: int = 0):
        L = load()
        h = C.c_void_p()
        rc = L.bk_create(device, 0, C.byref(h))
        if rc != OK or not h.value:
            raise NativeUnavailable(f"bk_create(device={device}) failed with {rc} (no usable GPU?)")
        self._L, self._h, self.device = L, h, device
        self._lock = threading.Lock()

    def close(self):
        if self._h is not None and self._h.value:
            self._L.bk_destroy(self._h)
        self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def ptr(self):
        return self._h

    def error(self) -> str:
        buf = C.create_string_buffer(512)
        self._L.bk_last_error(self._h, buf, 512)
        return buf.value.decode(errors="replace")

    def check(self, rc: int, what: str):
        if rc != OK:
            raise RuntimeError(f"{what} failed ({rc}): {self.error()}")

    def set_stream(self, stream_ptr: int | None):
        """stream_ptr: a hipStream_t value (0 = null stream) or None for the handle's own."""
        v = STREAM_OWN if stream_ptr is None else stream_ptr
        self.check(self._L.bk_set_stream(self._h, C.c_void_p(v)), "bk_set_stream")

    def stream_create(self, cu_mask=None) -> int:
        """A new stream owned by this handle (bk_stream_create); cu_mask: uint32 words,
        bit i = compute unit i allowed (None = all).  Returns the hipStream_t value."""
        out = C.c_void_p()
        if cu_mask is None:
            rc = self._L.bk_stream_create(self._h, None, 0, C.byref(out))
        else:
            m = np.ascontiguousarray(cu_mask, dtype=np.uint32)
            rc = self._L.bk_stream_create(self._h, m.ctypes.data, len(m), C.byref(out))
        self.check(rc, "bk_stream_create")
        return int(out.value)

    def synchronize(self):
        self.check(self._L.bk_synchronize(self._h), "bk_synchronize")

    def set_done(self, ptr: int | None):
        """bk_mcts_set_done: later bk_mcts launches on this handle store search g's result
        word in done[g] as it finishes (ptr: a uint64 array the device can write, e.g. a
        HostBuffer); None turns it off."""
        self.check(self._L.bk_mcts_set_done(self._h, C.c_void_p(ptr or 0)), "bk_mcts_set_done")

    def mcts_failure(self):
        """The handle's bk_mcts failure record (bk_debug_mcts_failure) as a dict, or None if
        no search on it ever broke a tree invariant."""
        w = (C.c_uint32 * DIAG_WORDS)()
        rc = self._L.bk_debug_mcts_failure(self._h, w, DIAG_WORDS)
        if rc < 0:
            self.check(rc, "bk_debug_mcts_failure")
        if rc == 0:
            return None
        w = list(w)
        kern = DIAG_KERNELS[w[1]] if w[1] < len(DIAG_KERNELS) else w[1]
        if w[0] == 0x200:  # BK_DIAG_DOUBLE_START
            return {"reason": "DOUBLE_START", "kernel": kern, "launch": w[2], "game_in_launch": w[3],
                    "handout_counter": w[12], "handed": w[17], "block": w[18], "wave": w[19], "hw_id": w[20],
                    "n_games": w[21]}
        np_ = min(int(w[16]), 22)
        return {"reason": {16: "ELOG", 32: "EINTERNAL"}.get(w[0], w[0]),
                "kernel": kern, "launch": w[2],
                "game_in_launch": w[3], "node": w[4], "visits": w[5], "n_exp": w[6], "n_legal": w[7],
                "child0": C.c_int32(w[8]).value, "iterations_done": w[9], "depth": w[10], "log_len": w[11],
                "handout_counter": w[12], "node_cap": w[13], "nodes_used": w[14], "iterations": w[15],
                "path": w[18:18 + np_], "path_visits": w[40:40 + np_]}

    def set_tuning(self, name: str, value: int | None):
        """bk_set_tuning by environment-variable name (TUNE_KEYS); None = automatic."""
        self.check(self._L.bk_set_tuning(self._h, TUNE_KEYS[name], -1 if value is None else int(value)),
                   "bk_set_tuning")

    def get_tuning(self, name: str) -> int | None:
        v = C.c_int64()
        self.check(self._L.bk_get_tuning(self._h, TUNE_KEYS[name], C.byref(v)), "bk_get_tuning")
        return None if v.value < 0 else int(v.value)

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        self.check(self._L.bk_last_kernel_ms(self._h, C.byref(ms)), "bk_last_kernel_ms")
        return float(ms.value)

    def last_kernel(self) -> str:
        """Name of the kernel the last timed call launched (bk_last_kernel)."""
        return (self._L.bk_last_kernel(self._h) or b"").decode()

    # -- hot path -------------------------------------------------------------------
    def movegen(self, states_ptr, players_ptr, n, rows_ptr, count_ptr, mem):
        with self._lock:
            rc = self._L.bk_movegen(self._h, C.c_void_p(states_ptr), C.c_void_p(players_ptr), n,
                                    C.c_void_p(rows_ptr or 0), C.c_void_p(count_ptr or 0), mem)
        self.check(rc, "bk_movegen")

    def movegen_mask(self, states_ptr, players_ptr, n, mask_ptr, count_ptr, mem):
        with self._lock:
            rc = self._L.bk_movegen_mask(self._h, C.c_void_p(states_ptr), C.c_void_p(players_ptr), n,
                                         C.c_void_p(mask_ptr or 0), C.c_void_p(count_ptr or 0), mem)
        self.check(rc, "bk_movegen_mask")

    def has_moves(self, states_ptr, n, out_ptr, mem):
        with self._lock:
            rc = self._L.bk_has_moves(self._h, C.c_void_p(states_ptr), n, C.c_void_p(out_ptr), mem)
        self.check(rc, "bk_has_moves")

    def rollout(self, roots_ptr, n_roots, index_ptr, n_playouts, cfg: BkRolloutCfg, seeds_ptr, out_ptr, mem):
        with self._lock:
            rc = self._L.bk_rollout(self._h, C.c_void_p(roots_ptr), n_roots, C.c_void_p(index_ptr or 0),
                                    n_playouts, C.byref(cfg), C.c_void_p(seeds_ptr or 0), C.c_void_p(out_ptr), mem)
        self.check(rc, "bk_rollout")

    def fastmcts(self, n_games, offset_ptr, iters_ptr, base_ptr, mt_ptr, log_ptr, log_len, fix_off_ptr, fix_ent_ptr,
                 fix_len, c, out_ptr, visits_ptr, mem):
        with self._lock:
            rc = self._L.bk_fastmcts(self._h, n_games, C.c_void_p(offset_ptr), C.c_void_p(iters_ptr),
                                     C.c_void_p(base_ptr), C.c_void_p(mt_ptr), C.c_void_p(log_ptr), log_len,
                                     C.c_void_p(fix_off_ptr), C.c_void_p(fix_ent_ptr or None), fix_len,
                                     float(c), C.c_void_p(out_ptr), C.c_void_p(visits_ptr or None), mem)
        self.check(rc, "bk_fastmcts")

    def debug_fastmcts_select(self, n, visits_ptr, totals_ptr, root_visits, log_ptr, log_len, fix_off_ptr,
                              fix_ent_ptr, fix_len, c) -> int:
        best = C.c_int32(-1)
        with self._lock:
            rc = self._L.bk_debug_fastmcts_select(self._h, n, C.c_void_p(visits_ptr), C.c_void_p(totals_ptr),
                                                  root_visits, C.c_void_p(log_ptr), log_len, C.c_void_p(fix_off_ptr),
                                                  C.c_void_p(fix_ent_ptr or None), fix_len, float(c), C.byref(best))
        self.check(rc, "bk_debug_fastmcts_select")
        return best.value

    def rollout_frontier(self, roots_ptr, sets_ptr, n_roots, index_ptr, n_playouts, cfg: BkRolloutCfg, seeds_ptr,
                         out_ptr, states_ptr, osets_ptr, mem):
        with self._lock:
            rc = self._L.bk_rollout_frontier(self._h, C.c_void_p(roots_ptr), C.c_void_p(sets_ptr), n_roots,
                                             C.c_void_p(index_ptr or 0), n_playouts, C.byref(cfg),
                                             C.c_void_p(seeds_ptr or 0), C.c_void_p(out_ptr or 0),
                                             C.c_void_p(states_ptr or 0), C.c_void_p(osets_ptr or 0), mem)
        self.check(rc, "bk_rollout_frontier")

    def mcts(self, roots_ptr, sets_ptr, players_ptr, hash_ptr, n_games, cfg: BkMctsCfg, zob_ptr, n_zob, zidx_ptr,
             mt_ptr, ttk_ptr, ttv_ptr, ttc_ptr, log_ptr, log_len, nodes_ptr, rewards_ptr, flags_ptr, out_ptr, mem):
        v = lambda x: C.c_void_p(x or 0)  # noqa: E731
        with self._lock:
            rc = self._L.bk_mcts(self._h, v(roots_ptr), v(sets_ptr), v(players_ptr), v(hash_ptr), n_games,
                                 C.byref(cfg), v(zob_ptr), n_zob, v(zidx_ptr), v(mt_ptr), v(ttk_ptr), v(ttv_ptr),
                                 v(ttc_ptr), v(log_ptr), log_len, v(nodes_ptr), v(rewards_ptr), v(flags_ptr),
                                 v(out_ptr), mem)
        self.check(rc, "bk_mcts")

    def arena_advance(self, states_ptr, sets_ptr, n, cfg: BkRolloutCfg, masks_ptr, rng_ptr, out_ptr, mem):
        with self._lock:
            rc = self._L.bk_arena_advance(self._h, C.c_void_p(states_ptr), C.c_void_p(sets_ptr), n, C.byref(cfg),
                                          C.c_void_p(masks_ptr), C.c_void_p(rng_ptr), C.c_void_p(out_ptr), mem)
        self.check(rc, "bk_arena_advance")

    def arena_step(self, states_ptr, sets_ptr, n, cfg: BkRolloutCfg, masks_ptr, quick_ptr, forced_ptr, rng_ptr,
                   out_ptr, stop_ptr, mem):
        with self._lock:
            rc = self._L.bk_arena_step(self._h, C.c_void_p(states_ptr), C.c_void_p(sets_ptr), n, C.byref(cfg),
                                       C.c_void_p(masks_ptr), C.c_void_p(quick_ptr), C.c_void_p(forced_ptr),
                                       C.c_void_p(rng_ptr), C.c_void_p(out_ptr), C.c_void_p(stop_ptr), mem)
        self.check(rc, "bk_arena_step")

    def advance(self, roots_ptr, n_roots, index_ptr, n, cfg: BkRolloutCfg, seeds_ptr, out_ptr, mem):
        with self._lock:
            rc = self._L.bk_advance(self._h, C.c_void_p(roots_ptr), n_roots, C.c_void_p(index_ptr or 0), n,
                                    C.byref(cfg), C.c_void_p(seeds_ptr or 0), C.c_void_p(out_ptr), mem)
        self.check(rc, "bk_advance")


_default = {}


def default_handle(device: int = 0) -> Handle:
    key = (threading.get_ident(), device)
    h = _default.get(key)
    if h is None:
        h = Handle(device)
        _default[key] = h
    return h
