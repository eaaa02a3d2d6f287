/*
 * blokus_hip.h -- C ABI of the MI355X-native Blokus hot path.
 *
 * The reference (TGALLOWAY1/ReinforcementLearning_Blokus) is pure Python and has
 * no FFI; its hot path is reached through Python calls.  Every entry point below
 * names the reference function it replaces (file:line in the reference tree).
 * The Python host layer `reinforcementlearning_blokus_amd` binds these symbols
 * with ctypes (see INTEGRATION.md for the binding a maintainer would add).
 *
 * Conventions
 *   - plain C types only; no torch / HIP types in the signatures
 *   - every call returns int status: 0 = ok, < 0 = error (bk_last_error has text)
 *   - buffers are caller-owned; `mem` says whether pointers are host or device
 *   - a handle owns one HIP stream (or borrows the caller's) plus scratch; use one
 *     handle per host thread (the library never calls exit()).
 */
#ifndef BLOKUS_HIP_H
#define BLOKUS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BK_ABI_VERSION 7
#define BK_BOARD 20
#define BK_CELLS 400
#define BK_PLAYERS 4
#define BK_PIECES 21
#define BK_ORIENTS 91   /* ALL_PIECE_ORIENTATIONS total, engine/pieces.py:257 */
#define BK_MASK_WORDS 7 /* 400 bits as 7 x u64, bit = r*20+c (engine/bitboard.py:19) */

/* Status codes */
#define BK_OK 0
#define BK_EINVAL -1
#define BK_EHIP -2
#define BK_ENOMEM -3
#define BK_EOVERFLOW -4
#define BK_ECHECK -5 /* a device-side consistency check failed (bk_debug_mcts_failure, ABI 6) */

/* Pointer residency for buffer arguments */
#define BK_MEM_HOST 0
#define BK_MEM_DEVICE 1

/*
 * Packed game state: 256 bytes, POD, little-endian.
 * Mirrors engine/board.py:54-78 (Board.__init__): player_bits[p] as 400-bit
 * little-endian integers, player_pieces_used, player_first_move, current_player,
 * move_count.  Frontier sets are NOT part of the state: the legal-move SET does
 * not depend on them, only the reference list ORDER does, and the
 * host orders results with the live frontier (bk_movegen returns dense masks).
 */
typedef struct bk_state {
    uint64_t planes[BK_PLAYERS][BK_MASK_WORDS]; /* 224 B: Board.player_bits[p]            */
    uint32_t used[BK_PLAYERS];                  /*  16 B: bit (piece_id-1) = piece used     */
    uint8_t first_move;     /* bit p: Board.player_first_move[p] (engine/board.py:65)        */
    uint8_t current_player; /* 0..3 = Player.value-1 (engine/board.py:18-23)                 */
    uint8_t out_mask;       /* bit p: p is known to have no legal move (monotone, may be 0)  */
    uint8_t flags;          /* reserved, 0                                                   */
    uint16_t move_count;    /* Board.move_count                                              */
    uint16_t reserved16;
    uint32_t reserved[2];
} bk_state;

/* Playout semantics */
#define BK_SEM_ARENA 0  /* B: pass when stuck, terminal when nobody can move;
                           analytics/tournament/arena_runner.py:652-697 + engine/game.py:182-349 */
#define BK_SEM_ROLLOUT 1 /* A: MCTSAgent._rollout, mcts/mcts_agent.py:470-554 (cap, break, delta) */
#define BK_SEM_ADVANCE 2 /* play max_plies random moves (pass when stuck, stop early when nobody
                            can move) and return the reached state: the batched analogue of
                            tests/utils_game_states.py:12-57 generate_random_valid_state      */

/* Legal-move list order used to turn a random index into a move */
#define BK_ORDER_NAIVE 0    /* piece asc, orientation asc, anchor row-major:
                               LegalMoveGenerator._get_legal_moves_naive, move_generator.py:153 */
#define BK_ORDER_FRONTIER 1 /* reference default frontier order (move_generator.py:261): the
                               bk_rollout_frontier entry (bk_rollout returns BK_EINVAL for it) */

/* Random streams */
#define BK_RNG_PHILOX 0   /* native: Philox4x32-10 keyed (seed, playout), counter = draw */
#define BK_RNG_NUMPY_MT 1 /* compat: numpy RandomState(seed).randint(0, n) per seat
                             (agents/random_agent.py:29,49); MT19937 + masked rejection   */

typedef struct bk_rollout_cfg {
    int32_t semantics;  /* BK_SEM_*                                                       */
    int32_t order;      /* BK_ORDER_*                                                     */
    int32_t rng;        /* BK_RNG_*                                                       */
    int32_t max_plies;  /* BK_SEM_ROLLOUT cap (MCTSAgent max_rollout_moves, default 50);
                           BK_SEM_ARENA: max turns (arena max_turns, default 2500)         */
    uint64_t seed;      /* BK_RNG_PHILOX key                                              */
    int32_t seats_share_stream; /* compat: 1 = one agent stream for every seat (MCTSAgent
                                   rollout_agent), 0 = one agent per seat (arena)         */
    int32_t heuristic_seats;    /* bit p: seat p plays HeuristicAgent (agents/heuristic_agent.py
                                   :39-244) instead of RandomAgent; BK_ORDER_FRONTIER only.
                                   Its choice is certified exact (result status bit 4 set
                                   otherwise)                               */
    uint32_t stream_base;       /* BK_RNG_PHILOX: playout i of this call draws from stream
                                   (seed, stream_base + i), so a job sharded over ranks plays
                                   the games of its global playout ids (ABI 4)             */
    int32_t reserved;
} bk_rollout_cfg;

/* One playout result: 32 bytes */
typedef struct bk_result {
    int16_t scores[BK_PLAYERS]; /* ARENA: BlokusGame.get_score (board + corner + centre bonus);
                                   ROLLOUT: Board.get_score (engine/board.py:562)             */
    uint8_t winner_mask;        /* bit p: p in GameResult.winner_ids (engine/game.py:216)    */
    uint8_t status;             /* 0 ok; bit0: rng stream overflow (compat mode); bit1:
                                   frontier table overflow; bit2: bad root_index (device path);
                                   bit4 (informational): a HeuristicAgent draw fell within
                                   2^-40 of a cumulative-probability boundary (that choice
                                   is not certified equal to the reference's);             
                                   bit3: ARENA run stopped by the max_plies turn cap before
                                   every player was known to be stuck (passes / turns are
                                   then raw and reserved[0] = passes since the last move)  */
    uint16_t plies;             /* moves placed during the playout                          */
    uint16_t passes;            /* arena passes (arena_runner.py:660-664)                   */
    uint16_t turns;             /* arena turn_count                                         */
    int32_t reward;             /* ROLLOUT: final - initial Board.get_score of root player  */
    uint32_t draws;             /* random numbers consumed                                  */
    uint32_t reserved[2];
} bk_result;

typedef struct bk_handle_s* bk_handle;

/* ---- lifecycle ------------------------------------------------------------------ */
int bk_abi_version(void);
int bk_tables_version(void);
/* device = HIP device ordinal; flags reserved (0) */
int bk_create(int device, uint32_t flags, bk_handle* out);
int bk_destroy(bk_handle h);
/* Launch on a caller stream (hipStream_t as void*; NULL = the HIP null stream, which is
   torch's default stream); BK_STREAM_OWN restores the handle's own stream. */
#define BK_STREAM_OWN ((void*)~(uintptr_t)0)
int bk_set_stream(bk_handle h, void* stream);
/* A stream owned by the handle (destroyed by bk_destroy), usable with bk_set_stream or by
   the caller: cu_mask[mask_words] (bit i = compute unit i may run its work; NULL / 0 words
   = all units) via hipExtStreamCreateWithCUMask.  The config-4 driver keeps a few CUs
   free of its long search kernels this way, so the short per-round kernels never queue
   behind them. */
int bk_stream_create(bk_handle h, const uint32_t* cu_mask, int32_t mask_words, void** out_stream);
/* Wait for the handle's stream.  Device-path launches (BK_MEM_DEVICE) return before the
   kernel ends, so their input errors and guard trips surface here: BK_EOVERFLOW if a
   persistent kernel's iteration guard tripped (results incomplete), BK_EINVAL if a
   root_index entry was outside [0, n_roots) (that playout ran from root 0 with status
   bit 2); both cleared once reported.  BK_ECHECK: a bk_mcts search broke a tree invariant
   (bk_debug_mcts_failure has the record). */
int bk_synchronize(bk_handle h);
int bk_last_error(bk_handle h, char* buf, size_t len);

/* Tuning and test overrides (ABI 5; no reference counterpart).  bk_create reads each
   from the environment variable of the same name once (BK_MG_GROUPS, ...); later changes
   of the environment do not reach an existing handle, and no entry point reads the
   environment.  bk_set_tuning sets one for this handle (-1 = automatic: the library's
   measured choice).  Values are range-checked where they are used, as before. */
enum {
    BK_TUNE_MG_GROUPS = 0,       /* movegen orientation groups per board-player set      */
    BK_TUNE_MG_STAGE,            /* bk_movegen_mask: 0 = per-lane stores (k_movegen_m)    */
    BK_TUNE_MG_PARTS,            /* k_movegen_ml orientation ranges: 4, 5, 7 or 13        */
    BK_TUNE_MG_PART_WAVES,       /* waves per k_movegen_ml block                          */
    BK_TUNE_DEBUG_MAX_ITERS,     /* playout kernels' step guard (tests force a trip)      */
    BK_TUNE_HANDOUT,             /* playout hand-out 0..2                   */
    BK_TUNE_MCTS_COOP,           /* bk_mcts: 1 = one wave per search, 0 = one lane        */
    BK_TUNE_COOP_BLOCKS_PER_CU,  /* k_mcts_coop(_h) resident blocks per CU                */
    BK_TUNE_MCTS_SPREAD,         /* bk_mcts per-lane kernels: searches every spread lanes */
    BK_TUNE_TREE_BATCH,          /* bk_mcts lockstep tree-phase threshold                 */
    BK_TUNE_COOP_WALK,           /* k_mcts_coop(_h): 0 = serial frontier walks            */
    BK_TUNE_COOP_BAL,            /* k_mcts_coop_h: 0 = per-lane HeuristicAgent sums       */
    BK_TUNE_MCTS_PAIR,           /* bk_mcts spread 2: 0 = unsplit lanes (k_mcts)          */
    BK_TUNE_COUNT
};
int bk_set_tuning(bk_handle h, int32_t key, int64_t value);
int bk_get_tuning(bk_handle h, int32_t key, int64_t* value);

/* ---- tables ------------------------------------------------------------------------ */
/* Orientation table, global orientation id g in [0, 91): piece_id, orientation index,
   cell count and sorted normalized offsets (engine/pieces.py:147-253).  offs = 10 ints. */
int bk_orient_info(int g, int32_t* piece_id, int32_t* orient, int32_t* ncells, int32_t* offs);

/* ---- hot path ------------------------------------------------------------------------ */
/*
 * Batched legal-move generation.  Replaces LegalMoveGenerator.get_legal_moves
 * (engine/move_generator.py:130) for n (state, player) pairs.
 *   out_rows  : n x 91 x 20 uint32, bit c of row r = anchor (r, c) legal for that
 *               orientation (anchor = top-left of the orientation's bounding box,
 *               exactly Move.anchor_row/anchor_col); may be NULL (counts only)
 *   out_count : n uint32 total legal moves (len(get_legal_moves)); may be NULL
 * players[i] in 0..3.  All pointers share residency `mem`.
 */
int bk_movegen(bk_handle h, const bk_state* states, const uint8_t* players, int32_t n,
               uint32_t* out_rows, uint32_t* out_count, int mem);

/*
 * The same legal-move sets as dense 400-bit masks (the SURVEY 8(b) bk_movegen form):
 *   out_mask  : n x 91 x 7 uint64; bit b of word w is cell 64 w + b = r * 20 + c (the
 *               numbering of Board.player_bits, engine/bitboard.py:19-40): orientation g
 *               anchored at (r, c) is legal.  Bits 400..447 are zero.  5,096 B per
 *               board-player; 8-byte aligned; may be NULL (counts only)
 *   out_count : n uint32 total legal moves; may be NULL
 * Replaces LegalMoveGenerator.get_legal_moves (engine/move_generator.py:130-151, the set;
 * the host orders it).  ABI version 3.
 */
int bk_movegen_mask(bk_handle h, const bk_state* states, const uint8_t* players, int32_t n,
                    uint64_t* out_mask, uint32_t* out_count, int mem);

/* has_legal_moves for all 4 players of n states (move_generator.py:961): out_mask4[i]
   bit p set if player p has a legal move. */
int bk_has_moves(bk_handle h, const bk_state* states, int32_t n, uint8_t* out_mask4, int mem);

/*
 * Random playouts.  For playout i = 0..n_playouts-1 start from
 * roots[root_index[i]] (root_index may be NULL: i % n_roots) and play to the end
 * under cfg.  compat_seeds (BK_RNG_NUMPY_MT only): n_playouts x 4 uint32 seeds, one
 * numpy RandomState seed per seat (seats_share_stream: entry 0 is used).
 * Replaces the inner loops of mcts/mcts_agent.py:470-554 and the arena game loop.
 */
int bk_rollout(bk_handle h, const bk_state* roots, int32_t n_roots, const int32_t* root_index,
               int32_t n_playouts, const bk_rollout_cfg* cfg, const uint32_t* compat_seeds,
               bk_result* out, int mem);

/* BK_SEM_ADVANCE: like bk_rollout but writes the final state of every playout to
   out_states (n_playouts records); out may be NULL. */
int bk_advance(bk_handle h, const bk_state* roots, int32_t n_roots, const int32_t* root_index,
               int32_t n_playouts, const bk_rollout_cfg* cfg, const uint32_t* compat_seeds,
               bk_state* out_states, int mem);

/*
 * Reference frontier ORDER on the GPU.
 *
 * The reference's default generator (engine/move_generator.py:261-559) lists a
 * (piece, orientation)'s anchors in the order its frontier SET iterates: a CPython 3.10
 * set of (row, col) tuples whose slot layout is fixed by the exact add/discard history
 * of engine/board.py:315-367 (update_frontier_after_move) and set.copy() (Board.copy,
 * engine/board.py:643-660).  bk_fset is that hash table, restated bit for bit
 * (Objects/setobject.c: LINEAR_PROBES 9, PERTURB_SHIFT 5, resize to used*4 when
 * fill*5 >= mask*3, copy re-inserts in slot order), one per player.  Iteration order =
 * slot order of keys >= 0.
 */
#define BK_FSET_SLOTS 256
typedef struct bk_fset {
    int16_t key[BK_PLAYERS][BK_FSET_SLOTS]; /* cell r*20+c; -1 unused; -2 dummy      */
    uint16_t mask[BK_PLAYERS];              /* table size - 1 (7 .. 255)               */
    uint16_t fill[BK_PLAYERS];              /* active + dummy slots                    */
    uint16_t used[BK_PLAYERS];              /* active slots                            */
    uint16_t reserved[BK_PLAYERS];
} bk_fset; /* 2080 bytes */

/* Host-side table maintenance for host Boards (no GPU needed):
   Board() (engine/board.py:54-78 init_frontiers): every player's set = {start corner} */
int bk_fset_init(bk_fset* s);
/* place_piece's frontier update for `player` (engine/board.py:315-367).  `after` is the
   board AFTER the piece's cells were written (the reference writes the grid first);
   cells in place_piece order (r*20+c). */
int bk_fset_place(bk_fset* s, const bk_state* after, int32_t player, const int32_t* cells, int32_t n);
/* set.copy() of every player's set (Board.copy, engine/board.py:643-660) */
int bk_fset_copy(bk_fset* dst, const bk_fset* src);
/* iteration order of player's set into out (cap entries); returns the count or < 0 */
int bk_fset_list(const bk_fset* s, int32_t player, int32_t* out, int32_t cap);
/* Diagnostics (tests): one set operation on player's set, set.add((r, c)) (add = 1) or
   set.discard((r, c)) (add = 0), key = r*20+c: the probe / insert / resize code every
   frontier-order kernel runs; add | 2: resize through a small scratch, as the kernels'
   LDS-staged tables do (tables of <= 128 slots, a 32-key scratch).  Returns BK_OK, or 1 when
   the op resized through that scratch (add | 2, <= 32 active keys: the test counts them).
   BK_EOVERFLOW: the table outgrew its 256 slots (128 with add | 2). */
int bk_debug_fset_op(bk_fset* s, int32_t player, int32_t key, int32_t add);

/*
 * bk_rollout / bk_advance in the reference's FRONTIER order (cfg->order ==
 * BK_ORDER_FRONTIER): root_sets[n_roots] carry the roots' frontier tables; with
 * BK_RNG_NUMPY_MT the playouts are the reference's default-config games move for move.
 * BK_SEM_ARENA / BK_SEM_ROLLOUT: out[n_playouts]; ARENA may also ask for the final
 * states and tables (out_states and out_sets both set, else both NULL).
 * BK_SEM_ROLLOUT starts from set.copy() of the root tables, as MCTSAgent._rollout plays
 * on sim = board.copy() (mcts/mcts_agent.py:470).
 * BK_SEM_ADVANCE: out_states[n_playouts] and out_sets[n_playouts] (out may be NULL).
 * A table that would outgrow BK_FSET_SLOTS stops its playout with status 2.
 */
int bk_rollout_frontier(bk_handle h, const bk_state* roots, const bk_fset* root_sets, int32_t n_roots,
                        const int32_t* root_index, int32_t n_playouts, const bk_rollout_cfg* cfg,
                        const uint32_t* compat_seeds, bk_result* out, bk_state* out_states,
                        bk_fset* out_sets, int mem);

/*
 * Arena games with search seats (config 4, analytics/tournament/arena_runner.py:578-777):
 * advance each of n games in place until the player to move is a STOP seat that has a
 * legal move (its agent -- MCTSAgent / FastMCTSAgent -- is run by the caller, which then
 * places the move and calls again), or the game is over, or it reached cfg->max_plies
 * turns in total.  Other seats play RandomAgent (randint) or, where seat_masks[i] bit p is
 * set, HeuristicAgent, each from its own numpy stream carried in rng_state[i][16] (seat p:
 * MT19937 cursor {pos, mt[pos], mt[pos + 1], mt[pos + 397]} of the first 227 outputs of its
 * seed; bk_mt_cursor_init makes fresh ones).  seat_masks[i]: bits 0-3 heuristic seats,
 * bits 4-7 stop seats.  states[i] / sets[i] (the position and its frontier tables) are
 * read and rewritten; states[i].reserved[0] / [1] carry the game's turn_count / passes
 * across calls (0 at the start).  out[i]: status BK_STATUS_STOP (32) = stopped at a stop
 * seat (current_player of states[i]), else the finished game's result (status bit 3: cut
 * by max_plies; passes / turns in out count this call only).  cfg: BK_SEM_ARENA,
 * BK_ORDER_FRONTIER, BK_RNG_NUMPY_MT, seats_share_stream 0.  Device pointers: rng_state
 * 16-byte aligned.
 */
#define BK_STATUS_STOP 32
int bk_arena_advance(bk_handle h, bk_state* states, bk_fset* sets, int32_t n, const bk_rollout_cfg* cfg,
                     const uint8_t* seat_masks, uint32_t* rng_state, bk_result* out, int mem);
/*
 * bk_arena_advance with the search seats' moves and their inputs kept on the device, so an
 * arena round is bk_arena_step -> bk_mcts / bk_fastmcts -> bk_arena_step with no
 * position or table crossing PCIe (config 4).  Extra arguments (each may be NULL):
 * forced[i]: the move the agent at game i's stop seat chose in the previous round, placed
 *   first: -1 none (a stopped game stays stopped); g * 400 + 20 r + c a move
 *   (bk_mcts best_move); BK_FORCE_INDEX | k the k-th entry of the mover's legal list in
 *   the reference's order (FastMCTSAgent's child index into get_legal_moves);
 *   BK_FORCE_SKIP: game i is not touched at all (its search is still running: no
 *   result, no stop info, state and tables unchanged).
 * quick_masks[i] bit p: stop seat p is a FastMCTSAgent; when game i stops there,
 *   stop_out[i] receives its root's FastMCTS inputs: the legal-move count, and
 *   _quick_move_evaluation (agents/fast_mcts_agent.py:285-298: of the first 3 moves by
 *   piece id descending, stable, the one nearest the centre by |r - 9.5| + |c - 9.5|,
 *   stable) as its list index and its reward pid * 0.1 + (20 - dist) * 0.05 (:260-283).
 */
#define BK_FORCE_INDEX 0x40000000
#define BK_FORCE_SKIP (-2)
typedef struct bk_stop_info {
    int32_t n_legal;      /* legal moves of the player to move                        */
    int32_t quick_index;  /* list index of _quick_move_evaluation's move              */
    double quick_reward;  /* _fast_rollout's reward before the noise term             */
} bk_stop_info;

int bk_arena_step(bk_handle h, bk_state* states, bk_fset* sets, int32_t n, const bk_rollout_cfg* cfg,
                  const uint8_t* seat_masks, const uint8_t* quick_masks, const int32_t* forced,
                  uint32_t* rng_state, bk_result* out, bk_stop_info* stop_out, int mem);

/* numpy RandomState(seed) cursor for rng_state (host, no GPU) */
int bk_mt_cursor_init(uint32_t seed, uint32_t* out4);

/*
 * FastMCTS simulate loop (agents/fast_mcts_agent.py:153-256) for n_games independent
 * roots, one wave per game.  Game i's root children are legal[legal_offset[i] ..
 * legal_offset[i+1]) (any int payload; only the count and order matter: expansion pops
 * the LAST entry first, fast_mcts_agent.py:62).  Each iteration expands an untried
 * child or picks the UCB1 argmax (first max in child order; exploration term
 * c*(2*log(root_visits)/visits)**0.5 with log taken from log_table, which the host fills
 * with CPython math.log(i) for i < log_len, and ** 0.5 reproduced bit for bit through the
 * pow_fix tables of bk_pow_half_fix below), then adds reward = base[i] +
 * random()*0.1, random() being CPython random.Random's genrand_res53 from the state
 * mt_state[i] (625 words: random.getstate()[1]); a NaN base[i] means reward 0.0 with no
 * draw (empty cached legal list, fast_mcts_agent.py:255).  mt_state is in/out: the
 * advanced state is written back.  Results per game in out; visits_out (optional, may
 * be NULL) receives every root child's visit count at its legal index (flat, by
 * legal_offset; 0 = never expanded).  Replaces the per-iteration
 * Python loop of FastMCTSAgent.think (fast_mcts_agent.py:153-166).
 */
#define BK_FASTMCTS_TOP 10
#define BK_FASTMCTS_MAX_CHILDREN 2048
typedef struct bk_fastmcts_out {
    int32_t best_index;   /* index into the game's legal list of the most visited child  */
    int32_t iterations;   /* iterations run                                              */
    int32_t n_children;   /* root children expanded                                      */
    int32_t n_top;        /* entries used in top_*                                       */
    int32_t top_index[BK_FASTMCTS_TOP];  /* by visits desc, ties in child order        */
    int32_t top_visits[BK_FASTMCTS_TOP];
    double top_q[BK_FASTMCTS_TOP];       /* total_reward / visits                       */
} bk_fastmcts_out;

int bk_fastmcts(bk_handle h, int32_t n_games, const int32_t* legal_offset, const int32_t* iterations,
                const double* base, uint32_t* mt_state, const double* log_table, int32_t log_len,
                const int32_t* pow_fix_offsets, const int32_t* pow_fix_entries, int32_t pow_fix_rows,
                double exploration, bk_fastmcts_out* out, int32_t* visits_out, int mem);

/*
 * The exploration term is (2 * math.log(N) / v) ** 0.5 (fast_mcts_agent.py:52): CPython
 * float ** calls C pow(), which in glibc is not correctly rounded, so for ~0.085 % of
 * (N, v) it is one ulp off the correctly rounded sqrt() a GPU computes.  The kernel takes
 * sqrt and applies the listed corrections.  bk_pow_half_fix computes them on the host with
 * the process's own libm pow() (the function CPython calls):
 *   for N in [0, rows), v in [1, N]: x = (2.0 * log_table[N]) / v; if pow(x, 0.5) !=
 *   sqrt(x), entry (v << 1) | (pow > sqrt) in entries[offsets[N] .. offsets[N + 1]).
 * offsets: rows + 1 ints.  Cost ~N^2/2 sqrt (pow only near rounding midpoints, where it
 * can differ).  Returns BK_OK; BK_EOVERFLOW with *n_entries = the count needed when cap is
 * too small; BK_EINVAL if pow and sqrt ever differ by more than 1 ulp.
 * bk_fastmcts reads offsets / entries as pow_fix_offsets / pow_fix_entries with
 * pow_fix_rows = rows (<= log_len, same log_table): selections at root visits N >= rows
 * use the plain sqrt (the host builds rows up to 16,385: exact for searches of up to
 * 16,384 iterations).
 */
int bk_pow_half_fix(const double* log_table, int32_t rows, int32_t* offsets, int32_t* entries, int32_t cap,
                    int32_t* n_entries);

/* Diagnostics (no reference counterpart): one FastMCTS selection step on the device --
   the UCB1 argmax (first max in child order) over n children with the given visits
   (all > 0) and total rewards, parent visits N, with k_fastmcts's exact arithmetic and
   pow corrections -- so tests can pin near-ties.  out_best: the chosen child index. */
int bk_debug_fastmcts_select(bk_handle h, int32_t n, const uint32_t* visits, const double* totals, uint32_t root_visits,
                             const double* log_table, int32_t log_len, const int32_t* pow_fix_offsets,
                             const int32_t* pow_fix_entries, int32_t pow_fix_rows, double exploration,
                             int32_t* out_best);

/*
 * bk_mcts -- MCTSAgent.select_action searches (mcts/mcts_agent.py:304-582, MCTSNode
 * :19-191) with RandomAgent or HeuristicAgent rollouts (cfg.rollout_policy) and the Zobrist
 * transposition table (mcts/zobrist.py:12-220), one search per game, all on the GPU.
 * Bit-exact with the reference for the same inputs: frontier-order legal lists
 * (root_sets = the Board's frontier tables, see bk_fset_*), untried.pop() expansion,
 * UCB1 in IEEE double with np.log values from log_table (log_table[v] = np.log(v)),
 * first-best ties, the rollout agent's numpy MT19937 stream (mt_state[625] per game:
 * key[624] then pos; in/out), TT hits reusing the cached reward.
 *
 * Inputs per game: roots[g] / root_sets[g] (the position), players[g] (the searching
 * player, MCTSNode.player), root_hash[g] (ZobristHash.hash_board of the position; NULL:
 * computed on the device from roots and the game's key table),
 * zobrist_index[g] (which 2088-entry key table of `zobrist` the agent uses: 20*20*5 cell
 * keys, 4 turn keys, 4*21 piece keys, mcts/zobrist.py:41-68).
 * TT per game: tt_keys/tt_vals[g * cfg.tt_cap ...] open addressing (linear probing,
 * slot = key & (tt_cap - 1), empty slot = NaN value), tt_count[g] entries; in/out so the
 * table persists across an agent's searches like the reference's dict.
 * nodes[g * cfg.node_cap ...]: the tree (node 0 = root).  A node's children are one
 * contiguous block in expansion order; the block holds min(n_legal, 4) slots at the
 * first expansion and is moved to a block twice as large (capped at n_legal) each time
 * it fills, so a search of I iterations never needs more than 4*I + 1 slots.  Left on
 * return for inspection.
 * Chunked searches: a launch with cfg.iter_stop = k stops every search after k
 * iterations; a later launch with cfg.resume = 1 (same buffers, larger iter_stop)
 * continues them from nodes / out / tt / mt_state exactly where they stopped.  The
 * result equals one launch of cfg.iterations.
 * rewards / hit_flags (optional, [g * cfg.iterations + i]): per iteration the simulated
 * reward and 1 if it came from the TT (stats["rollout_rewards"] = the non-hit ones).
 * out[g].status != 0 means the search stopped early (see BK_MCTS_E*): enlarge the pool /
 * TT and retry from the saved inputs.
 */
#define BK_MCTS_NODE_EVALUATED 1u
typedef struct bk_mcts_node {
    double total;       /* total_reward                                               */
    uint32_t visits;
    int32_t child0;     /* first slot of the child block, -1 = none                   */
    uint16_t move;      /* g * 400 + anchor cell of the move leading here (root 0xFFFF) */
    uint16_t n_exp;     /* len(children)                                              */
    uint16_t n_legal;   /* len(legal moves) once evaluated                            */
    uint16_t flags;     /* BK_MCTS_NODE_EVALUATED                                     */
} bk_mcts_node;         /* 24 bytes */

typedef struct bk_mcts_cfg {
    int32_t iterations;        /* MCTSAgent.iterations (also the rewards row stride)   */
    int32_t max_rollout_moves; /* MCTSAgent.max_rollout_moves (> 0)                    */
    double exploration;        /* exploration_constant                                 */
    int32_t use_tt;            /* use_transposition_table                              */
    int32_t node_cap;          /* node slots per game                                  */
    int32_t tt_cap;            /* TT slots per game, power of two (>= 2 when use_tt)   */
    int32_t time_limit_us;     /* > 0: stop at the first iteration boundary past it    */
    int32_t iter_stop;         /* > 0: this launch stops each search once it has run
                                  iter_stop iterations in total (chunked searches)      */
    int32_t resume;            /* 1: continue the searches left in nodes / out / tt /
                                  mt_state by an earlier launch (iter_stop chunks)      */
    int32_t rollout_policy;    /* BK_MCTS_ROLLOUT_*: the rollout_agent                  */
    int32_t flags;             /* BK_MCTS_ASYNC: with BK_MEM_DEVICE, return once the
                                  launch is enqueued (no wait; a tripped step guard is
                                  then reported by bk_synchronize).  The running search
                                  uses the handle's scratch, so the handle takes no other
                                  launch (BK_EINVAL) until bk_synchronize, which waits
                                  on the stream the search was launched on: one
                                  asynchronous search per handle at a time            */
} bk_mcts_cfg;
#define BK_MCTS_ASYNC 1
/* BK_MCTS_STATE_ROWS (ABI 7, BK_MEM_DEVICE only): mt_state, tt_keys, tt_vals and tt_count
   hold one row per agent (n_zobrist rows), search g using row zobrist_index[g]: the MT
   state is copied in at the search's start and back at its end, the TT probed and filled
   in place, all with system-scope (L2-bypassing) accesses -- so a launch needs no gather /
   scatter of agent state, and a later launch may search with an agent as soon as its
   earlier search is done (bk_mcts_set_done) even while that launch still runs.  No two
   searches of one launch may share a row. */
#define BK_MCTS_STATE_ROWS 2
#define BK_MCTS_ROLLOUT_RANDOM 0    /* RandomAgent (agents/random_agent.py:49)            */
#define BK_MCTS_ROLLOUT_HEURISTIC 1 /* HeuristicAgent (agents/heuristic_agent.py:39-244),
                                       MCTSAgent's default (mcts/mcts_agent.py:275-281);
                                       choices certified exact, else BK_MCTS_EUNCERT    */

#define BK_MCTS_EPOOL 1u   /* node pool full                    */
#define BK_MCTS_EFSET 2u   /* frontier table overflow           */
#define BK_MCTS_ETT 4u     /* TT full                           */
#define BK_MCTS_EPATH 8u   /* tree deeper than BK_MCTS_MAX_DEPTH */
#define BK_MCTS_ELOG 16u   /* log_table too short               */
#define BK_MCTS_EINTERNAL 32u /* consistency check failed        */
#define BK_MCTS_EUNCERT 64u   /* informational (the search goes on): a HeuristicAgent draw
                                 fell within 2^-40 of a probability boundary, so that
                                 choice is not certified equal to the reference's        */
#define BK_MCTS_MAX_DEPTH 63
typedef struct bk_mcts_out {
    int32_t best_move;       /* g*400+cell of the most visited root child (first on ties), -1 */
    int32_t iterations_run;
    int32_t tt_hits;         /* simulations answered by the TT                           */
    int32_t rollouts;        /* simulations that ran a rollout                           */
    int32_t nodes_used;
    int32_t root_children;
    uint32_t status;         /* BK_MCTS_E* bits                                          */
    int32_t rollout_plies;   /* moves played by this search's rollouts (sum)             */
} bk_mcts_out;

int bk_mcts(bk_handle h, const bk_state* roots, const bk_fset* root_sets, const uint8_t* players,
            const uint64_t* root_hash, int32_t n_games, const bk_mcts_cfg* cfg, const uint64_t* zobrist,
            int32_t n_zobrist, const int32_t* zobrist_index, uint32_t* mt_state, uint64_t* tt_keys,
            double* tt_vals, int32_t* tt_count, const double* log_table, int32_t log_len,
            bk_mcts_node* nodes, double* rewards, uint8_t* hit_flags, bk_mcts_out* out, int mem);

/*
 * Failure record of a bk_mcts search whose tree broke an invariant (ABI 6; no reference
 * counterpart -- the reference's dict-and-object tree cannot be written by another
 * search).  A node with more visits than the log table allows (BK_MCTS_ELOG: a correct
 * search of I iterations never exceeds I) or a root whose visits differ from the
 * iterations run (BK_MCTS_EINTERNAL; mcts/mcts_agent.py:572-582 backpropagates every
 * iteration through the root) means the search's node pool was written by something
 * else.  The first such search of a launch records what it saw in a sticky device
 * buffer; bk_synchronize (and a host-memory bk_mcts) then return BK_ECHECK once, and
 * bk_debug_mcts_failure copies the record: returns 1 with out[0..n) filled, 0 if no
 * search ever failed on this handle.  Words: see BK_DIAG_*.
 */
#define BK_DIAG_WORDS 64
#define BK_DIAG_REASON 0      /* BK_MCTS_ELOG or BK_MCTS_EINTERNAL                      */
#define BK_DIAG_KERNEL 1      /* BK_DIAG_K_*                                            */
#define BK_DIAG_LAUNCH 2      /* bk_mcts launch number on this handle (1, 2, ...)       */
#define BK_DIAG_GAME 3        /* the search's index in its launch                       */
#define BK_DIAG_NODE 4        /* node index in the search's pool (0 = root)             */
#define BK_DIAG_VISITS 5      /* that node's visits, n_exp, n_legal, child0: words 5..8 */
#define BK_DIAG_ITERATION 9   /* iterations the search had run                          */
#define BK_DIAG_DEPTH 10      /* selection depth when it fired (ELOG)                   */
#define BK_DIAG_LOG_LEN 11
#define BK_DIAG_HANDOUT 12    /* the launch's game hand-out counter when it fired       */
#define BK_DIAG_NODE_CAP 13   /* node_cap, nodes_used, cfg.iterations: words 13..15     */
#define BK_DIAG_PATH_LEN 16   /* root-to-node path entries recorded (<= 22)             */
#define BK_DIAG_PATH 18       /* path node indices: words 18..39; their visits: 40..61
                                 (ELOG / EINTERNAL records)                             */
/* Any kernel: a search handed out twice in one launch records BK_DIAG_DOUBLE_START: the
   search (word 3), the hand-out counter (12), the value handed (17), the block and wave
   that started it the second time (18, 19), the wave's HW_ID register (20), n_games (21). */
#define BK_DIAG_DOUBLE_START 0x200u
#define BK_DIAG_K_LANE 0      /* k_mcts      */
#define BK_DIAG_K_PAIR 1      /* k_mcts_pair */
#define BK_DIAG_K_H 2         /* k_mcts_h    */
#define BK_DIAG_K_COOP 3      /* k_mcts_coop */
#define BK_DIAG_K_COOP_H 4    /* k_mcts_coop_h */
int bk_debug_mcts_failure(bk_handle h, uint32_t* out, int32_t n);

/*
 * Per-search completion (ABI 7; no reference counterpart -- arena_runner.py:578-777 runs
 * one game at a time).  bk_mcts_set_done(h, done): every later bk_mcts launch on h stores,
 * once search g's agent rows are written back, done[g] = best_move (bits 0..31) |
 * iterations_run (32..55) | status (56..62) | 1 << 63 -- one 64-bit store; NULL turns it
 * off.  With done in memory from bk_host_alloc (mapped, coherent host memory), a host
 * polls done[] while the launch runs and takes each search's move as soon as it is final:
 * a launch lasts as long as its longest search (config 4: 2.3x the mean), its games need
 * not.  The caller zeroes done[0..n_games) before each launch; `out` is complete when the
 * launch ends.
 * bk_host_alloc: `bytes` of pinned, device-mapped, coherent host memory (the device
 * uses the same address), or NULL; bk_host_free releases it.
 */
int bk_mcts_set_done(bk_handle h, uint64_t* done);
void* bk_host_alloc(size_t bytes);
int bk_host_free(void* p);

/* Average duration (ms) of the most recent bk_rollout/bk_movegen kernel on the handle
   stream, measured with HIP events around that launch. */
int bk_last_kernel_ms(bk_handle h, float* ms);
/* Name of the kernel the last timed call on h launched ("" before any), e.g. "k_mcts_pair"
   or "k_mcts_coop_h" for bk_mcts, which picks its kernel from the batch size: lets a
   profiler's per-kernel counters be matched to the call.  Owned by the library.          */
const char* bk_last_kernel(bk_handle h);

/* Diagnostics (no reference counterpart): per-section shader-clock cycles summed over
   waves since the last reset, from a library built with -DBK_SECTION_PROF
   (tools/sections.py).  The product build returns BK_EINVAL and zeros. */
int bk_debug_sections(bk_handle h, uint64_t* out, int32_t n, int32_t reset);

#ifdef __cplusplus
}
#endif
#endif /* BLOKUS_HIP_H */
