// blokus_kernels.hip -- MI355X (gfx950) kernels + C-ABI for the Blokus hot path.
//
// Replaces, for batches of independent 20x20 4-player boards:
//   engine/move_generator.py:130-559  LegalMoveGenerator.get_legal_moves (legal SET)
//   engine/move_generator.py:961-1054 has_legal_moves
//   mcts/mcts_agent.py:470-554        MCTSAgent._rollout          (BK_SEM_ROLLOUT)
//   analytics/tournament/arena_runner.py:652-697 game loop        (BK_SEM_ARENA)
//   engine/game.py:182-349            game over / GameResult scoring
//
// Design (DESIGN.md has the full story):
//   * one lane = one board (one game); 64 games per wave, all control flow uniform
//     except per-game data.  No MFMA: this is integer bit work on the VALU.
//   * board rows are 32-bit words with column x at bit x; bits 20..31 model the
//     off-board columns.  A legal anchor set of one orientation for all 20 anchor
//     columns of one anchor row is then
//         ok[r] = ~OR_cells(B[r+d] >> c) & OR_cells(C[r+d] >> c)
//     with B = blocked cells (occupied | orth-adjacent-to-own | off-board) and
//     C = corner cells (frontier).  Right shifts, ORs and v_bitop3_b32 issue at full
//     rate on gfx950 (v_lshl_or_b32 / v_lshlrev_b32 / v_or3_b32 at half rate,
//     tools/valu_probe2.hip), so a term costs one v_lshrrev_b32 plus half a
//     three-input v_bitop3_b32 OR.
//   * the 20 board rows live in VGPRs (static index).  Orientations are grouped in 49
//     "stencil classes" (height + static sequence of (piece row, single|pair) terms,
//     tools/gen_tables.py); each class is straight-line code looping at run time over
//     its orientations, whose column shifts are uniform (SGPR) operands.
//   * per-orientation prefix counts go to LDS ([orient][lane], u16) so that a
//     uniform random index can be mapped back to (orientation, row, column) in the
//     reference's naive list order without storing any mask.
//   * the rollout kernel is persistent: each lane pulls playouts from a global
//     counter, keeps its board in a lane-strided scratch slab (L2-resident rows),
//     and never returns to the host between plies.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sched.h>

#include <mutex>
#include <thread>
#include <new>
#include <vector>

#include "../../include/blokus_hip.h"
#include "orient_table.h"

#define BK_TABLES_VERSION 1

// Translation units.  build.py compiles this file once per unit, in parallel: -DBK_TU=u
// defines unit u's kernels (the other kernels are only declared), BK_U_HOST the C-ABI
// (host code only, --offload-host-only).  Without BK_TU (a one-shot build) the file
// defines everything.  Device templates are instantiated only in the units that use them.
#define BK_U_HOST 1
#define BK_U_MOVEGEN 2
#define BK_U_ROLLOUT 3
#define BK_U_ROLLOUT_FR 4
#define BK_U_ROLLOUT_FRH 5
#define BK_U_FASTMCTS 6
#define BK_U_MCTS 7
#define BK_U_MCTS_PAIR 8
#define BK_U_MCTS_H 9
#define BK_U_COOP 10
#define BK_U_COOP_H 11
#ifndef BK_TU
#define BK_TU 0
#endif
#define BK_DEF(u) (BK_TU == 0 || BK_TU == (u))
// Locate pass 2 skips frontier cells with no anchor row within the piece's height, and
// compacts each 16-slot batch to the slots that can add an anchor before the row reads,
// so the wave runs them max-over-lanes-of-relevant-slots times instead of 16
// (frontier-order config 3 25.8 -> 27.9 M playouts/s, config 5 16.2 -> 17.2 M sims/s,
// profiles/r04/sweeps/r04p).  place_frontier loads a stage of <= STAGE_EAGER_MAX slots
// alongside the table's mask: one memory latency instead of two (+1.0 % for the 4-block
// k_rollout_fr, profiles/r04/sweeps/r04v).  The measured-slower alternatives of these
// and the other A/B knobs below are out of the source; DESIGN.md 4 keeps their numbers.
#define STAGE_EAGER_MAX 64

// Section timers (diagnostic build only, -DBK_SECTION_PROF): per-wave shader-clock
// cycles spent in each section of a kernel's loop, summed over waves into
// g_sections[] (read with bk_debug_sections: every unit registers a reader of its own
// copy, and the reads are summed).  Compiled out of the product build.
#define BK_NSECT 16
#ifdef BK_SECTION_PROF
static __device__ unsigned long long g_sections[BK_NSECT];
void bk_register_sections(int (*rd)(unsigned long long*, int));
#if BK_TU != BK_U_HOST
static int bk_read_sections(unsigned long long* v, int reset) {
    unsigned long long t[BK_NSECT];
    if (hipMemcpyFromSymbol(t, HIP_SYMBOL(g_sections), sizeof t) != hipSuccess) return -1;
    for (int i = 0; i < BK_NSECT; ++i) v[i] += t[i];
    if (reset) {
        memset(t, 0, sizeof t);
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sections), t, sizeof t) != hipSuccess) return -1;
    }
    return 0;
}
static const int bk_sections_registered = (bk_register_sections(bk_read_sections), 0);
#endif
#define SECT_DECL uint64_t sect_acc[BK_NSECT] = {0}; uint64_t sect_t = clock64();
#define SECT(i) do { const uint64_t now_ = clock64(); sect_acc[i] += now_ - sect_t; sect_t = now_; } while (0)
#define SECT_FLUSH do { if ((threadIdx.x & (WAVE - 1)) == 0) for (int i_ = 0; i_ < BK_NSECT; ++i_) \
        if (sect_acc[i_]) atomicAdd(&g_sections[i_], (unsigned long long)sect_acc[i_]); } while (0)
#else
#define SECT_DECL
#define SECT(i) do {} while (0)
#define SECT_FLUSH do {} while (0)
#endif
#define WAVE 64
#define BLOCK 256
#define ROWMASK 0x000FFFFFu  // columns 0..19

// Lane-pair exchanges (k_mcts_pair: lanes 2q, 2q + 1 share a search) on DPP quad_perm --
// ALU latency, where __shfl is a ds_bpermute round trip.  Both lanes of the pair must be
// active (they run in lockstep wherever these are used).
__device__ __forceinline__ int pair_other(int v) {  // the partner's value (lane ^ 1)
    return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);  // quad_perm [1, 0, 3, 2]
}
__device__ __forceinline__ int pair_even(int v) {  // the even lane's value (lane & ~1)
    return __builtin_amdgcn_update_dpp(0, v, 0xA0, 0xF, 0xF, false);  // quad_perm [0, 0, 2, 2]
}
#define OFFBOARD 0xFFF00000u // columns 20..31
// word views of int16 frontier tables: may_alias, or type-based alias analysis lets the
// compiler move them across int16 accesses of the same bytes
typedef uint32_t bk_u32_alias __attribute__((may_alias));
typedef uint4 bk_u4_alias __attribute__((may_alias));

__constant__ uint32_t kInfo[BK_NUM_ORIENTS] = BK_ORIENT_INFO_INIT;
__constant__ uint32_t kCells[BK_NUM_ORIENTS][5] = BK_ORIENT_CELLS_INIT;
__constant__ uint32_t kClass[BK_NUM_ORIENTS][2] = BK_CLASS_TABLE_INIT;

// frontier_ops: per orientation, bit 9 q + o set iff q < n and op o of cell q is the first
// op of its kind (add / discard) on its cell relative to the anchor -- later ones are
// no-ops of update_frontier_after_move (a diagonal or orthogonal shared by two cells, or
// a cell that is also another cell's orthogonal).  Built at compile time from the cells.
struct FopsTable {
    uint64_t m[BK_NUM_ORIENTS];
};
constexpr FopsTable make_fops_first() {
    constexpr uint32_t info[BK_NUM_ORIENTS] = BK_ORIENT_INFO_INIT;
    constexpr uint32_t cells[BK_NUM_ORIENTS][5] = BK_ORIENT_CELLS_INIT;
    constexpr int dr[9] = {0, -1, -1, 1, 1, -1, 1, 0, 0}, dc[9] = {0, -1, 1, -1, 1, 0, 0, -1, 1};
    FopsTable t{};
    for (int g = 0; g < BK_NUM_ORIENTS; ++g) {
        const int n = (int)((info[g] >> 8) & 0xFFu);
        uint64_t seen_add = 0, seen_dis = 0, m = 0;
        for (int q = 0; q < n; ++q) {
            const int pq = ((int)(cells[g][q] >> 8) + 1) * 7 + (int)(cells[g][q] & 0xFFu) + 1;
            for (int o = 0; o < 9; ++o) {
                const uint64_t b = 1ull << (pq + 7 * dr[o] + dc[o]);
                uint64_t& seen = (o >= 1 && o <= 4) ? seen_add : seen_dis;
                if (!(seen & b)) m |= 1ull << (9 * q + o);
                seen |= b;
            }
        }
        t.m[g] = m;
    }
    return t;
}
__constant__ FopsTable kFopsFirst = make_fops_first();

// The picked orientation's table entries (kInfo, kCells, kFopsFirst), loaded once per ply
// with the loads issued together right after the pick, for locate / apply / the frontier
// update, which otherwise each reload them (a dependent memory latency apiece)
struct OrientRow {
    uint32_t info;
    uint32_t cell[5];
    uint64_t ffirst;
};
__device__ __forceinline__ OrientRow orient_row(int gs) {
    OrientRow o;
    o.info = kInfo[gs];
#pragma unroll
    for (int q = 0; q < 5; ++q) o.cell[q] = kCells[gs][q];
    o.ffirst = kFopsFirst.m[gs];
    return o;
}

// ------------------------------------------------------------------------------------
// state <-> rows
// ------------------------------------------------------------------------------------
// Extract row R (bits 20R..20R+19 of the 400-bit little-endian player int): column c
// -> bit c.
__device__ __forceinline__ uint32_t plane_row(const uint64_t* w, int R) {
    const int bit = 20 * R, word = bit >> 6, off = bit & 63;
    uint64_t v = w[word] >> off;
    if (off > 44) v |= w[word + 1] << (64 - off);
    return (uint32_t)(v & 0xFFFFFull);
}

// Slab: one contiguous 464-byte record per lane (own planes, occupancy, compat RNG).
// All offsets are compile-time immediates from one per-lane base (the mover plane
// adds one per-lane term), rows move as dwordx4; the record stays L1/L2-resident.
#define SLAB_FIELDS 5
#define SLAB_RNG_BASE (SLAB_FIELDS * 20)
// Each lane's record starts on a 128-byte line (512-byte stride instead of 464): with
// FsLane's padding below, frontier-order config 3 31.9 -> 33.5 M playouts/s
// (profiles/r05/sweeps/r05b); the per-lane records of 262,144 resident lanes far exceed
// the L2 and the Infinity Cache, so every line a ply touches is a memory round trip
// frontier-order rollouts: the four players' table headers (mask, fill, used as uint16)
// live in the slab, in the line the occupancy plane ends in (read every ply anyway),
// instead of in the FsLane record's own header line
#define SLAB_HDR_BASE (SLAB_RNG_BASE + 16)
#define SLAB_WORDS 128
static_assert(SLAB_HDR_BASE + 6 <= SLAB_WORDS, "the table headers fit the slab");
struct Slab {
    uint32_t* base;  // = slab + slot * SLAB_WORDS (16-byte aligned)
    __device__ __forceinline__ uint32_t& at(int f, int R) const { return base[f * 20 + R]; }
    __device__ __forceinline__ uint32_t& word(int w) const { return base[w]; }
};

// ------------------------------------------------------------------------------------
// derive the mover's blocked / corner rows (engine/board.py:136-220 rules,
// frontier definition engine/board.py:247-313)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void derive_rows(const uint32_t (&own)[20], const uint32_t (&occ)[20],
                                            bool first, int p, uint32_t (&B)[20], uint32_t (&C)[20]) {
    // start corners: RED (0,0) BLUE (0,19) YELLOW (19,19) GREEN (19,0)
    const int crow = (p == 0 || p == 1) ? 0 : 19;
    const uint32_t cbit = (p == 0 || p == 3) ? 0x00000001u : 0x00080000u;
#pragma unroll
    for (int R = 0; R < 20; ++R) {
        const uint32_t up = R > 0 ? own[R - 1] : 0u;
        const uint32_t dn = R < 19 ? own[R + 1] : 0u;
        const uint32_t orth = own[R] | (own[R] << 1) | (own[R] >> 1) | up | dn;
        const uint32_t vd = up | dn;
        const uint32_t diag = ((vd << 1) | (vd >> 1)) & ROWMASK;
        const uint32_t blocked = occ[R] | orth | OFFBOARD;
        B[R] = blocked;
        const uint32_t cf = (R == crow) ? (cbit & ~occ[R]) : 0u;
        C[R] = first ? cf : (diag & ~blocked);
    }
}

// ------------------------------------------------------------------------------------
// the stencil scan
// ------------------------------------------------------------------------------------
// Mover planes.  B/C = blocked / corner rows; BP/CP = the same for a horizontal pair of
// cells (BP[R] = B[R] | B[R] >> 1), BV/CV for a vertical pair (BV[R] = B[R] | B[R + 1]):
// a pair of cells of a piece costs one term instead of two.  The stencil table
// (tools/gen_tables.py) covers the 410 cells of the 91 orientations with the fewest
// terms.  Each row is stored as one 64-bit word, C in the high half and B in the low
// half, so ONE v_lshrrev_b64 shifts a term's B and C rows together (the stream runs at
// the single-issue rate, where a 64-bit shift costs what a 32-bit one does).  Shifts are
// at most 3 (tools/gen_tables.py), so the C bits that enter B's top bits (>= 29) are
// never read, and B's bits 20..28 stay the OFFBOARD ones.
struct Planes {
    uint64_t BC[20], BCP[20], BCV[20];
    __device__ __forceinline__ uint32_t b(int R) const { return (uint32_t)BC[R]; }
    __device__ __forceinline__ uint32_t c(int R) const { return (uint32_t)(BC[R] >> 32); }
};

__device__ __forceinline__ void derive_rows(const uint32_t (&own)[20], const uint32_t (&occ)[20], bool first, int p,
                                            Planes& P) {
    uint32_t B[20], C[20];
    derive_rows(own, occ, first, p, B, C);
#pragma unroll
    for (int R = 0; R < 20; ++R) P.BC[R] = ((uint64_t)C[R] << 32) | B[R];
}

__device__ __forceinline__ void make_pairs(Planes& P) {
#pragma unroll
    for (int R = 0; R < 20; ++R) {
        // B's bit 31 (OFFBOARD) absorbs C's bit 0
        P.BCP[R] = P.BC[R] | (P.BC[R] >> 1);
        P.BCV[R] = R < 19 ? (P.BC[R] | P.BC[R + 1]) : P.BC[R];  // row 19: never a pair's top
    }
}

// popcount-accumulate as ONE v_bcnt_u32_b32 (the compiler otherwise reassociates the
// sum into bcnt(x,0) + v_add3 trees)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

// v_bitop3_b32 truth tables over (a, b, c) = (0xF0, 0xCC, 0xAA)
#define LUT_OR3 0xFE     // a | b | c
#define LUT_OR2_ANDN 0x54 // (a | b) & ~c
#define LUT_ANDN 0x30    // a & ~b
#define BITOP3(a, b, c, lut) __builtin_amdgcn_bitop3_b32((a), (b), (c), (lut))

// One stencil class: height H, static term sequence T... (t = piece row * 4 + kind).
// Term 0 sits at column 0 (no shift); term k >= 1 is shifted by the uniform column
// sh[k].  For every anchor row r < 21 - H calls f(r, ok) with ok = legal anchor
// columns (bit x = column x).
template <int H, int... T>
struct StencilClass {
    static constexpr int NT = sizeof...(T);
    static constexpr int NR = 21 - H;
    static constexpr int ts[NT] = {T...};

    template <int K>
    __device__ __forceinline__ static uint64_t tv(const Planes& P, int r, const uint32_t (&sh)[5]) {
        constexpr int d = ts[K] >> 2, kind = ts[K] & 3;
        const uint64_t v = kind == 1 ? P.BCP[r + d] : kind == 2 ? P.BCV[r + d] : P.BC[r + d];
        return K == 0 ? v : v >> sh[K];
    }
    __device__ __forceinline__ static uint32_t lo(uint64_t v) { return (uint32_t)v; }
    __device__ __forceinline__ static uint32_t hi(uint64_t v) { return (uint32_t)(v >> 32); }
    // OR of terms K.. into (b, c); the last C term folds into ok
    template <int K>
    __device__ __forceinline__ static uint32_t fold(const Planes& P, int r, const uint32_t (&sh)[5], uint32_t b,
                                                    uint32_t c) {
        if constexpr (K + 2 <= NT - 1) {
            const uint64_t t0 = tv<K>(P, r, sh), t1 = tv<K + 1>(P, r, sh);
            b = BITOP3(b, lo(t0), lo(t1), LUT_OR3);
            c = BITOP3(c, hi(t0), hi(t1), LUT_OR3);
            return fold<K + 2>(P, r, sh, b, c);
        } else if constexpr (K + 2 == NT) {  // two left: B merges both, C merges one + ok
            const uint64_t t0 = tv<K>(P, r, sh), t1 = tv<K + 1>(P, r, sh);
            b = BITOP3(b, lo(t0), lo(t1), LUT_OR3);
            c = c | hi(t0);
            return BITOP3(c, hi(t1), b, LUT_OR2_ANDN);
        } else if constexpr (K + 1 == NT) {  // one left
            const uint64_t t0 = tv<K>(P, r, sh);
            b = b | lo(t0);
            return BITOP3(c, hi(t0), b, LUT_OR2_ANDN);
        } else {
            return BITOP3(c, b, b, LUT_ANDN);
        }
    }
    // LANE_W1: w1 differs per lane (the lane-pair split of count_class_pair)
    template <bool LANE_W1 = false, typename F>
    __device__ __forceinline__ static void scan(const Planes& P, uint32_t w1, F&& f) {
        // Shift amounts go to VGPRs: a VALU op reading an SGPR is never dual-issued on
        // gfx950 (tools/valu_probe2.hip).  NOTE: the v_bcnt below keeps
        // the whole stream at the single-issue rate anyway, so today this is neutral.
        uint32_t sh[5];
        sh[0] = 0;
#pragma unroll
        for (int k = 1; k < NT; ++k) {
            const uint32_t v = (w1 >> (3 * (k - 1))) & 7u;
            if constexpr (LANE_W1) sh[k] = v;
            else asm("v_mov_b32 %0, %1" : "=v"(sh[k]) : "s"(v));
        }
        // row by row: without the barriers the scheduler interleaves all rows for ILP
        // and the live set no longer fits 3 waves per SIMD (other waves hide latency)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const uint64_t t0 = tv<0>(P, r, sh);
            f(r, fold<1>(P, r, sh, lo(t0), hi(t0)));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
};

// Per-orientation counts in LDS, 10 bits each, three per dword: orientation g lives in
// dword g / 3 at bit 10 * (g % 3), laid out [dword][lane] (31 dwords per lane).  The
// rollout zeroes a lane's dwords before each movegen and ds_add_u32's every count in
// (counts <= 400 < 1024, so fields never carry into each other).
#define CNT_DWORDS ((BK_NUM_ORIENTS + 2) / 3)
// rollout kernel: per-wave LDS area of 40 dwords per lane.  The counts (31 dwords) are
// dead once the move's orientation is picked; the same bytes then hold the mover's
// B/C rows 0..19 as [row][lane]{B, C} pairs for locate_move_lds.
#define ROLL_WORDS_PER_WAVE (40 * WAVE)
// resident 256-lane blocks per CU for k_rollout / k_advance (the launch bound).  4 (128
// VGPRs, 8 B/lane of scratch; 4 x 40 KB fills the CU's LDS exactly): config 3's 262,144
// playouts are then one per resident slot, 62.3 M vs 61.0 M playouts/s at 3 (168 VGPRs;
// profiles/r04/sweeps/r04i).  With the vertical-pair planes (tools/gen_tables.py
// BK_GEN_VPAIR=1, 243 instead of 287 terms) the kernel needs 2 (226 VGPRs) and measured
// 42.2 M vs 48.7 M playouts/s -- the lost latency hiding costs more than the 15 % fewer
// stencil ops
#ifndef ROLL_BLOCKS_PER_CU
#define ROLL_BLOCKS_PER_CU 4
#endif
// frontier tables smaller than this many slots are staged in LDS for place_frontier
// (0: probe the table in global memory).  k_rollout_fr: 64, so its area stays at the 40
// dwords per lane the counts and rows need and 4 blocks of 256 lanes fill a CU's LDS (4
// waves/SIMD); the ~12 % of plies whose mover has a 128-slot table probe it in place.
// k_mcts (config 5: 65,536 searches = one 256-lane block per CU, LDS to spare): 128.
#ifndef BK_FS_STAGE_FR
#define BK_FS_STAGE_FR 64
#endif
#ifndef BK_FS_STAGE_MCTS
#define BK_FS_STAGE_MCTS 128
#endif
// frontier-order kernels: per lane max(40, stage / 2) dwords; after the move is located
// the area also stages the mover's frontier table ([slot pair][lane])
#define ROLL_WORDS_STAGE(S) (((S) / 2 > 40 ? (S) / 2 : 40) * WAVE)
#define ROLL_WORDS_FR ROLL_WORDS_STAGE(BK_FS_STAGE_FR)
// resident 256-lane blocks per CU of k_rollout_fr (the launch bound).  The kernel reads
// the CPython cell hashes (3.2 KB) from global memory through the L1, so 4 blocks x 40 KB
// of areas fill the CU's LDS: at 4 blocks/CU (128 VGPRs, 256 B/lane of scratch, spills
// mostly on the cold paths) 31.8 M playouts/s vs 27.9 M at 3 blocks with the hashes in
// LDS, 26.8 M at 3 blocks with them in global memory (profiles/r04/sweeps/r04r).
#define FR_BLOCKS_PER_CU 4
// Tables probed in global memory read 8-slot chunks (FsetRef::gchunk, fs_probe);
// LDS-staged frontier tables resize through an LDS scratch (fs_resize_lds) where the
// caller has one, else through the record's global tmp (fs_resize).
#ifndef MCTS_BLOCKS_PER_CU
#define MCTS_BLOCKS_PER_CU 2
#endif

// Legal-move counts of one board-player for the class's table entries [i0, i1); with
// STORE, also the per-orientation counts (cl = this lane's dword 0, stride WAVE).
// Orientations whose piece no lane of the wave may still play are skipped with a
// uniform branch.
template <bool STORE, int H, int... T>
__device__ __forceinline__ uint32_t count_class(int i0, int i1, const Planes& P, uint32_t avail, uint32_t* cl) {
    uint32_t total = 0;
    uint32_t w0 = kClass[i0][0], w1 = kClass[i0][1];
#pragma unroll 1
    for (int i = i0; i < i1; ++i) {
        const int nx = i + 1 < i1 ? i + 1 : i;  // prefetch the next entry
        const uint32_t n0 = kClass[nx][0], n1 = kClass[nx][1];
        const uint32_t piece = w0 & 0xFFu;
        const int g = (int)(w0 >> 8);
        const bool av = (avail >> (piece - 1u)) & 1u;
        if (__builtin_amdgcn_ballot_w64(av) != 0ull) {
            uint32_t c = 0;
            StencilClass<H, T...>::scan(P, w1, [&](int, uint32_t ok) { c = bcnt_acc(ok, c); });
            c = av ? c : 0u;
            if constexpr (STORE) atomicAdd(cl + (g / 3) * WAVE, c << (10 * (g % 3)));
            total += c;
        }
        w0 = n0; w1 = n1;
    }
    return total;
}

// count_class for a lane PAIR that shares one board-player (k_mcts_pair): the even lane
// counts the class's entries i0, i0 + 2, ..., the odd lane i0 + 1, i0 + 3, ... (both
// entries of a pair run in the same instructions, with per-lane shift amounts, piece and
// orientation), so a class of n entries costs ceil(n / 2) scans instead of n.  Each
// orientation's count lands in the column of the lane that counted it; the other lane's
// field stays 0, so the two columns add up to the full count vector (pick_orient<true>).
template <bool STORE, int H, int... T>
__device__ __forceinline__ uint32_t count_class_pair(int i0, int i1, const Planes& P, uint32_t avail, uint32_t* cl,
                                                     bool odd) {
    uint32_t total = 0;
#pragma unroll 1
    for (int ia = i0; ia < i1; ia += 2) {
        const bool has_b = ia + 1 < i1;  // uniform
        const int ib = has_b ? ia + 1 : ia;
        const uint32_t a0 = kClass[ia][0], a1 = kClass[ia][1], b0 = kClass[ib][0], b1 = kClass[ib][1];
        const uint32_t w0 = odd ? b0 : a0, w1 = odd ? b1 : a1;
        const uint32_t piece = w0 & 0xFFu;
        const int g = (int)(w0 >> 8);
        const bool av = ((avail >> (piece - 1u)) & 1u) && (has_b || !odd);
        if (__builtin_amdgcn_ballot_w64(av) != 0ull) {
            uint32_t c = 0;
            StencilClass<H, T...>::template scan<true>(P, w1, [&](int, uint32_t ok) { c = bcnt_acc(ok, c); });
            c = av ? c : 0u;
            if constexpr (STORE) atomicAdd(cl + (g / 3) * WAVE, c << (10 * (g % 3)));
            total += c;
        }
    }
    return total;
}

// PAIR: lanes 2j and 2j + 1 hold the same board-player and split the entries
// (count_class_pair); each returns its share of the total.
template <bool STORE, bool PAIR = false>
__device__ __forceinline__ uint32_t movegen_counts(const Planes& P, uint32_t avail, uint32_t* cnt, int lane) {
    uint32_t t = 0;
    uint32_t* cl = cnt + lane;  // this lane's dwords; the orientation part is uniform
    if constexpr (STORE) {
#pragma unroll
        for (int j = 0; j < CNT_DWORDS; ++j) cl[j * WAVE] = 0u;
    }
    // opaque table offset (always 0): otherwise everything about the one-orientation
    // classes is hoisted out of the persistent loop and lives in (spilled) registers.
    // readfirstlane: an asm output counts as divergent, which would turn the table
    // loads and every shift amount into VGPR values.
    int tb0 = 0;
    asm volatile("" : "+s"(tb0));
    tb0 = __builtin_amdgcn_readfirstlane(tb0);
    // the running total is pinned after every class (the empty asm): left to itself the
    // compiler keeps the 49 class totals live to the end of the stencil and sums them
    // there, ~40 VGPRs that spilled in the frontier-order kernel
    if constexpr (PAIR) {
        const bool odd = (lane & 1) != 0;
#define BK_COUNT_CLASS(i0, i1, H, ...) t += count_class_pair<STORE, H, __VA_ARGS__>(i0 + tb0, i1 + tb0, P, avail, cl, odd); \
        asm volatile("" : "+v"(t));
        BK_CLASS_LIST(BK_COUNT_CLASS)
#undef BK_COUNT_CLASS
    } else {
#define BK_COUNT_CLASS(i0, i1, H, ...) t += count_class<STORE, H, __VA_ARGS__>(i0 + tb0, i1 + tb0, P, avail, cl); \
        asm volatile("" : "+v"(t));
        BK_CLASS_LIST(BK_COUNT_CLASS)
#undef BK_COUNT_CLASS
    }
    return t;
}

// Dense legal rows of every orientation (k_movegen): calls f(g, piece, ok[20])
template <int H, int... T, typename F>
__device__ __forceinline__ void rows_class(int i0, int i1, const Planes& P, F&& f) {
#pragma unroll 1
    for (int i = i0; i < i1; ++i) {
        const uint32_t w0 = kClass[i][0], w1 = kClass[i][1];
        uint32_t ok[20];
#pragma unroll
        for (int r = 0; r < 20; ++r) ok[r] = 0u;
        StencilClass<H, T...>::scan(P, w1, [&](int r, uint32_t v) { ok[r] = v; });
        f((int)(w0 >> 8), w0 & 0xFFu, ok);
    }
}

template <typename F>
__device__ __forceinline__ void all_rows(const Planes& P, F&& f) {
#define BK_ROWS_CLASS(i0, i1, H, ...) rows_class<H, __VA_ARGS__>(i0, i1, P, f);
    BK_CLASS_LIST(BK_ROWS_CLASS)
#undef BK_ROWS_CLASS
}

// orientation holding the k-th legal move (naive order: g ascending) and its rank in it.
// PAIR: the counts are split over this lane's column and the next one (movegen_counts<.., true>)
template <bool PAIR = false>
__device__ __forceinline__ int pick_orient(const uint32_t* cnt, int lane, uint32_t k, uint32_t& kk) {
    // dword level first (the three 10-bit fields summed), then the field inside the
    // dword that holds index k
    uint32_t run = 0, before = 0, hit = 0;
    int hd = CNT_DWORDS - 1;
    bool found = false;
#pragma unroll 1
    for (int h0 = 0; h0 < CNT_DWORDS; h0 += 8) {  // 8 LDS reads in flight per batch
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = (h0 + j < CNT_DWORDS) ? cnt[(h0 + j) * WAVE + lane] + (PAIR ? cnt[(h0 + j) * WAVE + lane + 1] : 0u)
                                         : 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t s = (v[j] & 0x3FFu) + ((v[j] >> 10) & 0x3FFu) + (v[j] >> 20);
            const bool in = !found && k < run + s;
            hd = in ? h0 + j : hd;
            before = in ? run : before;
            hit = in ? v[j] : hit;
            found |= in;
            run += s;
        }
    }
    uint32_t r = k - before;
    const uint32_t c0 = hit & 0x3FFu, c1 = (hit >> 10) & 0x3FFu;
    int f = 2;
    if (r < c0) {
        f = 0;
    } else if (r < c0 + c1) {
        f = 1;
        r -= c0;
    } else {
        r -= c0 + c1;
    }
    kk = r;
    return found ? 3 * hd + f : BK_NUM_ORIENTS - 1;
}

// Recompute orientation gs (per-lane, divergent) row r_ok values with per-lane
// row selects, then locate the kk-th legal move in naive order (anchor row-major).
__device__ __forceinline__ void locate_move(int gs, uint32_t kk, const uint32_t (&B)[20],
                                            const uint32_t (&C)[20], int& out_r, int& out_c) {
    const uint32_t info = kInfo[gs];
    const int n = (int)((info >> 8) & 0xFFu);
    uint32_t cd[5], cc[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t cell = kCells[gs][k];
        cd[k] = cell >> 8;
        cc[k] = cell & 0xFFu;
    }
    int found_r = -1, found_c = 0;
    uint32_t rem = kk;
#pragma unroll
    for (int r = 0; r < 20; ++r) {
        uint32_t ab = 0, ac = 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (k < n) {
                const uint32_t d = cd[k];
                uint32_t b = 0xFFFFFFFFu, cv = 0u;
#pragma unroll
                for (int dd = 0; dd < 5; ++dd)
                    if (r + dd < 20 && d == (uint32_t)dd) { b = B[r + dd]; cv = C[r + dd]; }
                ab |= b >> cc[k];
                ac |= cv >> cc[k];
            }
        }
        const uint32_t ok = ac & ~ab;
        const uint32_t pc = __builtin_popcount(ok);
        if (found_r < 0) {
            if (rem < pc) {
                // rem-th set bit from the bottom (column ascending)
                uint32_t x = ok;
                for (uint32_t j = 0; j < rem; ++j) x &= x - 1u;
                found_r = r;
                found_c = __builtin_ctz(x);
            } else {
                rem -= pc;
            }
        }
    }
    out_r = found_r;
    out_c = found_c;
}

// locate_move with the mover's B/C rows in LDS (rows[R * WAVE] = {B[R], C[R]}, R < 20):
// the per-lane cell rows become per-lane LDS addresses instead of 5-way register
// selects.  Cells beyond the orientation's count repeat cell 0 (ORing a term twice is
// harmless).  Anchor rows past 20 - height cannot hold the piece: they are evaluated
// at the last valid row (so every read stays in rows 0..19) and then dropped.
__device__ __forceinline__ void locate_move_lds(const OrientRow& orow, uint32_t kk, const uint2* rows, int& out_r,
                                                int& out_c) {
    const uint32_t info = orow.info;
    const int n = (int)((info >> 8) & 0xFFu);
    const int rlim = 20 - (int)((info >> 16) & 0xFFu);
    const uint2* base[5];
    uint32_t sh[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t cell = k < n ? orow.cell[k] : orow.cell[0];
        base[k] = rows + (cell >> 8) * WAVE;
        sh[k] = cell & 0xFFu;
    }
    int found_r = -1, found_c = 0;
    uint32_t rem = kk;
#pragma unroll
    for (int r = 0; r < 20; ++r) {
        const int rr = r < rlim ? r : rlim;
        uint2 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = base[k][rr * WAVE];
        uint32_t ab = BITOP3(v[0].x >> sh[0], v[1].x >> sh[1], v[2].x >> sh[2], LUT_OR3);
        uint32_t ac = BITOP3(v[0].y >> sh[0], v[1].y >> sh[1], v[2].y >> sh[2], LUT_OR3);
        ab = BITOP3(ab, v[3].x >> sh[3], v[4].x >> sh[4], LUT_OR3);
        ac = BITOP3(ac, v[3].y >> sh[3], v[4].y >> sh[4], LUT_OR3);
        const uint32_t ok = r <= rlim ? (ac & ~ab) : 0u;
        const uint32_t pc = __builtin_popcount(ok);
        if (found_r < 0) {
            if (rem < pc) {
                uint32_t x = ok;  // rem-th set bit from the bottom (column ascending)
                for (uint32_t j = 0; j < rem; ++j) x &= x - 1u;
                found_r = r;
                found_c = __builtin_ctz(x);
            } else {
                rem -= pc;
            }
        }
    }
    out_r = found_r;
    out_c = found_c;
}
__device__ __forceinline__ void locate_move_lds(int gs, uint32_t kk, const uint2* rows, int& out_r, int& out_c) {
    locate_move_lds(orient_row(gs), kk, rows, out_r, out_c);
}

// Frontier-order variant (BK_ORDER_FRONTIER): the kk-th anchor of orientation gs in the
// reference's list order (engine/move_generator.py:261-559).  Pass 1 writes the legal
// anchors of gs over the B half of each LDS row.  Pass 2 walks the mover's frontier set
// in slot order and the orientation's cells in order; an anchor counts at its first
// (frontier cell, cell k) hit, and its bit is cleared when it is counted.
// Pass 1 of locate_move_frontier alone: the legal anchors of gs over the C half of each
// LDS row (rows[r].y; the B half stays)
__device__ __forceinline__ void locate_pass1(int gs, uint2* rows) {
    const uint32_t info = kInfo[gs];
    const int n = (int)((info >> 8) & 0xFFu);
    const int rlim = 20 - (int)((info >> 16) & 0xFFu);
    const uint2* base[5];
    uint32_t sh[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t cell = kCells[gs][k < n ? k : 0];
        base[k] = rows + (cell >> 8) * WAVE;
        sh[k] = cell & 0xFFu;
    }
#pragma unroll
    for (int r = 0; r < 20; ++r) {
        const int rr = r < rlim ? r : rlim;
        uint2 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = base[k][rr * WAVE];
        uint32_t ab = BITOP3(v[0].x >> sh[0], v[1].x >> sh[1], v[2].x >> sh[2], LUT_OR3);
        uint32_t ac = BITOP3(v[0].y >> sh[0], v[1].y >> sh[1], v[2].y >> sh[2], LUT_OR3);
        ab = BITOP3(ab, v[3].x >> sh[3], v[4].x >> sh[4], LUT_OR3);
        ac = BITOP3(ac, v[3].y >> sh[3], v[4].y >> sh[4], LUT_OR3);
        rows[r * WAVE].y = r <= rlim ? (ac & ~ab) : 0u;
    }
}

// RS: uint4 distance between 16-slot runs of the table (2: a plain array; 64: the lane
// pair's LDS-DMA stage of k_mcts_pair)
template <int RS = 2>
__device__ __forceinline__ void locate_move_frontier(const OrientRow& orow, uint32_t kk, uint2* rows,
                                                     const int16_t* key, int mask, int& out_r, int& out_c) {
    const uint32_t info = orow.info;
    const int n = (int)((info >> 8) & 0xFFu);
    const int rlim = 20 - (int)((info >> 16) & 0xFFu);
    const uint2* base[5];
    uint32_t sh[5];
    int cd[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t cell = k < n ? orow.cell[k] : orow.cell[0];
        base[k] = rows + (cell >> 8) * WAVE;
        sh[k] = cell & 0xFFu;
        cd[k] = (int)(cell >> 8);
    }
    uint32_t arows = 0;  // bit r + 4: anchor row r holds a legal anchor (a superset later)
#pragma unroll
    for (int r = 0; r < 20; ++r) {
        const int rr = r < rlim ? r : rlim;
        uint2 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = base[k][rr * WAVE];
        uint32_t ab = BITOP3(v[0].x >> sh[0], v[1].x >> sh[1], v[2].x >> sh[2], LUT_OR3);
        uint32_t ac = BITOP3(v[0].y >> sh[0], v[1].y >> sh[1], v[2].y >> sh[2], LUT_OR3);
        ab = BITOP3(ab, v[3].x >> sh[3], v[4].x >> sh[4], LUT_OR3);
        ac = BITOP3(ac, v[3].y >> sh[3], v[4].y >> sh[4], LUT_OR3);
        // the anchors go to the C half: row r's C word is not read again (later rows
        // read rows >= r + 1), and the B half stays intact for frontier_ops
        const uint32_t okr = r <= rlim ? (ac & ~ab) : 0u;
        rows[r * WAVE].y = okr;
        arows |= okr ? (1u << (r + 4)) : 0u;
    }
    // Pass 2 reads the table 16 slots per pair of uint4 loads into registers, all
    // indices static (a dynamically indexed key array would live in scratch memory); the
    // next 16 slots' loads are issued before this batch is walked.  Per frontier cell f =
    // (fr, fc) the new anchors of piece row d (anchor row fr - d) are the legal, not yet
    // counted anchors among columns fc - c of the row's cells: one LDS row read and a mask
    // (rev[d] has bit 4 - c per cell (d, c); (rev[d] << fc) >> 4 puts them at fc - c).
    // A slot whose anchors hold the kk-th is resolved in cell order at the end (the
    // anchors of one frontier cell are distinct, and counting them as a set keeps every
    // other slot's contribution exact).
    const int H = (int)((info >> 16) & 0xFFu);
    const uint32_t hmask = (1u << H) - 1u;
    uint32_t rev[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
        for (int d = 0; d < 5; ++d) rev[d] |= (k < n && cd[k] == d) ? (1u << (4 - (int)sh[k])) : 0u;
    uint32_t cnt = 0;
    int hit_f = -1;
    const bk_u4_alias* k4 = reinterpret_cast<const bk_u4_alias*>(key);
    uint4 qa = k4[0], qb = k4[1];  // tables hold >= 8 slots; the storage has 256
#pragma unroll 1
    for (int b0 = 0; b0 <= mask && hit_f < 0; b0 += 16) {
        const int nb0 = b0 + 16 <= mask ? b0 + 16 : b0;
        const uint4 na = k4[(nb0 >> 4) * RS], nb = k4[(nb0 >> 4) * RS + 1];
        const uint32_t w[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
        // the batch's slots that can add an anchor, then one divergent pass over just
        // those: the wave runs the row reads max-over-lanes-of-relevant-slots times
        uint32_t rel = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int f = (int)(int16_t)((j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFFu));
            const int fr = f >= 0 ? f / 20 : 0;
            rel |= (f >= 0 && b0 + j <= mask && ((arows >> (fr + 5 - H)) & hmask)) ? (1u << j) : 0u;
        }
#pragma unroll 1
        while (rel && hit_f < 0) {
            const int j = __builtin_ctz(rel);
            rel &= rel - 1u;
            uint32_t wj = w[0];
#pragma unroll
            for (int q = 1; q < 8; ++q) wj = (j >> 1) == q ? w[q] : wj;
            const int f = (int)(int16_t)((j & 1) ? (wj >> 16) : (wj & 0xFFFFu));
            const int fr = f / 20, fc = f - 20 * fr;
            uint32_t hm[5], tot = 0;
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                const int ar = fr - d;
                hm[d] = (d < H && ar >= 0) ? (rows[(ar < 0 ? 0 : ar) * WAVE].y & ((rev[d] << fc) >> 4)) : 0u;
                tot += __builtin_popcount(hm[d]);
            }
            if (cnt + tot > kk) { hit_f = f; continue; }
#pragma unroll
            for (int d = 0; d < 5; ++d)
                if (hm[d]) rows[(fr - d) * WAVE].y &= ~hm[d];
            cnt += tot;
        }
        qa = na; qb = nb;
    }
    int found_r = -1, found_c = 0;
    if (hit_f >= 0) {  // the (kk - cnt)-th new anchor of frontier cell hit_f, in cell order
        const int fr = hit_f / 20, fc = hit_f - 20 * fr;
        uint32_t rem = kk - cnt;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (k >= n || found_r >= 0) continue;
            const int ar = fr - cd[k], acl = fc - (int)sh[k];
            if (ar < 0 || acl < 0) continue;
            if (!((rows[ar * WAVE].y >> acl) & 1u)) continue;
            if (rem == 0u) { found_r = ar; found_c = acl; } else { --rem; }
        }
    }
    out_r = found_r;
    out_c = found_c;
}
template <int RS = 2>
__device__ __forceinline__ void locate_move_frontier(int gs, uint32_t kk, uint2* rows, const int16_t* key, int mask,
                                                     int& out_r, int& out_c) {
    locate_move_frontier<RS>(orient_row(gs), kk, rows, key, mask, out_r, out_c);
}

// locate_move_frontier for a lane PAIR holding one search (k_mcts_pair): both lanes call
// it with the even lane's orientation, rank, table and LDS row column (rows).  Pass 1:
// the even lane computes anchor rows 0..9 and the odd lane rows 10..19 (all reads before
// the writes, so no lane overwrites a C row the other still reads).  Pass 2: both walk
// the same table slots; the even lane tests piece rows d = 0..2 and the odd lane d = 3, 4,
// and the two partial counts are added across the pair (one DPP move), so a slot costs
// three row reads instead of five.  Anchors are cleared by the lane that counted them
// (different rows), so the walk sees exactly the single-lane state.  Same result as
// locate_move_frontier in both lanes.
template <int RS = 2>
__device__ __forceinline__ void locate_frontier_pair(int gs, uint32_t kk, uint2* rows, const int16_t* key, int mask,
                                                     bool odd, int& out_r, int& out_c) {
    const uint32_t info = kInfo[gs];
    const int n = (int)((info >> 8) & 0xFFu);
    const int rlim = 20 - (int)((info >> 16) & 0xFFu);
    const uint2* base[5];
    uint32_t sh[5];
    int cd[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t cell = kCells[gs][k < n ? k : 0];
        base[k] = rows + (cell >> 8) * WAVE;
        sh[k] = cell & 0xFFu;
        cd[k] = (int)(cell >> 8);
    }
    const int r0 = odd ? 10 : 0;
    uint32_t okv[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const int r = r0 + i;
        const int rr = r < rlim ? r : rlim;
        uint2 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = base[k][rr * WAVE];
        uint32_t ab = BITOP3(v[0].x >> sh[0], v[1].x >> sh[1], v[2].x >> sh[2], LUT_OR3);
        uint32_t ac = BITOP3(v[0].y >> sh[0], v[1].y >> sh[1], v[2].y >> sh[2], LUT_OR3);
        ab = BITOP3(ab, v[3].x >> sh[3], v[4].x >> sh[4], LUT_OR3);
        ac = BITOP3(ac, v[3].y >> sh[3], v[4].y >> sh[4], LUT_OR3);
        okv[i] = r <= rlim ? (ac & ~ab) : 0u;
    }
    uint32_t arows = 0;  // bit r + 4: anchor row r holds a legal anchor (a superset later)
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        rows[(r0 + i) * WAVE].y = okv[i];
        arows |= okv[i] ? (1u << (r0 + i + 4)) : 0u;
    }
    arows |= (uint32_t)pair_other((int)arows);
    const int H = (int)((info >> 16) & 0xFFu);
    const uint32_t hmask = (1u << H) - 1u;
    uint32_t rev[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
        for (int d = 0; d < 5; ++d) rev[d] |= (k < n && cd[k] == d) ? (1u << (4 - (int)sh[k])) : 0u;
    // this lane's piece rows d = d0 + t (t < 3 even, t < 2 odd)
    const int d0 = odd ? 3 : 0;
    uint32_t rt[3];
    rt[0] = odd ? rev[3] : rev[0];
    rt[1] = odd ? rev[4] : rev[1];
    rt[2] = odd ? 0u : rev[2];
    uint32_t cnt = 0;
    int hit_f = -1;
    const bk_u4_alias* k4 = reinterpret_cast<const bk_u4_alias*>(key);
    uint4 qa = k4[0], qb = k4[1];  // tables hold >= 8 slots; the storage has 256
#pragma unroll 1
    for (int b0 = 0; b0 <= mask && hit_f < 0; b0 += 16) {
        const int nb0 = b0 + 16 <= mask ? b0 + 16 : b0;
        const uint4 na = k4[(nb0 >> 4) * RS], nb = k4[(nb0 >> 4) * RS + 1];
        const uint32_t w[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
        uint32_t rel = 0;  // as locate_move_frontier (the pair's lanes hold the same mask)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int f = (int)(int16_t)((j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFFu));
            const int fr = f >= 0 ? f / 20 : 0;
            rel |= (f >= 0 && b0 + j <= mask && ((arows >> (fr + 5 - H)) & hmask)) ? (1u << j) : 0u;
        }
#pragma unroll 1
        while (rel && hit_f < 0) {
            const int j = __builtin_ctz(rel);
            rel &= rel - 1u;
            uint32_t wj = w[0];
#pragma unroll
            for (int q = 1; q < 8; ++q) wj = (j >> 1) == q ? w[q] : wj;
            const int f = (int)(int16_t)((j & 1) ? (wj >> 16) : (wj & 0xFFFFu));
            const int fr = f / 20, fc = f - 20 * fr;
            uint32_t hm[3], tot = 0;
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const int d = d0 + t;
                const int ar = fr - d;
                hm[t] = (d < H && ar >= 0) ? (rows[(ar < 0 ? 0 : ar) * WAVE].y & ((rt[t] << fc) >> 4)) : 0u;
                tot += __builtin_popcount(hm[t]);
            }
            const uint32_t both = tot + (uint32_t)pair_other((int)tot);
            if (cnt + both > kk) { hit_f = f; continue; }
#pragma unroll
            for (int t = 0; t < 3; ++t)
                if (hm[t]) rows[(fr - d0 - t) * WAVE].y &= ~hm[t];
            cnt += both;
        }
        qa = na; qb = nb;
    }
    int found_r = -1, found_c = 0;
    if (hit_f >= 0) {  // the (kk - cnt)-th new anchor of frontier cell hit_f, in cell order
        const int fr = hit_f / 20, fc = hit_f - 20 * fr;
        uint32_t rem = kk - cnt;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (k >= n || found_r >= 0) continue;
            const int ar = fr - cd[k], acl = fc - (int)sh[k];
            if (ar < 0 || acl < 0) continue;
            if (!((rows[ar * WAVE].y >> acl) & 1u)) continue;
            if (rem == 0u) { found_r = ar; found_c = acl; } else { --rem; }
        }
    }
    out_r = found_r;
    out_c = found_c;
}

// The set operations of update_frontier_after_move that CHANGE the mover's set.  The
// reference runs 9 ops per placed cell q (o = 0: discard the cell, 1..4: add the
// diagonals (-1,-1) (-1,1) (1,-1) (1,1) when addable, 5..8: discard the orthogonals
// (-1,0) (1,0) (0,-1) (0,1)); most are no-ops (an add of a member, a discard of a
// non-member), and a no-op leaves the CPython table untouched.  Membership is known
// without probing the table, from the board alone:
// * an EMPTY cell is a member iff it is on the true frontier (diagonal to own, not
//   orthogonal to own), or, before the player's first move, iff it is the start corner
//   (init_frontier_for_player, engine/board.py:389-404): adds happen exactly when a cell
//   joins the true frontier, discards exactly when it leaves;
// * an own cell is never a member (discarded when placed);
// * a cell another player occupied may be a stale member: a discard of it is a real op
//   whenever it is diagonal and not orthogonal to own (conservative; a discard of a
//   non-member is a harmless no-op).
// Adds target empty, non-orthogonal cells only, so no key is both added and discarded
// within a move; a key added twice (a diagonal of two cells, e.g. inside the U piece) or
// discarded twice (an orthogonal of two cells) is real at most at its first op
// (kFopsFirst).
// Bit 9 q + o of the result marks the ops to run, in the reference's order.  Window:
// 7 x 7 bits, rows ar - 1 .. ar + 5 and columns ac - 1 .. ac + 5 (bit 7 i + j).
// rows[R * WAVE].x = the mover's blocked rows BEFORE the move; slab = own planes before
// or after the move (the piece's cells m are masked out).
// FROM_SLAB: the blocked rows are derived from the slab (occupancy and own rows before
// the move) instead of read from the LDS rows (MCTS replay, where no movegen ran).
template <bool FROM_SLAB = false>
__device__ __forceinline__ uint64_t frontier_ops(const uint2* rows, const Slab& slab, int p, bool first,
                                                 const OrientRow& orow, int ar, int ac, const uint32_t (&m)[5]) {
    uint32_t o[9];  // own rows ar - 2 .. ar + 6 before the move
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        const int R = ar - 2 + j;
        const uint32_t pr = (j >= 2 && j <= 6) ? m[j - 2] : 0u;
        const uint32_t v = slab.at(p, R < 0 ? 0 : R > 19 ? 19 : R);
        o[j] = (R >= 0 && R <= 19) ? (v & ~pr) : 0u;
    }
    const int crow = (p == 0 || p == 1) ? 0 : 19;
    const uint32_t cbit = (p == 0 || p == 3) ? 0x00000001u : 0x00080000u;
    uint64_t wm = 0, wa = 0;  // maybe-member / real-add windows
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const int R = ar - 1 + i;
        const bool inb = R >= 0 && R <= 19;
        const uint32_t own = o[i + 1], up = o[i], dn = o[i + 2];
        const uint32_t orth = own | (own << 1) | (own >> 1) | up | dn;
        const uint32_t vd = up | dn;
        const uint32_t diag = ((vd << 1) | (vd >> 1)) & ROWMASK;
        const int Rc = R < 0 ? 0 : R > 19 ? 19 : R;
        const uint32_t b = !inb ? ~0u : FROM_SLAB ? (slab.at(4, Rc) | orth | OFFBOARD) : rows[Rc * WAVE].x;
        const uint32_t pr = (i >= 1 && i <= 5) ? m[i - 1] : 0u;
        const uint32_t pu = (i >= 2) ? m[i - 2] : 0u, pd = (i <= 4) ? m[i] : 0u;
        const uint32_t addable = ~(b | pr | (pr << 1) | (pr >> 1) | pu | pd) & ROWMASK;
        const uint32_t corner = (R == crow) ? cbit : 0u;
        const uint32_t mm = inb ? (first ? corner : (diag & ~orth)) : 0u;   // maybe a member
        const uint32_t mem = inb ? (first ? corner : (diag & ~b)) : 0u;     // a member (empty cells)
        const uint32_t ra = addable & ~mem;
        wm |= (uint64_t)(((mm << 1) >> ac) & 0x7Fu) << (7 * i);
        wa |= (uint64_t)(((ra << 1) >> ac) & 0x7Fu) << (7 * i);
    }
    // cell q's 3 x 3 neighbourhood moved to window bits 0..2, 7..9, 14..16 (centre 8), then
    // op o's bit gathered to bit o: discards (o = 0, 5..8) from wm, adds (1..4) from wa
    uint64_t real = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const uint32_t cell = orow.cell[q];  // entries past the piece's cells: masked below
        const int sh = ((int)(cell >> 8) + 1) * 7 + (int)(cell & 0xFFu) + 1 - 8;
        const uint32_t tm = (uint32_t)(wm >> sh), ta = (uint32_t)(wa >> sh);
        const uint32_t code = ((tm >> 8) & 1u) | ((ta << 1) & 2u) | (ta & 4u) | ((ta >> 11) & 8u) |
                              ((ta >> 12) & 16u) | ((tm << 4) & 32u) | ((tm >> 9) & 64u) | (tm & 128u) |
                              ((tm >> 1) & 256u);
        real |= (uint64_t)code << (9 * q);
    }
    real &= orow.ffirst;
    // the LDS rows of this lane are overwritten by other lanes' table staging right after
    // this call: every load above must complete first (no sinking past those stores)
    uint32_t lo = (uint32_t)real, hi = (uint32_t)(real >> 32);
    asm volatile("" : "+v"(lo), "+v"(hi) : : "memory");
    return ((uint64_t)hi << 32) | lo;
}
template <bool FROM_SLAB = false>
__device__ __forceinline__ uint64_t frontier_ops(const uint2* rows, const Slab& slab, int p, bool first, int gs,
                                                 int ar, int ac, const uint32_t (&m)[5]) {
    return frontier_ops<FROM_SLAB>(rows, slab, p, first, orient_row(gs), ar, ac, m);
}

// ------------------------------------------------------------------------------------
// random streams
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t philox_u32(uint32_t c0, uint32_t c1, uint64_t key) {
    uint32_t x0 = c0, x1 = c1, x2 = 0x5bd1e995u, x3 = 0u;
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, x0), lo0 = 0xD2511F53u * x0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, x2), lo1 = 0xCD9E8D57u * x2;
        const uint32_t y0 = hi1 ^ x1 ^ k0, y2 = hi0 ^ x3 ^ k1;
        x0 = y0; x1 = lo1; x2 = y2; x3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return x0;
}

__device__ __forceinline__ uint32_t mask_for(uint32_t rng) {
    uint32_t m = rng;
    m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
    return m;
}

__device__ __forceinline__ uint32_t mt_init_step(uint32_t x, uint32_t j) {
    return 1812433253u * (x ^ (x >> 30)) + j;
}

// numpy RandomState(seed) MT19937 stream restricted to its first 227 outputs, which
// need only the init_genrand sequence (no stored 624-word state): output i =
// temper(mt[i+397] ^ twist(mt[i], mt[i+1])).  (agents/random_agent.py:29,49)
struct MtCursor {
    uint32_t i, a, b, c;  // a = mt[i], b = mt[i+1], c = mt[i+397]
};

__device__ __forceinline__ MtCursor mt_cursor_init(uint32_t seed) {
    MtCursor m;
    m.i = 0; m.a = seed;
    m.b = mt_init_step(seed, 1);
    uint32_t x = m.b;
    for (uint32_t j = 2; j <= 397; ++j) x = mt_init_step(x, j);
    m.c = x;
    return m;
}

__device__ __forceinline__ uint32_t mt_cursor_next(MtCursor& m, bool& overflow) {
    if (m.i >= 227u) overflow = true;
    const uint32_t y = (m.a & 0x80000000u) | (m.b & 0x7fffffffu);
    uint32_t v = m.c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    v ^= v >> 11; v ^= (v << 7) & 0x9d2c5680u; v ^= (v << 15) & 0xefc60000u; v ^= v >> 18;
    m.i += 1;
    m.a = m.b;
    m.b = mt_init_step(m.b, m.i + 1);
    m.c = mt_init_step(m.c, m.i + 397);
    return v;
}

// ------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------
struct MovegenArgs {
    const bk_state* states;
    const uint8_t* players;  // NULL: all 4 players of each state (has_moves mode)
    int32_t n;
    uint32_t* out_rows;      // n x 91 x 20 (normal layout, bit c = column c) or NULL
    uint32_t* out_count;     // n or NULL
    uint8_t* out_mask4;      // has_moves mode
    int32_t groups;          // k_movegen_g: orientation groups per board-player
    uint64_t* out_mask;      // k_movegen_m: n x 91 x 7 (bit 20 r + c of the 400-bit mask) or NULL
    uint32_t part_masks[13][3];  // k_movegen_ml: bit i of part q = stencil entry i's orientation in range q
};

__device__ __forceinline__ void load_state_rows(const bk_state* s, uint32_t (&own)[4][20], uint32_t (&occ)[20]) {
#pragma unroll
    for (int R = 0; R < 20; ++R) occ[R] = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int R = 0; R < 20; ++R) {
            own[p][R] = plane_row(s->planes[p], R);
            occ[R] |= own[p][R];
        }
}

// Dense rows of the class's table entries i0 <= i < i1 with i % G == grp (k_movegen_g)
template <int H, int... T, typename F>
__device__ __forceinline__ void rows_class_group(int i0, int i1, int grp, int G, const Planes& P, F&& f) {
    int first = i0 + ((grp - i0 % G) + G) % G;
#pragma unroll 1
    for (int i = first; i < i1; i += G) {
        const uint32_t w0 = kClass[i][0], w1 = kClass[i][1];
        uint32_t ok[20];
#pragma unroll
        for (int r = 0; r < 20; ++r) ok[r] = 0u;
        StencilClass<H, T...>::scan(P, w1, [&](int r, uint32_t v) { ok[r] = v; });
        f((int)(w0 >> 8), w0 & 0xFFu, ok);
    }
}

// Batched movegen with the 91 orientations of each board-player split over G = a.groups
// wave-uniform groups (every G-th stencil-table entry): block b = one 64-lane wave for
// board-players 64 * (b / G) .. + 63 and group b % G, so 4,096 board-players run as
// 64 G waves instead of 64 (config 2 fills the chip).  Counts are summed with one
// atomicAdd per (board-player, group) into the zeroed out_count.
#define MG_GROUPS_MAX 91
#define MG_GROUPS_DEFAULT_MAX 32
#if BK_DEF(BK_U_MOVEGEN)
__global__ __launch_bounds__(WAVE) void k_movegen_g(MovegenArgs a) {
    const int G = a.groups;
    const int grp = blockIdx.x % G;
    const int i = (blockIdx.x / G) * WAVE + threadIdx.x;
    const bool live = i < a.n;
    const int idx = live ? i : 0;
    const bk_state* s = a.states + idx;
    const int p = a.players[idx] & 3;
    uint32_t own[20], occ[20];
#pragma unroll
    for (int R = 0; R < 20; ++R) { occ[R] = 0; own[R] = 0; }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int R = 0; R < 20; ++R) {
            const uint32_t row = plane_row(s->planes[q], R);
            occ[R] |= row;
            own[R] |= (q == p) ? row : 0u;
        }
    Planes P;
    derive_rows(own, occ, (s->first_move >> p) & 1u, p, P);
    make_pairs(P);
    const uint32_t avail = live ? (~s->used[p] & 0x1FFFFFu) : 0u;
    uint32_t total = 0;
    auto emit = [&](int g, uint32_t piece, const uint32_t (&ok)[20]) {
        const bool av = (avail >> (piece - 1u)) & 1u;
        uint4* dst = a.out_rows ? reinterpret_cast<uint4*>(a.out_rows + ((size_t)idx * BK_NUM_ORIENTS + g) * 20)
                                : nullptr;
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            uint4 v;
            v.x = av ? ok[4 * q + 0] : 0u;
            v.y = av ? ok[4 * q + 1] : 0u;
            v.z = av ? ok[4 * q + 2] : 0u;
            v.w = av ? ok[4 * q + 3] : 0u;
            total += __builtin_popcount(v.x) + __builtin_popcount(v.y) + __builtin_popcount(v.z) +
                     __builtin_popcount(v.w);
            if (live && dst) dst[q] = v;
        }
    };
#define BK_ROWS_GROUP(i0, i1, H, ...) rows_class_group<H, __VA_ARGS__>(i0, i1, grp, G, P, emit);
    BK_CLASS_LIST(BK_ROWS_GROUP)
#undef BK_ROWS_GROUP
    if (live && a.out_count && total) atomicAdd(a.out_count + i, total);
}
#else
__global__ void k_movegen_g(MovegenArgs a);
#endif

// k_movegen_g with the SURVEY 8(b) output: each orientation's legal anchors as one
// 400-bit mask (7 u64, bit 20 r + c, the reference's player_bits numbering), 5,096 B per
// board-player instead of 91 x 20 row words (7,280 B).  XCD-aware grid: block b runs on
// XCD b % 8 (round-robin dispatch), and the G group waves of one 64-board-player set all
// get blocks with the same b % 8, so the set's states are fetched from HBM once into that
// XCD's L2 (not once per XCD) and the partial 128-B lines of one board's mask, written by
// different group waves, merge in the same L2.
#define MG_XCDS 8
#if BK_DEF(BK_U_MOVEGEN)
__global__ __launch_bounds__(WAVE) void k_movegen_m(MovegenArgs a) {
    const int G = a.groups;
    const int xcd = blockIdx.x % MG_XCDS, j = blockIdx.x / MG_XCDS;
    const int set = xcd + MG_XCDS * (j / G), grp = j % G;
    const int i = set * WAVE + threadIdx.x;
    const bool live = i < a.n;
    const int idx = live ? i : 0;
    const bk_state* s = a.states + idx;
    const int p = a.players[idx] & 3;
    uint32_t own[20], occ[20];
#pragma unroll
    for (int R = 0; R < 20; ++R) { occ[R] = 0; own[R] = 0; }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int R = 0; R < 20; ++R) {
            const uint32_t row = plane_row(s->planes[q], R);
            occ[R] |= row;
            own[R] |= (q == p) ? row : 0u;
        }
    Planes P;
    derive_rows(own, occ, (s->first_move >> p) & 1u, p, P);
    make_pairs(P);
    const uint32_t avail = live ? (~s->used[p] & 0x1FFFFFu) : 0u;
    uint32_t total = 0;
    auto emit = [&](int g, uint32_t piece, const uint32_t (&ok)[20]) {
        const bool av = (avail >> (piece - 1u)) & 1u;
        uint64_t w[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 20; ++r) {
            const uint32_t v = av ? ok[r] : 0u;
            total += __builtin_popcount(v);
            constexpr int kBits = 20;
            const int off = kBits * r, q = off >> 6, sh = off & 63;  // compile-time per r
            w[q] |= (uint64_t)v << sh;
            if (sh > 64 - kBits) w[q + 1] |= (uint64_t)v >> (64 - sh);
        }
        if (live && a.out_mask) {
            // 16-byte-aligned stores (the width WRITE_SIZE counts exactly): the 56-byte
            // piece starts at an even or odd word (637 and 7 are odd), so it is three
            // 16-byte stores and one 8-byte store at the front or the back
            const size_t o = ((size_t)idx * BK_NUM_ORIENTS + g) * 7;
            uint64_t* dst = a.out_mask + o;
            const bool odd = ((o + ((uintptr_t)a.out_mask >> 3)) & 1u) != 0;
            uint64_t* d16 = odd ? dst + 1 : dst;
            const uint64_t p0 = odd ? w[1] : w[0], p1 = odd ? w[2] : w[1], p2 = odd ? w[3] : w[2];
            const uint64_t p3 = odd ? w[4] : w[3], p4 = odd ? w[5] : w[4], p5 = odd ? w[6] : w[5];
            reinterpret_cast<uint4*>(d16)[0] = make_uint4((uint32_t)p0, (uint32_t)(p0 >> 32), (uint32_t)p1, (uint32_t)(p1 >> 32));
            reinterpret_cast<uint4*>(d16)[1] = make_uint4((uint32_t)p2, (uint32_t)(p2 >> 32), (uint32_t)p3, (uint32_t)(p3 >> 32));
            reinterpret_cast<uint4*>(d16)[2] = make_uint4((uint32_t)p4, (uint32_t)(p4 >> 32), (uint32_t)p5, (uint32_t)(p5 >> 32));
            *(odd ? dst : dst + 6) = odd ? w[0] : w[6];
        }
    };
    if (set * WAVE < a.n) {  // a grid rounded up to a multiple of 8 sets has idle blocks
#define BK_ROWS_GROUP(i0, i1, H, ...) rows_class_group<H, __VA_ARGS__>(i0, i1, grp, G, P, emit);
        BK_CLASS_LIST(BK_ROWS_GROUP)
#undef BK_ROWS_GROUP
    }
    if (live && a.out_count && total) atomicAdd(a.out_count + i, total);
}
#else
__global__ void k_movegen_m(MovegenArgs a);
#endif

// Dense rows of the class's table entries i0 <= i < i1 whose orientation lies in this
// block's range (bit i of pm, no table loads), every Wp-th of them from wave w on
// (k_movegen_ml); rr counts the in-range entries of the earlier classes modulo Wp
// (wave-uniform)
template <int H, int... T, typename F>
__device__ __forceinline__ void rows_class_range(int i0, int i1, const uint32_t (&pm)[3], int w, int Wp, int& rr,
                                                 const Planes& P, F&& f) {
#pragma unroll 1
    for (int i = i0; i < i1; ++i) {
        const uint32_t word = i < 32 ? pm[0] : i < 64 ? pm[1] : pm[2];
        if (!((word >> (i & 31)) & 1u)) continue;
        const bool mine = rr == w;
        rr = rr + 1 == Wp ? 0 : rr + 1;
        if (!mine) continue;
        const uint32_t w0 = kClass[i][0], w1 = kClass[i][1];
        uint32_t ok[20];
#pragma unroll
        for (int r = 0; r < 20; ++r) ok[r] = 0u;
        StencilClass<H, T...>::scan(P, w1, [&](int r, uint32_t v) { ok[r] = v; });
        f((int)(w0 >> 8), w0 & 0xFFu, ok);
    }
}

#define MG_PART_WAVES_MAX 8
#if BK_DEF(BK_U_MOVEGEN)
// The block's staged segments (board-player b: words [0, nw) of stage + b * nw) to
// base + b * 637 with 16-byte stores (the width WRITE_SIZE reads exactly): unit u of
// board b covers the 16-byte-aligned word pair 2u - h, 2u - h + 1 of its segment (h = 1
// when the segment starts at an odd word: 637 is odd, so h = (b + hpar) & 1); a pair half
// outside the segment belongs to the neighbouring segment's block.  NWC > 0: nw, known.
template <int NU>
__device__ __forceinline__ void ml_write_segments(const uint64_t* stage, uint64_t* base, int nb, int nw, int hpar) {
    // NU = the most units a segment of this kernel's ranges needs (a compile-time
    // constant, so the unit -> board split is a multiply); units past a shorter
    // segment's end write nothing
#pragma unroll 1
    for (int k = (int)threadIdx.x; k < nb * NU; k += (int)blockDim.x) {
        const int b = k / NU, u = k - b * NU;
        const int w0 = 2 * u - ((b + hpar) & 1);
        const bool lo_in = w0 >= 0 && w0 < nw, hi_in = w0 + 1 < nw;
        const int off = b * (BK_NUM_ORIENTS * 7) + w0;  // words (w0 may be -1: signed)
        uint64_t* dst = base + off;
        const uint64_t* src = stage + b * nw + w0;
        if (lo_in && hi_in) {
            const uint64_t v0 = src[0], v1 = src[1];
            *reinterpret_cast<uint4*>(dst) =
                make_uint4((uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32));
        } else if (lo_in) {
            dst[0] = src[0];
        } else if (hi_in) {
            dst[1] = src[1];
        }
    }
}

template <int PARTS>
__device__ __forceinline__ void movegen_ml_body(const MovegenArgs& a) {
    constexpr int MG_PART_MAX = (BK_NUM_ORIENTS + PARTS - 1) / PARTS;
    __shared__ uint64_t stage[WAVE * MG_PART_MAX * 7];
    const int Wp = (int)(blockDim.x / WAVE);
    const int w = (int)(threadIdx.x / WAVE), lane = (int)(threadIdx.x % WAVE);
    const int xcd = blockIdx.x % MG_XCDS, j = blockIdx.x / MG_XCDS;
    const int set = xcd + MG_XCDS * (j / PARTS), part = j % PARTS;
    if (set * WAVE >= a.n) return;  // a grid rounded up to a multiple of 8 sets: whole idle blocks
    const int glo = part * BK_NUM_ORIENTS / PARTS, ghi = (part + 1) * BK_NUM_ORIENTS / PARTS;
    const int nw = BK_NUM_ORIENTS % PARTS == 0 ? BK_NUM_ORIENTS / PARTS * 7 : (ghi - glo) * 7;
    const int i = set * WAVE + lane;
    const bool live = i < a.n;
    const int idx = live ? i : 0;
    const bk_state* s = a.states + idx;
    const int p = a.players[idx] & 3;
    uint32_t own[20], occ[20];
#pragma unroll
    for (int R = 0; R < 20; ++R) { occ[R] = 0; own[R] = 0; }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int R = 0; R < 20; ++R) {
            const uint32_t row = plane_row(s->planes[q], R);
            occ[R] |= row;
            own[R] |= (q == p) ? row : 0u;
        }
    Planes P;
    derive_rows(own, occ, (s->first_move >> p) & 1u, p, P);
    make_pairs(P);
    const uint32_t avail = live ? (~s->used[p] & 0x1FFFFFu) : 0u;
    uint32_t total = 0;
    uint64_t* mine = stage + lane * nw - glo * 7;
    auto emit = [&](int g, uint32_t piece, const uint32_t (&ok)[20]) {
        const bool av = (avail >> (piece - 1u)) & 1u;
        uint64_t wd[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 20; ++r) {
            const uint32_t v = av ? ok[r] : 0u;
            total += __builtin_popcount(v);
            constexpr int kBits = 20;
            const int off = kBits * r, q = off >> 6, sh = off & 63;  // compile-time per r
            wd[q] |= (uint64_t)v << sh;
            if (sh > 64 - kBits) wd[q + 1] |= (uint64_t)v >> (64 - sh);
        }
#pragma unroll
        for (int q = 0; q < 7; ++q) mine[g * 7 + q] = wd[q];
    };
    int rr = 0;
    const uint32_t pm[3] = {a.part_masks[part][0], a.part_masks[part][1], a.part_masks[part][2]};
#define BK_ROWS_RANGE(i0, i1, H, ...) rows_class_range<H, __VA_ARGS__>(i0, i1, pm, w, Wp, rr, P, emit);
    BK_CLASS_LIST(BK_ROWS_RANGE)
#undef BK_ROWS_RANGE
    if (live && a.out_count && total) atomicAdd(a.out_count + i, total);
    __syncthreads();
    if (a.out_mask) {
        const int nb = a.n - set * WAVE < WAVE ? a.n - set * WAVE : WAVE;
        uint64_t* base = a.out_mask + (size_t)set * WAVE * (BK_NUM_ORIENTS * 7) + glo * 7;
        const int hpar = (glo + (int)(((uintptr_t)a.out_mask >> 3) & 1u)) & 1;
        ml_write_segments<MG_PART_MAX * 7 / 2 + 1>(stage, base, nb, nw, hpar);
    }
}
__global__ __launch_bounds__(MG_PART_WAVES_MAX * WAVE) void k_movegen_ml4(MovegenArgs a) { movegen_ml_body<4>(a); }
__global__ __launch_bounds__(MG_PART_WAVES_MAX * WAVE) void k_movegen_ml5(MovegenArgs a) { movegen_ml_body<5>(a); }
__global__ __launch_bounds__(MG_PART_WAVES_MAX * WAVE) void k_movegen_ml7(MovegenArgs a) { movegen_ml_body<7>(a); }
__global__ __launch_bounds__(MG_PART_WAVES_MAX * WAVE) void k_movegen_ml13(MovegenArgs a) { movegen_ml_body<13>(a); }
#else
__global__ void k_movegen_ml4(MovegenArgs a);
__global__ void k_movegen_ml5(MovegenArgs a);
__global__ void k_movegen_ml7(MovegenArgs a);
__global__ void k_movegen_ml13(MovegenArgs a);
#endif

#if BK_DEF(BK_U_MOVEGEN)
__global__ __launch_bounds__(BLOCK) void k_has_moves(MovegenArgs a) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    const bool live = i < a.n;
    const bk_state* s = a.states + (live ? i : 0);
    uint32_t occ[20];
#pragma unroll
    for (int R = 0; R < 20; ++R) occ[R] = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int R = 0; R < 20; ++R) occ[R] |= plane_row(s->planes[q], R);
    uint8_t mask = 0;
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
        // the mover's rows re-read from the state (L1/L2) each time: a [4][20] register
        // array indexed by the runtime player would be demoted to scratch memory
        uint32_t ow[20];
        Planes P;
#pragma unroll
        for (int R = 0; R < 20; ++R) ow[R] = plane_row(s->planes[p], R);
        derive_rows(ow, occ, (s->first_move >> p) & 1u, p, P);
        make_pairs(P);
        const uint32_t total = movegen_counts<false>(P, live ? (~s->used[p] & 0x1FFFFFu) : 0u, nullptr, lane);
        mask |= (uint8_t)((total > 0) << p);
    }
    if (live) a.out_mask4[i] = mask;
}
#else
__global__ void k_has_moves(MovegenArgs a);
#endif

// ------------------------------------------------------------------------------------
// Frontier sets: CPython 3.10 set of (row, col) tuples, restated for the reference's
// frontier ORDER (engine/board.py:315-367 update_frontier_after_move; Objects/
// setobject.c set_add_entry / set_discard_entry / set_table_resize / set_merge).
// Shared by the device (tables in a per-lane global record) and the host ABI.
// ------------------------------------------------------------------------------------
__constant__ uint64_t kCellHash[BK_CELLS] = BK_CELL_HASH_INIT;
static const uint64_t kCellHashHost[BK_CELLS] = BK_CELL_HASH_INIT;

#define FS_PROBES 9
#define FS_SHIFT 5
#define FS_UNUSED ((int16_t)-1)
#define FS_DUMMY ((int16_t)-2)

struct FsetRef {  // one player's table: runs of 2^sh slots, run j at key[j * stride]
    int16_t* key = nullptr;
    int stride = 2;   // 2: a plain array; 2 * WAVE: slot pairs of one lane interleaved in LDS;
                      // 512 (sh 4): 16-slot runs of a lane pair's LDS-DMA stage (k_mcts_pair)
    uint16_t* mask = nullptr;
    uint16_t* fill = nullptr;
    uint16_t* used = nullptr;
    uint32_t cap = 0; // largest table this storage holds (power of 2)
    const uint64_t* hash = nullptr;  // hash((r, c)) by cell
    int sh = 1;       // log2 of the run length
    uint32_t* dirty = nullptr;  // if set: bit j marks 8-slot chunk j written (all: a resize)
    bool gchunk = false;  // a plain array in global memory: probes read 8-slot chunks (fs_probe)
    __host__ __device__ __forceinline__ int16_t& at(uint32_t i) const {
        return key[(i >> sh) * (uint32_t)stride + (i & ((1u << sh) - 1u))];
    }
    __host__ __device__ __forceinline__ void mark(uint32_t i) const {
        if (dirty) *dirty |= 1u << ((i >> 3) & 31u);
    }
};

__host__ __device__ __forceinline__ FsetRef fs_ref(bk_fset* s, int p, const uint64_t* htab) {
    return FsetRef{s->key[p], 2, &s->mask[p], &s->fill[p], &s->used[p], BK_FSET_SLOTS, htab};
}

// set_insert_clean: first unused slot of the probe sequence.  The linear probes walk
// the slots after i, but the next perturbation step starts from i itself, not from the
// last slot probed (CPython advances `entry`, not `i`; checked against CPython 3.10's
// set.copy() in tests/test_fset_copy.py)
__host__ __device__ inline void fs_insert_clean(FsetRef t, uint32_t mask, int16_t k) {
    const uint64_t h = t.hash[k];
    uint64_t perturb = h;
    uint32_t i = (uint32_t)h & mask, e = i;
    uint32_t left = i + FS_PROBES <= mask ? FS_PROBES : 0u;
    while (t.at(e) != FS_UNUSED) {
        if (left > 0u) {
            --left;
            ++e;
        } else {
            perturb >>= FS_SHIFT;
            i = (i * 5u + 1u + (uint32_t)perturb) & mask;
            e = i;
            left = i + FS_PROBES <= mask ? FS_PROBES : 0u;
        }
    }
    t.at(e) = k;
}

// Occupancy of a table of <= 256 slots in registers: set_insert_clean's probe sequence
// on a fresh table needs only "is slot i unused", so a clean re-insert never reads the
// destination back.
struct SlotBits {
    uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    __host__ __device__ __forceinline__ bool test(uint32_t i) const {
        const uint32_t q = i >> 6;
        const uint64_t w = q == 0u ? w0 : q == 1u ? w1 : q == 2u ? w2 : w3;
        return ((w >> (i & 63u)) & 1ull) != 0ull;
    }
    __host__ __device__ __forceinline__ void set(uint32_t i) {
        const uint64_t b = 1ull << (i & 63u);
        const uint32_t q = i >> 6;
        w0 |= q == 0u ? b : 0ull;
        w1 |= q == 1u ? b : 0ull;
        w2 |= q == 2u ? b : 0ull;
        w3 |= q == 3u ? b : 0ull;
    }
};

// fs_insert_clean's slot for key hash h in a fresh table of mask + 1 slots whose used
// slots are `o` (marks the slot used)
__host__ __device__ __forceinline__ uint32_t fs_clean_slot(uint64_t h, uint32_t mask, SlotBits& o) {
    uint64_t perturb = h;
    uint32_t i = (uint32_t)h & mask, e = i;
    uint32_t left = i + FS_PROBES <= mask ? FS_PROBES : 0u;
#pragma unroll 1
    while (o.test(e)) {  // fs_insert_clean's sequence
        if (left > 0u) {
            --left;
            ++e;
        } else {
            perturb >>= FS_SHIFT;
            i = (i * 5u + 1u + (uint32_t)perturb) & mask;
            e = i;
            left = i + FS_PROBES <= mask ? FS_PROBES : 0u;
        }
    }
    o.set(e);
    return e;
}

// set_table_resize through a small LDS scratch `tmp` (FsetRef layout; the caller checks
// that tmp.cap >= used keys): the active keys, read 16 slots at a time (the reads
// issued together), go to tmp in slot order; the table is cleared and they are
// re-inserted with their slots from a register occupancy bitmap (fs_clean_slot:
// set_insert_clean's probe sequence), 8 keys and their cell hashes loaded at a time.  A
// resize that stays within the storage has used * 4 < newsize <= cap, so tmp never holds
// more than cap / 4 keys.  The table itself may be staged in LDS or in global memory (a
// table too large for the stage: its slots are read 16 at a time as well).  Equal to
// fs_resize slot for slot (tests/test_fset_copy.py
// through bk_debug_fset_op).  fs_resize instead copies every slot to the record's tmp in
// global memory and re-inserts one dependent memory latency at a time: resizes were ~86 %
// of k_rollout_fr's set-operation time and ~90 % of k_mcts_pair's
// (profiles/r05/sweeps/r05n, -DBK_SECTION_PROF).
__host__ __device__ inline bool fs_resize_lds(FsetRef t, FsetRef tmp, uint32_t minused) {
    uint32_t newsize = 8;
    while (newsize <= minused) newsize <<= 1;
    if (newsize > t.cap) return false;
    const uint32_t omask = *t.mask;
    uint32_t n = 0;
    for (uint32_t b = 0; b <= omask; b += 16) {
        uint32_t w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            w[j] = b + 2u * (uint32_t)j <= omask ? *reinterpret_cast<const bk_u32_alias*>(&t.at(b + 2u * (uint32_t)j))
                                                 : 0xFFFFFFFFu;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int16_t k = (int16_t)(w[q >> 1] >> (16 * (q & 1)));
            if (k >= 0) tmp.at(n++) = k;
        }
    }
    for (uint32_t j = 0; j < newsize; j += 2) *reinterpret_cast<bk_u32_alias*>(&t.at(j)) = 0xFFFFFFFFu;
    *t.mask = (uint16_t)(newsize - 1u);
    *t.fill = *t.used;
    SlotBits o;
    for (uint32_t b = 0; b < n; b += 8) {
        int16_t k[8];
        uint64_t h[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) k[q] = b + (uint32_t)q < n ? tmp.at(b + (uint32_t)q) : (int16_t)-1;
#pragma unroll
        for (int q = 0; q < 8; ++q) h[q] = k[q] >= 0 ? t.hash[k[q]] : 0ull;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (k[q] >= 0) t.at(fs_clean_slot(h[q], newsize - 1u, o)) = k[q];
    }
    return true;
}

// set_table_resize(minused): fresh table, active entries re-inserted in slot order.
// tmp (stride 1) holds the old keys.  false: the storage cannot hold the new table.
__host__ __device__ inline bool fs_resize(FsetRef t, int16_t* tmp, uint32_t minused) {
    uint32_t newsize = 8;
    while (newsize <= minused) newsize <<= 1;
    if (newsize > t.cap) return false;
    const uint32_t omask = *t.mask;
    for (uint32_t i = 0; i <= omask; ++i) tmp[i] = t.at(i);
    for (uint32_t i = 0; i < newsize; ++i) t.at(i) = FS_UNUSED;
    *t.mask = (uint16_t)(newsize - 1);
    *t.fill = *t.used;
    for (uint32_t i = 0; i <= omask; ++i)
        if (tmp[i] >= 0) fs_insert_clean(t, newsize - 1, tmp[i]);
    return true;
}

// One probe routine for both set operations, so kernels carry a single copy of the
// probe loop (set_lookkey / set_add_entry / set_discard_entry, Objects/setobject.c):
// * add: an existing key is a no-op; a new key takes the LAST dummy seen on its probe
//   chain, else the unused slot that ended the search (then maybe resize);
// * discard: the key's slot becomes a dummy (absent key: no-op).
// false: the table outgrew its storage (add only).  ltmp.key set: an LDS-staged table,
// resized through the LDS scratch ltmp (fs_resize_lds); else through tmp (fs_resize).
// The probe sequence of key k (hash h) in table t: the slot e where the search stops (k
// found, or the first unused slot) with its value kk, and the last dummy seen before it
// (freeslot, -1 if none).  From i = hash & mask the 10 slots i .. i + 9 when they fit
// below mask (LINEAR_PROBES 9), else slot i alone, then i = (5 i + 1 + perturb) & mask
// with perturb >>= 5.  Slot indices stay 32-bit: only the low bits of 5 i + 1 + perturb
// survive the mask.  One slot per step, as one flat loop (a divergent nested loop costs
// the wave far more exec-mask bookkeeping than its VALU work).  Reading two or four slots
// per step from the pair-stored tables measured slower (frontier-order config 3 34.1 ->
// 33.2 / 33.0 M playouts/s, config 5 17.6 -> 17.1 / 17.0 M; profiles/r05/sweeps/r05f):
// most chains end at their first or second slot.
// t.gchunk (a table probed in global memory, k_rollout_fr's 128-slot tables): the probe
// reads the 16-byte chunk holding slot e (8 slots, one memory latency) and walks the
// linear run from registers, loading the next chunk only when the sequence leaves it.
__host__ __device__ inline void fs_probe(FsetRef t, int16_t k, uint64_t h, uint32_t mask, uint32_t& e_out,
                                         int16_t& kk_out, int32_t& freeslot) {
    uint64_t perturb = h;
    uint32_t i = (uint32_t)h & mask, e = i;
    uint32_t left = i + FS_PROBES <= mask ? FS_PROBES : 0u;
    freeslot = -1;
    int16_t kk;
    if (t.gchunk) {
        const bk_u4_alias* k4 = reinterpret_cast<const bk_u4_alias*>(t.key);
        uint32_t cb = e >> 3;
        uint4 c = k4[cb];
        for (;;) {
            if ((e >> 3) != cb) {
                cb = e >> 3;
                c = k4[cb];
            }
            const uint32_t q = (e >> 1) & 3u;
            const uint32_t w = q == 0u ? c.x : q == 1u ? c.y : q == 2u ? c.z : c.w;
            kk = (int16_t)(w >> (16u * (e & 1u)));
            if (kk == FS_UNUSED || kk == k) break;
            if (kk == FS_DUMMY) freeslot = (int32_t)e;
            if (left > 0u) {
                --left;
                ++e;
            } else {
                perturb >>= FS_SHIFT;
                i = (i * 5u + 1u + (uint32_t)perturb) & mask;
                e = i;
                left = i + FS_PROBES <= mask ? FS_PROBES : 0u;
            }
        }
        e_out = e;
        kk_out = kk;
        return;
    }
    for (;;) {
        kk = t.at(e);
        if (kk == FS_UNUSED || kk == k) break;
        if (kk == FS_DUMMY) freeslot = (int32_t)e;
        if (left > 0u) {
            --left;
            ++e;
        } else {
            perturb >>= FS_SHIFT;
            i = (i * 5u + 1u + (uint32_t)perturb) & mask;
            e = i;
            left = i + FS_PROBES <= mask ? FS_PROBES : 0u;
        }
    }
    e_out = e;
    kk_out = kk;
}

// the set operation without its resize: true when the add filled the table to the resize
// threshold (the caller then runs fs_resize_any before the next operation)
__host__ __device__ inline bool fs_op_nr(FsetRef t, int16_t k, bool add, uint64_t h) {
    const uint32_t mask = *t.mask;
    uint32_t e;
    int16_t kk;
    int32_t freeslot;
    fs_probe(t, k, h, mask, e, kk, freeslot);
    if (kk == k) {  // present: discard leaves a dummy, add is a no-op
        if (!add) {
            t.at(e) = FS_DUMMY;
            t.mark(e);
            *t.used -= 1;
        }
        return false;
    }
    if (!add) return false;
    if (freeslot >= 0) {
        *t.used += 1;
        t.at((uint32_t)freeslot) = k;
        t.mark((uint32_t)freeslot);
        return false;
    }
    *t.fill += 1;
    *t.used += 1;
    t.at(e) = k;
    t.mark(e);
    return (uint64_t)*t.fill * 5 >= (uint64_t)mask * 3;
}

// set_table_resize after an add reached the threshold (set_add_entry's resize call)
__host__ __device__ inline bool fs_resize_any(FsetRef t, int16_t* tmp, FsetRef ltmp) {
    if (t.dirty) *t.dirty = ~0u;  // every slot is rewritten
    const uint32_t minused = *t.used > 50000 ? *t.used * 2u : *t.used * 4u;
#if defined(BK_SECTION_PROF) && defined(__HIP_DEVICE_COMPILE__)
    // diagnostic (section slot 15): wave cycles in resizes, counted by the first lane of
    // each resize branch
    const uint64_t rt0 = clock64();
    const bool rok = ltmp.key && *t.used <= ltmp.cap ? fs_resize_lds(t, ltmp, minused) : fs_resize(t, tmp, minused);
    const uint64_t rex = __builtin_amdgcn_read_exec();
    if ((uint32_t)__lane_id() == (uint32_t)__builtin_ctzll(rex)) atomicAdd(&g_sections[15], clock64() - rt0);
    return rok;
#else
    return ltmp.key && *t.used <= ltmp.cap ? fs_resize_lds(t, ltmp, minused) : fs_resize(t, tmp, minused);
#endif
}

__host__ __device__ inline bool fs_op_h(FsetRef t, int16_t* tmp, int16_t k, bool add, uint64_t h,
                                       FsetRef ltmp = FsetRef{}) {
    return !fs_op_nr(t, k, add, h) || fs_resize_any(t, tmp, ltmp);
}

__host__ __device__ inline bool fs_op(FsetRef t, int16_t* tmp, int16_t k, bool add) {
    return fs_op_h(t, tmp, k, add, t.hash[k]);
}
__host__ __device__ inline bool fs_add(FsetRef t, int16_t* tmp, int16_t k) { return fs_op(t, tmp, k, true); }
__host__ __device__ inline void fs_discard(FsetRef t, int16_t k) { fs_op(t, nullptr, k, false); }

// an empty table of 8 slots (set_clear / make_new_set).  Slots beyond mask are never
// read (every walk stops at mask; growing a table clears its new slots first)
__host__ __device__ inline void fs_clear(FsetRef t) {
    for (uint32_t i = 0; i < 8; ++i) t.at(i) = FS_UNUSED;
    *t.mask = 7;
    *t.fill = 0;
    *t.used = 0;
}

// update_frontier_after_move for player p, engine/board.py:315-367.  occ(r, c) / own(r, c)
// read the board AFTER all the piece's cells were written.  false: table overflow.
// addable(nr, nc): the in-bounds diagonal neighbour is empty and not orthogonally
// adjacent to the mover (both on the board after the move).  The op sequence (discard
// the cell, add its diagonals, discard its orthogonals, cell by cell) is the reference's.
template <typename Add>
__host__ __device__ inline bool fs_place_pred(FsetRef t, int16_t* tmp, const int32_t* cells, int n, Add addable) {
    // fully unrolled (static cell / op indices): measured faster on gfx950 than a
    // compact runtime op loop, whose divergent-loop bookkeeping costs more than the
    // larger code (the I-cache miss rate stays ~0.1 %, profiles/r01_pmc_frontier)
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        if (i >= n) break;
        const int r = cells[i] / 20, c = cells[i] % 20;
#pragma unroll
        for (int o = 0; o < 9; ++o) {
            // o = 0: the cell; 1..4: diagonals (-1,-1) (-1,1) (1,-1) (1,1), added when
            // addable; 5..8: orthogonals (-1,0) (1,0) (0,-1) (0,1), discarded
            const bool add = o >= 1 && o <= 4;
            const int nr = r + (o == 1 || o == 2 || o == 5 ? -1 : o == 3 || o == 4 || o == 6 ? 1 : 0);
            const int nc = c + (o == 1 || o == 3 || o == 7 ? -1 : o == 2 || o == 4 || o == 8 ? 1 : 0);
            if (nr < 0 || nr >= 20 || nc < 0 || nc >= 20) continue;
            if (add && !addable(nr, nc)) continue;
            if (!fs_op(t, tmp, (int16_t)(nr * 20 + nc), add)) return false;
        }
    }
    return true;
}

template <typename Occ, typename Own>
__host__ __device__ inline bool fs_place(FsetRef t, int16_t* tmp, const int32_t* cells, int n, Occ occ, Own own) {
    auto addable = [&](int nr, int nc) {
        if (occ(nr, nc)) return false;
        if (nr > 0 && own(nr - 1, nc)) return false;
        if (nr < 19 && own(nr + 1, nc)) return false;
        if (nc > 0 && own(nr, nc - 1)) return false;
        if (nc < 19 && own(nr, nc + 1)) return false;
        return true;
    };
    return fs_place_pred(t, tmp, cells, n, addable);
}

// set.copy() (make_new_set + set_merge into an empty set).  false: the copy's table
// would not fit the storage (d left empty)
__host__ __device__ inline bool fs_copy(FsetRef d, const int16_t* skey, uint32_t smask, uint32_t sfill,
                                        uint32_t sused) {
    fs_clear(d);
    if (sused == 0) return true;
    if (sused * 5 >= 7u * 3u) {  // (fill + other->used) * 5 >= mask * 3 on the fresh table
        uint32_t newsize = 8;
        while (newsize <= sused * 2) newsize <<= 1;
        if (newsize > d.cap) return false;
        for (uint32_t i = 8; i < newsize; ++i) d.at(i) = FS_UNUSED;
        *d.mask = (uint16_t)(newsize - 1);
    }
    if (*d.mask == smask && sfill == sused) {
        for (uint32_t i = 0; i <= smask; ++i) d.at(i) = skey[i];
        *d.fill = (uint16_t)sfill;
        *d.used = (uint16_t)sused;
        return true;
    }
    *d.fill = (uint16_t)sused;
    *d.used = (uint16_t)sused;
    for (uint32_t i = 0; i <= smask; ++i)
        if (skey[i] >= 0) fs_insert_clean(d, *d.mask, skey[i]);
    return true;
}

// Run the ops marked in `real` (frontier_ops) on table t, in order: one probe routine in
// a per-lane loop, so a wave runs as many probe chains as its busiest lane has real ops
// (typically ~10) instead of all 45.  false: table overflow.
// BATCH false: every lane of the wave runs the same table (the cooperative kernels), so
// resizes run inline
template <bool BATCH = true>
__device__ __forceinline__ bool fs_run_ops(FsetRef t, int16_t* tmp, const int32_t (&cells)[5], uint64_t real,
                                           FsetRef ltmp = FsetRef{}) {
    // key offset + 21 of op o, 6 bits each: 0, -21, -19, 19, 21, -20, 20, -1, 1
    constexpr uint64_t KD = (21ull << 0) | (0ull << 6) | (2ull << 12) | (40ull << 18) | (42ull << 24) |
                            (1ull << 30) | (41ull << 36) | (20ull << 42) | (22ull << 48);
    auto key_of = [&](int s) {
        const int q = (s * 57) >> 9;  // s / 9 for s < 45
        const int op = s - 9 * q;
        const int cell = q == 0 ? cells[0] : q == 1 ? cells[1] : q == 2 ? cells[2] : q == 3 ? cells[3] : cells[4];
        return cell + (int)((KD >> (6 * op)) & 63ull) - 21;
    };
    if constexpr (!BATCH) {
#pragma unroll 1
        while (real) {
            const int s = (int)__builtin_ctzll(real);
            real &= real - 1ull;
            const int op = s - 9 * ((s * 57) >> 9);
            const int key = key_of(s);
            // (a wave-parallel version -- op hashes loaded up front, one lane per slot of
            // the first linear probe run, ballot for the stop -- measured 3 % slower:
            // most chains stop at their first slot; profiles/r06/sweeps/r06w)
            if (!fs_op_h(t, tmp, (int16_t)key, (unsigned)(op - 1) < 4u, t.hash[key], ltmp)) return false;
        }
        return true;
    }
    // A lane whose add reaches the resize threshold leaves the op loop; once every lane of
    // the wave has finished or stopped there, the resizes run together (one pass of the
    // resize code per round instead of one per op iteration that has a resizing lane:
    // ~6 lanes of a wave resize a table per frontier-order ply), then the ops go on.
    bool ok = true;
#pragma unroll 1
    for (;;) {
        bool need = false;
#pragma unroll 1
        while (real && !need) {
            const int s = (int)__builtin_ctzll(real);
            real &= real - 1ull;
            const int op = s - 9 * ((s * 57) >> 9);
            const int key = key_of(s);
            // (loading the next ops' hashes ahead, 3 or 6 in flight, measured slower:
            // 34.2 -> 33.6 M frontier-order playouts/s, profiles/r05/sweeps/r05g)
            const uint64_t h = t.hash[key];
            need = fs_op_nr(t, (int16_t)key, (unsigned)(op - 1) < 4u, h);
        }
        if (need && !fs_resize_any(t, tmp, ltmp)) {
            ok = false;  // the table outgrew this storage: the caller starts over elsewhere
            real = 0;
        }
        if (__builtin_amdgcn_ballot_w64(real != 0ull) == 0ull) break;
    }
    return ok;
}

// the LDS scratch of fs_resize_lds: this lane's [slot pair][lane] column from ltk, room
// for `keys` keys (none: nullptr)
__device__ __forceinline__ FsetRef lds_tmp(int16_t* ltk, uint32_t keys) {
    FsetRef r{};
    if (ltk) {
        r.key = ltk;
        r.stride = 2 * WAVE;
        r.cap = keys;
    }
    return r;
}

// per-lane frontier record in the rollout kernel: the tables plus resize scratch.
// padded to whole 128-byte lines, so each player's table starts on a line and a table of
// <= 64 slots is ONE line (2,592 -> 2,688 bytes; see the slab's padding)
struct FsLane {
    bk_fset s;
    int16_t tmp[BK_FSET_SLOTS];
    int16_t pad[48];  // 2592 -> 2688 bytes
};

// update_frontier_after_move (engine/board.py:315-367) of player p's table in fl for a
// piece at cells[0..n): the ops marked in `real` (frontier_ops).  A table of < STAGE
// slots is staged in LDS so the probe chains wait on LDS, not L2/HBM: lk = this lane's dword of [slot pair][lane] (slots 2j, 2j + 1 in dword j *
// WAVE): one ds_write_b32 / ds_read_b32 per slot pair, and a probe of ANY slot by each
// lane hits bank `lane` (conflict-free).  A larger table (or a move that grows one past
// the stage) is updated in place.  false: table overflow.
// fs_copy_dev's size rule: the copy of a table with `used` active keys has newsize
// slots; the copy is slot-for-slot the source when the size is unchanged and the source
// has no dummies (set_merge's same-size path)
__device__ __forceinline__ uint32_t fs_copy_size(uint32_t used) {
    uint32_t newsize = 8;
    if (used * 5 >= 7u * 3u)
        while (newsize <= used * 2) newsize <<= 1;
    return newsize;
}

// Board.copy() of table q of fl in place (the copy replaces the table): the source keys
// go to fl->tmp, the destination is cleared and the keys re-inserted in slot order with
// their slots chosen from a register bitmap.  Equal to fs_copy_dev into another record.
// false: the copy would not fit the storage (table left empty, as fs_copy_dev).
__device__ __forceinline__ bool fs_recopy_global(FsLane* fl, int q, const uint64_t* htab) {
    bk_fset* s = &fl->s;
    const uint32_t smask = s->mask[q], sfill = s->fill[q], sused = s->used[q];
    const uint32_t newsize = fs_copy_size(sused);
    if (newsize - 1 == smask && sfill == sused) return true;  // a copy of a copy
    if (newsize > BK_FSET_SLOTS) {
        fs_clear(fs_ref(s, q, htab));
        return false;
    }
    bk_u4_alias* k4 = reinterpret_cast<bk_u4_alias*>(s->key[q]);
    bk_u4_alias* t4 = reinterpret_cast<bk_u4_alias*>(fl->tmp);
#pragma unroll 1
    for (uint32_t i = 0; i <= smask / 8; ++i) t4[i] = k4[i];
    const uint4 unused = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
#pragma unroll 1
    for (uint32_t i = 0; i < newsize / 8; ++i) k4[i] = unused;
    s->mask[q] = (uint16_t)(newsize - 1);
    s->fill[q] = (uint16_t)sused;
    s->used[q] = (uint16_t)sused;
    SlotBits o;
#pragma unroll 1
    for (uint32_t i = 0; i <= smask / 8; ++i) {
        const uint4 v = t4[i];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int16_t k = (int16_t)((j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFFu));
            if (k >= 0) s->key[q][fs_clean_slot(htab[k], newsize - 1, o)] = k;
        }
    }
    return true;
}

// RECOPY: the table after the ops is replaced by its Board.copy() (MCTSNode boards are
// copies of copies, mcts_agent.py:113-145): from the LDS stage, the keys are re-inserted
// straight into the global table (slots from a register bitmap), so the copy costs no
// second record and no reads of global memory.
struct NoMark {
    __device__ __forceinline__ void operator()(int) const {}
};

// mark(i): section boundaries for the diagnostic build (-DBK_SECTION_PROF)
// hdr: player p's (mask, fill, used) when kept outside the record (the rollout slab);
// nullptr: the record's own header
// ltk: an LDS column for fs_resize_lds's scratch (STAGE / 4 keys, [slot pair][lane]), or
// nullptr (resizes go through the record's global tmp)
template <int STAGE, bool RECOPY = false, typename Mark = NoMark>
__device__ __forceinline__ bool place_frontier(FsLane* fl, int p, int16_t* lk, const uint64_t* htab,
                                               const int32_t (&cells)[5], uint64_t real, Mark mark = Mark(),
                                               uint16_t* hdr = nullptr, int16_t* ltk = nullptr) {
    bk_fset* gfs = &fl->s;
    uint16_t* const hm = hdr ? hdr : &gfs->mask[p];
    uint16_t* const hf = hdr ? hdr + 1 : &gfs->fill[p];
    uint16_t* const hu = hdr ? hdr + 2 : &gfs->used[p];
    // stages of <= STAGE_EAGER_MAX slots load all STAGE slots at once, alongside the
    // mask (the storage holds BK_FSET_SLOTS >= STAGE): one memory latency instead of the
    // mask's, then the table's
    constexpr bool EAGER = STAGE > 0 && STAGE <= STAGE_EAGER_MAX;
    const bk_u4_alias* src4 = reinterpret_cast<const bk_u4_alias*>(gfs->key[p]);
    uint4 pre[EAGER ? STAGE / 8 : 1];
    if constexpr (EAGER) {
#pragma unroll
        for (int i = 0; i < STAGE / 8; ++i) pre[i] = src4[i];
    }
    const uint32_t gmask = *hm;
    bk_u32_alias* lw = reinterpret_cast<bk_u32_alias*>(lk);
    if (STAGE > 0 && gmask < (uint32_t)STAGE) {
#pragma unroll
        for (int i = 0; i < STAGE / 8; ++i) {
            if ((uint32_t)(8 * i) <= gmask) {
                const uint4 v = EAGER ? pre[EAGER ? i : 0] : src4[i];
                lw[(4 * i + 0) * WAVE] = v.x;
                lw[(4 * i + 1) * WAVE] = v.y;
                lw[(4 * i + 2) * WAVE] = v.z;
                lw[(4 * i + 3) * WAVE] = v.w;
            }
        }
        const uint16_t m0 = (uint16_t)gmask, f0 = *hf, u0 = *hu;
        uint16_t m = m0, f = f0, u = u0;
        uint32_t dirty = 0;  // 8-slot chunks the ops wrote: only those go back to the table
        FsetRef t{lk, 2 * WAVE, &m, &f, &u, (uint32_t)STAGE, htab, 1, &dirty};
        mark(8);
        const bool ran = fs_run_ops(t, fl->tmp, cells, real, lds_tmp(ltk, STAGE / 4));
        mark(9);
        if (ran) {
            bk_u4_alias* dst4 = reinterpret_cast<bk_u4_alias*>(gfs->key[p]);
            const uint32_t newsize = fs_copy_size(u);
            if (!RECOPY || (newsize - 1 == m && f == u)) {  // (a copy of a clean table is the table)
#pragma unroll
                for (int i = 0; i < STAGE / 8; ++i) {
                    if ((uint32_t)(8 * i) <= m && ((dirty >> i) & 1u))
                        dst4[i] = make_uint4(lw[(4 * i + 0) * WAVE], lw[(4 * i + 1) * WAVE],
                                             lw[(4 * i + 2) * WAVE], lw[(4 * i + 3) * WAVE]);
                }
                if (m != m0) *hm = m;
                if (f != f0) *hf = f;
                if (u != u0) *hu = u;
                return true;
            }
            // the copy: newsize <= 2 * STAGE <= BK_FSET_SLOTS (u < STAGE * 3 / 5)
            const uint4 unused = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
#pragma unroll 1
            for (uint32_t i = 0; i < newsize / 8; ++i) dst4[i] = unused;
            *hm = (uint16_t)(newsize - 1); *hf = u; *hu = u;
            SlotBits o;
            int16_t* dk = gfs->key[p];
#pragma unroll 1
            for (uint32_t j = 0; j <= m / 2; ++j) {
                const uint32_t w = lw[j * WAVE];
                const int16_t k0 = (int16_t)(w & 0xFFFFu), k1 = (int16_t)(w >> 16);
                if (k0 >= 0) dk[fs_clean_slot(htab[k0], newsize - 1, o)] = k0;
                if (k1 >= 0) dk[fs_clean_slot(htab[k1], newsize - 1, o)] = k1;
            }
            return true;
        }
    }
    // (a table too large for the stage: its resizes use the lane's whole column of the
    // area, STAGE keys, as their scratch -- the stage is not in use)
    FsetRef gt{gfs->key[p], 2, hm, hf, hu, BK_FSET_SLOTS, htab};
    gt.gchunk = ltk != nullptr;  // (the playout kernels: k_rollout_fr)
    if (!fs_run_ops(gt, fl->tmp, cells, real, lds_tmp(ltk ? lk : nullptr, (uint32_t)STAGE))) return false;
    if constexpr (RECOPY) return fs_recopy_global(fl, p, htab);  // (MCTS records: hdr is nullptr)
    return true;
}

// k_mcts_pair's LDS-DMA stage of the mover's table: the lane pair (2q, 2q + 1) loads run
// k (slots 16k .. 16k + 15, 32 bytes) of pair q's table with one global_load_lds_dwordx4
// per lane, so run k of pair q sits at dwords DMA_BASE + 256 k + 8 q of the wave's area.
#define DMA_RUNS 8                       // tables of <= 128 slots are staged
#define DMA_RUN_DWORDS (WAVE * 4)        // one wave-instruction: 64 lanes x 16 bytes
#define DMA_RUN_I16 (2 * DMA_RUN_DWORDS)

// place_frontier on the DMA stage (stage_q = pair q's slot 0; mask / fill / used as
// loaded): the ops in LDS, then the table (or, RECOPY, its copy) written to fl.  Falls
// back to the global table when the ops outgrow the stage.
// RUN_U4: uint4 distance between 16-slot runs (k_mcts_pair's pair stage: 64; the
// cooperative kernels' one-per-wave stage, a plain array: 2)
// inplace: stage_q IS the record's table (k_mcts_coop_h's McLane in LDS): the ops run on
// it directly with its full storage, and nothing is written back
template <bool RECOPY, int RUN_U4 = DMA_RUN_DWORDS / 4, typename Mark = NoMark>
__device__ __forceinline__ bool place_frontier_dma(FsLane* fl, int p, int16_t* stage_q, const uint64_t* htab,
                                                   const int32_t (&cells)[5], uint64_t real, Mark mark = Mark(),
                                                   int16_t* ltk = nullptr, bool inplace = false) {
    bk_fset* gfs = &fl->s;
    const uint16_t m0 = gfs->mask[p], f0 = gfs->fill[p], u0 = gfs->used[p];
    uint16_t m = m0, f = f0, u = u0;
    uint32_t dirty = 0;  // 8-slot chunks the ops wrote: only those go back to the table
    FsetRef t{stage_q, 8 * RUN_U4, &m, &f, &u, inplace ? (uint32_t)BK_FSET_SLOTS : 16u * DMA_RUNS, htab, 4, &dirty};
    constexpr bool BATCH = RUN_U4 != 2;  // (RUN_U4 2: the cooperative kernels' one stage per wave)
    const bool ran = fs_run_ops<BATCH>(t, fl->tmp, cells, real, lds_tmp(ltk, 32u));
    mark(5);
    if (ran) {
        bk_u4_alias* dst4 = reinterpret_cast<bk_u4_alias*>(gfs->key[p]);
        const bk_u4_alias* src4 = reinterpret_cast<const bk_u4_alias*>(stage_q);
        const uint32_t newsize = fs_copy_size(u);
        if (!RECOPY || (newsize - 1 == m && f == u)) {  // (a copy of a clean table is the table)
            if (!inplace) {
#pragma unroll
                for (int r = 0; r < DMA_RUNS; ++r) {
                    if ((uint32_t)(16 * r) <= m) {
                        if ((dirty >> (2 * r)) & 1u) dst4[2 * r] = src4[r * RUN_U4];
                        if ((dirty >> (2 * r + 1)) & 1u) dst4[2 * r + 1] = src4[r * RUN_U4 + 1];
                    }
                }
            }
            if (m != m0) gfs->mask[p] = m;
            if (f != f0) gfs->fill[p] = f;
            if (u != u0) gfs->used[p] = u;
            return true;
        }
        // (never in place: the copy reads the stage while it rewrites the table)
        const uint4 unused = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
#pragma unroll 1
        for (uint32_t i = 0; i < newsize / 8; ++i) dst4[i] = unused;
        gfs->mask[p] = (uint16_t)(newsize - 1); gfs->fill[p] = u; gfs->used[p] = u;
        SlotBits o;
        int16_t* dk = gfs->key[p];
#pragma unroll 1
        for (uint32_t i = 0; i <= m; i += 8) {
            const uint4 v = src4[(i >> 4) * RUN_U4 + ((i >> 3) & 1u)];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int16_t k = (int16_t)((j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFFu));
                if (k >= 0) dk[fs_clean_slot(htab[k], newsize - 1, o)] = k;
            }
        }
        return true;
    }
    if (inplace) return false;  // (the ops ran on the table: past its 256 slots)
    if (!fs_run_ops<BATCH>(fs_ref(gfs, p, htab), fl->tmp, cells, real, lds_tmp(ltk, 80u))) return false;
    return RECOPY ? fs_recopy_global(fl, p, htab) : true;
}

// ------------------------------------------------------------------------------------
// HeuristicAgent policy (agents/heuristic_agent.py:39-244) on the device.
//
// Score of a legal move (_evaluate_move :68-103): size + 2 * corners - 1.5 * edge' +
// 0.5 * centre, with corners = sum over the piece's cells of the in-bounds diagonal
// neighbours that are empty and not orthogonally adjacent to the mover (board BEFORE the
// move; a neighbour reached from two cells counts twice, :107-138), edge' = cells with
// min(r, c, 19 - r, 19 - c) <= 2, halved once move_count / 100.0 >= 0.3 (:140-176), and
// centre = 1 - |anchor - (9.5, 9.5)| / sqrt(2 * 9.5^2) (:178-199).  4 * score =
// K4 + 2 * centre with the integer K4 = 4 n + 8 corners - w edge (w = 6 early, 3 late).
// The move is rng.choice(n, p=softmax(scores)) (:61-65, :223-244): one random_sample()
// u (genrand_res53 of the agent's numpy MT19937) and the first list index whose
// cumulative probability exceeds u.
//
// Exactness.  numpy's exp is not reproducible across hosts (AVX-512 SIMD vs libm), so
// the probabilities are not recomputed bit for bit; the CHOICE is.  Here e = exp(score)
// = TK[K4] * TC[anchor] (exp(K4 / 4) and exp(centre / 2), tables per block) and the
// cumulative sums run in double: every computed cumulative probability is within
// ~1e-13 of the exact value, and so is the reference's.  The kernel takes the first move
// whose cumulative e exceeds u * total and verifies that u * total lies more than
// HEUR_MARGIN * total inside that move's interval; then the reference (any host) picks
// the same index.  A draw closer than that to an interval end (probability ~1e-9 per draw
// with ~500 moves) sets status bit 4: the choice is then still the exact-arithmetic one,
// but the reference's rounding could pick a neighbour.  Informational: nothing stops.
// ------------------------------------------------------------------------------------
#define HK_MIN (-10)  // K4 range: 4 n + 8 corners - 6 edge in [-10, 180]
#define HK_N 191
#define HEUR_MARGIN 9.094947017729282e-13  // 2^-40 of the total (error bound ~1e-13)
#define BK_STATUS_UNCERT 16u

struct HeurShared {           // per block (LDS), built at kernel start
    double tk[HK_N];          // exp(K4 / 4)
    double tc[BK_CELLS];      // exp(centre(anchor) / 2)
    int32_t first[BK_PIECES + 1];  // first global orientation of each piece (+ 91)
};

__device__ void heur_shared_init(HeurShared* hs, int tid, int nthreads) {
    for (int i = tid; i < HK_N; i += nthreads) hs->tk[i] = exp(0.25 * (double)(i + HK_MIN));
    for (int a = tid; a < BK_CELLS; a += nthreads) {
        const double dr = (double)(a / 20) - 9.5, dc = (double)(a % 20) - 9.5;
        const double centre = 1.0 - sqrt(dr * dr + dc * dc) / sqrt(2.0 * (9.5 * 9.5));
        hs->tc[a] = exp(0.5 * centre);
    }
    for (int g = tid; g < BK_NUM_ORIENTS; g += nthreads) {
        const uint32_t pc = kInfo[g] & 0xFFu;
        if (g == 0 || (kInfo[g - 1] & 0xFFu) != pc) hs->first[pc - 1] = g;
    }
    if (tid == 0) hs->first[BK_PIECES] = BK_NUM_ORIENTS;
}

// e = exp(score) of orientation (n cells at (cd, cc)) with its box corner at (r, x);
// rows[R * WAVE].x = the mover's blocked row R before the move (empty and not
// orthogonally adjacent to the mover = ~B)
__device__ __forceinline__ double heur_e(int n, const uint32_t (&cd)[5], const uint32_t (&cc)[5], int r, int x,
                                         const uint2* rows, const HeurShared* hs, int edge_w) {
    int corners = 0, edge = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        if (k < n) {
            const int R = r + (int)cd[k], c = x + (int)cc[k];
            const uint32_t up = R > 0 ? (~rows[(R - 1) * WAVE].x & ROWMASK) : 0u;
            const uint32_t dn = R < 19 ? (~rows[(R + 1) * WAVE].x & ROWMASK) : 0u;
            // bits c - 1 and c + 1 of the rows above (bits 0, 2) and below (bits 1, 3)
            corners += __builtin_popcount((((up << 1) >> c) & 5u) | ((((dn << 1) >> c) & 5u) << 1));
            edge += (R <= 2 || R >= 17 || c <= 2 || c >= 17) ? 1 : 0;
        }
    }
    return hs->tk[4 * n + 8 * corners - edge_w * edge - HK_MIN] * hs->tc[r * 20 + x];
}

__device__ __forceinline__ void orient_cells(int g, int& n, uint32_t (&cd)[5], uint32_t (&cc)[5]) {
    n = (int)((kInfo[g] >> 8) & 0xFFu);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t cell = kCells[g][k];
        cd[k] = cell >> 8;
        cc[k] = cell & 0xFFu;
    }
}

// sum of e over orientation g's legal anchors (ok rows in rows[r * WAVE].y, r < nr);
// g is wave-uniform (a stencil-class entry)
__device__ __forceinline__ double heur_orient_sum(int g, int nr, const uint2* rows, const HeurShared* hs, int edge_w,
                                                  uint32_t& count) {
    int n;
    uint32_t cd[5], cc[5];
    orient_cells(g, n, cd, cc);
    double sum = 0.0;
    // rows holding legal anchors, then ONE per-lane loop over this lane's moves (row-major,
    // columns ascending: the summation order of a per-row loop).  The wave iterates max
    // over lanes of the orientation's move count, not the sum over rows of the per-row
    // maxima (most rows of most lanes are empty).
    uint32_t rm = 0;
#pragma unroll 1
    for (int r = 0; r < nr; ++r) {
        const uint32_t ok = rows[r * WAVE].y;
        count += __builtin_popcount(ok);
        rm |= (ok != 0u ? 1u : 0u) << r;
    }
    int r = 0;
    uint32_t ok = 0;
    while (ok | rm) {
        if (ok == 0u) {
            r = __builtin_ctz(rm);
            rm &= rm - 1u;
            ok = rows[r * WAVE].y;
        }
        const int x = __builtin_ctz(ok);
        ok &= ok - 1u;
        sum += heur_e(n, cd, cc, r, x, rows, hs, edge_w);
    }
    return sum;
}

// pass A over one stencil class: e sums per piece (psum[(piece - 1) * WAVE], doubles in
// LDS) and the legal-move count, for lanes whose mover plays the heuristic (avail = 0
// otherwise)
template <int H, int... T>
__device__ __forceinline__ void heur_class(int i0, int i1, const Planes& P, uint32_t avail, uint2* rows,
                                           double* psum, const HeurShared* hs, int edge_w, uint32_t& count) {
#pragma unroll 1
    for (int i = i0; i < i1; ++i) {
        const uint32_t w0 = kClass[i][0], w1 = kClass[i][1];
        const uint32_t piece = w0 & 0xFFu;
        const bool av = (avail >> (piece - 1u)) & 1u;
        if (__builtin_amdgcn_ballot_w64(av) == 0ull) continue;
        StencilClass<H, T...>::scan(P, w1, [&](int r, uint32_t ok) { rows[r * WAVE].y = av ? ok : 0u; });
        uint32_t c = 0;
        const double sg = heur_orient_sum((int)(w0 >> 8), 21 - H, rows, hs, edge_w, c);
        if (av) {
            psum[(piece - 1u) * WAVE] += sg;
            count += c;
        }
    }
}

__device__ __forceinline__ uint32_t heur_pass_a(const Planes& P, uint32_t avail, uint2* rows, double* psum,
                                                const HeurShared* hs, int edge_w) {
#pragma unroll
    for (int p = 0; p < BK_PIECES; ++p) psum[p * WAVE] = 0.0;
    uint32_t count = 0;
    int tb0 = 0;  // opaque 0 (see movegen_counts)
    asm volatile("" : "+s"(tb0));
    tb0 = __builtin_amdgcn_readfirstlane(tb0);
#define BK_HEUR_CLASS(i0, i1, H, ...) heur_class<H, __VA_ARGS__>(i0 + tb0, i1 + tb0, P, avail, rows, psum, hs, edge_w, count);
    BK_CLASS_LIST(BK_HEUR_CLASS)
#undef BK_HEUR_CLASS
    return count;
}

// legal anchor rows of orientation gs (per lane) from the {B, C} rows in LDS
__device__ __forceinline__ void lane_ok_rows(int gs, const uint2* rows, uint32_t (&ok)[20]) {
    const uint32_t info = kInfo[gs];
    const int n = (int)((info >> 8) & 0xFFu);
    const int rlim = 20 - (int)((info >> 16) & 0xFFu);
    const uint2* base[5];
    uint32_t sh[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t cell = kCells[gs][k < n ? k : 0];
        base[k] = rows + (cell >> 8) * WAVE;
        sh[k] = cell & 0xFFu;
    }
#pragma unroll
    for (int r = 0; r < 20; ++r) {
        const int rr = r < rlim ? r : rlim;
        uint2 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = base[k][rr * WAVE];
        uint32_t ab = BITOP3(v[0].x >> sh[0], v[1].x >> sh[1], v[2].x >> sh[2], LUT_OR3);
        uint32_t ac = BITOP3(v[0].y >> sh[0], v[1].y >> sh[1], v[2].y >> sh[2], LUT_OR3);
        ab = BITOP3(ab, v[3].x >> sh[3], v[4].x >> sh[4], LUT_OR3);
        ac = BITOP3(ac, v[3].y >> sh[3], v[4].y >> sh[4], LUT_OR3);
        ok[r] = r <= rlim ? (ac & ~ab) : 0u;
    }
}

__device__ __forceinline__ double lane_orient_sum(int gs, const uint32_t (&ok)[20], const uint2* rows,
                                                  const HeurShared* hs, int edge_w) {
    int n;
    uint32_t cd[5], cc[5];
    orient_cells(gs, n, cd, cc);
    double sum = 0.0;
#pragma unroll
    for (int r = 0; r < 20; ++r) {
        uint32_t w = ok[r];
        while (w) {
            const int x = __builtin_ctz(w);
            w &= w - 1u;
            sum += heur_e(n, cd, cc, r, x, rows, hs, edge_w);
        }
    }
    return sum;
}

// The heuristic's choice after pass A (psum per piece): target = u * total; the piece,
// then the orientation (list order: piece asc, orientation asc) whose cumulative e
// crosses it.  rows: {B, C} in LDS.  Returns the orientation (its legal rows in ok) and
// the cumulative e before it in R; uncertain when the crossing is not where the sums say
// (rounding: the choice is then not certified).
__device__ __forceinline__ int heur_pick_orient(const double* psum, const uint2* rows, const HeurShared* hs,
                                                int edge_w, double target, double& R, uint32_t (&ok)[20],
                                                bool& uncertain) {
    int pstar = -1;
    R = 0.0;
#pragma unroll 1
    for (int p = 0; p < BK_PIECES; ++p) {
        const double sp = psum[p * WAVE];
        if (pstar < 0 && sp > 0.0) {
            if (R + sp > target) pstar = p;
            else R += sp;
        }
    }
    if (pstar < 0) {  // u * total rounded up to the total: take the last piece with moves
        uncertain = true;
        R = 0.0;
        for (int p = 0; p < BK_PIECES; ++p)
            if (psum[p * WAVE] > 0.0) pstar = p;
#pragma unroll 1
        for (int p = 0; p < pstar; ++p) R += psum[p * WAVE];
    }
    int gstar = -1, glast = -1;
    double Rstar = R;
    bool found = false;
    const int g1 = hs->first[pstar + 1];
#pragma unroll 1
    for (int g = hs->first[pstar]; g < g1 && !found; ++g) {
        lane_ok_rows(g, rows, ok);
        glast = g;
        const double sg = lane_orient_sum(g, ok, rows, hs, edge_w);
        if (sg > 0.0) {
            gstar = g;
            Rstar = R;
            found = R + sg > target;
            R += sg;
        }
    }
    if (!found) uncertain = true;  // rounding: the last orientation with moves, uncertified
    if (gstar >= 0 && glast != gstar) lane_ok_rows(gstar, rows, ok);
    R = Rstar;
    return gstar;
}

// Walk orientation gs's anchors in the reference's frontier list order (pass 2 of
// locate_move_frontier) accumulating e until the cumulative sum passes target.  ok =
// gs's legal rows; rows[.].y is overwritten, rows[.].x (B) kept.
__device__ __forceinline__ void heur_walk_frontier(int gs, const uint32_t (&ok)[20], uint2* rows, const int16_t* key,
                                                   int mask, const HeurShared* hs, int edge_w, double target,
                                                   double R, double total, int& out_r, int& out_c,
                                                   bool& uncertain) {
#pragma unroll
    for (int r = 0; r < 20; ++r) rows[r * WAVE].y = ok[r];
    int n;
    uint32_t cd[5], cc[5];
    orient_cells(gs, n, cd, cc);
    int found_r = -1, found_c = 0, last_r = -1, last_c = 0;
    double last_lo = R, last_e = 0.0;
    const bk_u4_alias* k4 = reinterpret_cast<const bk_u4_alias*>(key);
#pragma unroll 1
    for (int b0 = 0; b0 <= mask && found_r < 0; b0 += 16) {
        const uint4 qa = k4[b0 >> 3], qb = k4[(b0 >> 3) + 1];
        const uint32_t w[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int f = (int)(int16_t)((j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFFu));
            if (found_r >= 0 || f < 0 || b0 + j > mask) continue;
            const int fr = f / 20, fc = f - 20 * fr;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                if (k >= n || found_r >= 0) continue;
                const int ar = fr - (int)cd[k], acl = fc - (int)cc[k];
                if (ar < 0 || ar > 19 || acl < 0 || acl > 19) continue;
                uint2* rp = rows + ar * WAVE;
                const uint32_t okw = rp->y;
                if (!((okw >> acl) & 1u)) continue;
                rp->y = okw & ~(1u << acl);
                const double e = heur_e(n, cd, cc, ar, acl, rows, hs, edge_w);
                last_r = ar; last_c = acl; last_lo = R; last_e = e;
                if (R + e > target) { found_r = ar; found_c = acl; continue; }
                R += e;
            }
        }
    }
    if (found_r < 0) {  // rounding put the target past the last anchor: take it, uncertified
        uncertain = true;
        found_r = last_r; found_c = last_c;
    }
    // certification: target well inside [lo, lo + e) of the chosen move
    if (!(target - last_lo > HEUR_MARGIN * total && last_lo + last_e - target > HEUR_MARGIN * total))
        uncertain = true;
    out_r = found_r;
    out_c = found_c;
}

// counter[2] of a handle: sticky error bits of device-path launches, reported (and
// cleared) by bk_synchronize
#define BK_STATUS_CAP 8u     // bk_result.status: arena run stopped by the turn cap
#define BK_STATUS_BADFORCE 64u  // bk_arena_step: the forced move is not legal here (game stopped)
// BK_STATUS_STOP (32, include/blokus_hip.h): bk_arena_advance stopped at a stop seat
#define BK_STICKY_GUARD 1u  // a persistent kernel's iteration guard tripped: results incomplete
#define BK_STICKY_ROOT 2u   // a root_index entry outside [0, n_roots)
#define BK_STICKY_FASTMCTS 4u  // k_fastmcts: a root with too many children or a short log table

struct RolloutArgs {
    const bk_state* roots;
    int32_t n_roots;
    const int32_t* root_index;
    int32_t n_playouts;
    bk_rollout_cfg cfg;
    const uint32_t* compat_seeds;
    bk_result* out;
    uint32_t* slab;
    uint32_t nslots;
    uint32_t* counter;  // [0] = next playout; [1] = error word
    uint32_t max_iters; // safety valve: loop iterations any lane can need
    bk_state* out_states; // BK_SEM_ADVANCE
    const bk_fset* root_sets;  // frontier order: roots' tables
    bk_fset* out_sets;         // frontier order + BK_SEM_ADVANCE
    FsLane* fslab;             // frontier order: one record per slot
    const uint8_t* seat_masks; // bk_arena_advance: per game, bits 0-3 heuristic seats, 4-7 stop seats
    uint32_t* rng_io;          // bk_arena_advance: per game 4 seats x MT cursor, in/out
    int32_t handout;           // 0: every lane pulls playouts from the counter; 1: slot s plays
                               // s, s + nslots, ...; 2: slot s plays s, then only slots
                               // < long_slots pull the rest from the counter (whole waves)
    uint32_t long_slots;
    const uint8_t* quick_masks;  // bk_arena_step: per game, bits 0-3 FastMCTS stop seats (stop_out)
    const int32_t* forced;       // bk_arena_step: per game, the stop seat's chosen move (or -1)
    bk_stop_info* stop_out;      // bk_arena_step: per game, the FastMCTS root inputs at a stop
};

// four per-player scalars (kept as separate SSA values: an array indexed by a
// per-lane player would be demoted to scratch memory)
struct Quad {
    uint32_t v0, v1, v2, v3;
    __device__ __forceinline__ uint32_t get(int q) const {
        return q == 0 ? v0 : (q == 1 ? v1 : (q == 2 ? v2 : v3));
    }
    __device__ __forceinline__ void set(int q, uint32_t x) {
        v0 = q == 0 ? x : v0; v1 = q == 1 ? x : v1; v2 = q == 2 ? x : v2; v3 = q == 3 ? x : v3;
    }
};

struct Game {
    int32_t pid;        // playout id, -1 = none
    Quad used;
    uint32_t first;     // bit p
    uint32_t out;       // bit p: known no legal move
    int32_t cur;
    Quad cells;         // squares covered per player
    int32_t plies, passes, turns, since_move;
    int32_t root_player, root_score;
    uint32_t draws;
    uint32_t pcount;    // philox counter
    uint32_t move_count0;
    uint32_t status;    // bk_result.status bits: 1 rng stream overflow, 2 frontier table overflow
    uint32_t hmask;     // seats playing HeuristicAgent
    uint32_t smask;     // stop seats (bk_arena_advance)
    int32_t cap;        // turn / ply budget of this game in this launch
    uint32_t turns0, passes0;  // bk_arena_advance: the game's counts before this launch
    int32_t forced;     // bk_arena_step: the stop seat's move to place first (-1: none)
};

__device__ __forceinline__ int board_score_q(const Game& g, int q) {  // q static
    return (int)g.cells.get(q) + ((g.used.get(q) == 0x1FFFFFu) ? 15 : 0);
}
__device__ __forceinline__ int board_score(const Game& g, int p) {  // p per-lane
    return (int)g.cells.get(p) + ((g.used.get(p) == 0x1FFFFFu) ? 15 : 0);
}

// write the lane's board back as a bk_state (BK_SEM_ADVANCE)
__device__ __forceinline__ void store_state(const RolloutArgs& a, const Game& g, const Slab& slab) {
    bk_state* o = a.out_states + g.pid;
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
        uint64_t w[7] = {0, 0, 0, 0, 0, 0, 0};
        const uint32_t* pl = slab.base + p * 20;
#pragma unroll
        for (int R = 0; R < 20; ++R) {
            const uint64_t v = pl[R];
            const int bit = 20 * R, word = bit >> 6, off = bit & 63;
            w[word] |= v << off;
            if (off > 44) w[word + 1] |= v >> (64 - off);
        }
#pragma unroll
        for (int k = 0; k < 7; ++k) o->planes[p][k] = w[k];
        o->used[p] = g.used.get(p);
    }
    o->first_move = (uint8_t)g.first;
    o->current_player = (uint8_t)g.cur;
    o->out_mask = (uint8_t)g.out;
    o->flags = 0;
    o->move_count = (uint16_t)(g.move_count0 + g.plies);
    o->reserved16 = 0;
    // bk_arena_advance: the game's arena turn_count / passes so far (raw, see finish_game)
    o->reserved[0] = a.seat_masks ? g.turns0 + (uint32_t)g.turns : 0u;
    o->reserved[1] = a.seat_masks ? g.passes0 + (uint32_t)g.passes : 0u;
}

// player p's table header in the rollout slab (frontier order, SLAB_HDR_BASE)
__device__ __forceinline__ uint16_t* slab_hdr(const Slab& slab, int p) {
    return reinterpret_cast<uint16_t*>(&slab.word(SLAB_HDR_BASE)) + 3 * p;
}

// a plain copy of the four tables: slots 0..mask of each (the rest is never read) and
// the counters, as uint4
__device__ __forceinline__ void copy_fset(bk_fset* dst, const bk_fset* src) {
    static_assert(sizeof(bk_fset) % 16 == 0 && BK_FSET_SLOTS % 8 == 0, "bk_fset is copied as uint4");
    const bk_u4_alias* tail_s = reinterpret_cast<const bk_u4_alias*>(&src->mask[0]);
    bk_u4_alias* tail_d = reinterpret_cast<bk_u4_alias*>(&dst->mask[0]);
    const uint4 t0 = tail_s[0], t1 = tail_s[1];  // mask[4] fill[4] used[4] reserved[4]
    tail_d[0] = t0;
    tail_d[1] = t1;
    const uint32_t masks[4] = {t0.x & 0xFFFFu, t0.x >> 16, t0.y & 0xFFFFu, t0.y >> 16};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bk_u4_alias* s4 = reinterpret_cast<const bk_u4_alias*>(src->key[q]);
        bk_u4_alias* d4 = reinterpret_cast<bk_u4_alias*>(dst->key[q]);
        const int nv = (int)(masks[q] + 1u) / 8;  // 8 slots per uint4
#pragma unroll 2
        for (int i = 0; i < nv; ++i) d4[i] = s4[i];
    }
}

// copy_fset with the headers (mask, fill, used) to / from the rollout slab instead of the
// record's header line (the record's own header is not kept up to date)
__device__ __forceinline__ void copy_fset_in(bk_fset* dst, const Slab& slab, const bk_fset* src) {
    const bk_u4_alias* tail_s = reinterpret_cast<const bk_u4_alias*>(&src->mask[0]);
    const uint4 t0 = tail_s[0], t1 = tail_s[1];  // mask[4] fill[4] used[4] reserved[4]
    const uint32_t masks[4] = {t0.x & 0xFFFFu, t0.x >> 16, t0.y & 0xFFFFu, t0.y >> 16};
    const uint32_t fills[4] = {t0.z & 0xFFFFu, t0.z >> 16, t0.w & 0xFFFFu, t0.w >> 16};
    const uint32_t useds[4] = {t1.x & 0xFFFFu, t1.x >> 16, t1.y & 0xFFFFu, t1.y >> 16};
    // (mask, fill, used) x 4 as 6 dwords
    slab.word(SLAB_HDR_BASE + 0) = masks[0] | (fills[0] << 16);
    slab.word(SLAB_HDR_BASE + 1) = useds[0] | (masks[1] << 16);
    slab.word(SLAB_HDR_BASE + 2) = fills[1] | (useds[1] << 16);
    slab.word(SLAB_HDR_BASE + 3) = masks[2] | (fills[2] << 16);
    slab.word(SLAB_HDR_BASE + 4) = useds[2] | (masks[3] << 16);
    slab.word(SLAB_HDR_BASE + 5) = fills[3] | (useds[3] << 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bk_u4_alias* s4 = reinterpret_cast<const bk_u4_alias*>(src->key[q]);
        bk_u4_alias* d4 = reinterpret_cast<bk_u4_alias*>(dst->key[q]);
        const int nv = (int)(masks[q] + 1u) / 8;  // 8 slots per uint4
#pragma unroll 2
        for (int i = 0; i < nv; ++i) d4[i] = s4[i];
    }
}

__device__ __forceinline__ void copy_fset_out(bk_fset* dst, const bk_fset* src, const Slab& slab) {
    uint32_t h[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) h[i] = slab.word(SLAB_HDR_BASE + i);
    const uint32_t masks[4] = {h[0] & 0xFFFFu, h[1] >> 16, h[3] & 0xFFFFu, h[4] >> 16};
    const uint32_t fills[4] = {h[0] >> 16, h[2] & 0xFFFFu, h[3] >> 16, h[5] & 0xFFFFu};
    const uint32_t useds[4] = {h[1] & 0xFFFFu, h[2] >> 16, h[4] & 0xFFFFu, h[5] >> 16};
    bk_u4_alias* tail_d = reinterpret_cast<bk_u4_alias*>(&dst->mask[0]);
    tail_d[0] = make_uint4(masks[0] | (masks[1] << 16), masks[2] | (masks[3] << 16), fills[0] | (fills[1] << 16),
                           fills[2] | (fills[3] << 16));
    tail_d[1] = make_uint4(useds[0] | (useds[1] << 16), useds[2] | (useds[3] << 16), 0u, 0u);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bk_u4_alias* s4 = reinterpret_cast<const bk_u4_alias*>(src->key[q]);
        bk_u4_alias* d4 = reinterpret_cast<bk_u4_alias*>(dst->key[q]);
        const int nv = (int)(masks[q] + 1u) / 8;
#pragma unroll 2
        for (int i = 0; i < nv; ++i) d4[i] = s4[i];
    }
}

// fs_copy of table q on the device, as uint4 rows (8 slots each): the same-shape case
// (set_merge's pointer copy) is a plain uint4 copy, the clean re-insert reads 8 keys per
// load.  Equal to fs_copy slot for slot.
__device__ __forceinline__ bool fs_copy_dev(bk_fset* d, int q, const bk_fset* s, const uint64_t* htab) {
    const uint32_t smask = s->mask[q], sfill = s->fill[q], sused = s->used[q];
    uint32_t newsize = 8;
    if (sused * 5 >= 7u * 3u)
        while (newsize <= sused * 2) newsize <<= 1;
    bk_u4_alias* d4 = reinterpret_cast<bk_u4_alias*>(d->key[q]);
    const bk_u4_alias* s4 = reinterpret_cast<const bk_u4_alias*>(s->key[q]);
    if (newsize > BK_FSET_SLOTS) {
        fs_clear(fs_ref(d, q, htab));
        return false;
    }
    d->mask[q] = (uint16_t)(newsize - 1);
    d->fill[q] = (uint16_t)sused;
    d->used[q] = (uint16_t)sused;
    if (newsize - 1 == smask && sfill == sused) {
#pragma unroll 2
        for (uint32_t i = 0; i < newsize / 8; ++i) d4[i] = s4[i];
        return true;
    }
    const uint4 unused = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);  // FS_UNUSED pairs
#pragma unroll 2
    for (uint32_t i = 0; i < newsize / 8; ++i) d4[i] = unused;
    if (sused == 0) return true;
    const FsetRef t = fs_ref(d, q, htab);
#pragma unroll 1
    for (uint32_t i = 0; i <= smask / 8; ++i) {
        const uint4 v = s4[i];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int16_t k = (int16_t)((j & 1) ? (w[j >> 1] >> 16) : (w[j >> 1] & 0xFFFFu));
            if (k >= 0) fs_insert_clean(t, newsize - 1, k);
        }
    }
    return true;
}

template <bool FR>
__device__ __forceinline__ void finish_game(const RolloutArgs& a, Game& g, const Slab& slab, uint32_t slot) {
    if (a.rng_io) {  // the seats' streams go on in the next call
        uint4 t[4];  // 16-byte copies, loads first
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] = reinterpret_cast<const uint4*>(&slab.word(SLAB_RNG_BASE))[q];
#pragma unroll
        for (int q = 0; q < 4; ++q) reinterpret_cast<uint4*>(a.rng_io + (size_t)g.pid * 16)[q] = t[q];
    }
    if (a.out_states != nullptr) {  // BK_SEM_ADVANCE, or an arena run that wants final states
        store_state(a, g, slab);
        if constexpr (FR) copy_fset_out(a.out_sets + g.pid, &a.fslab[slot].s, slab);
        if (a.out == nullptr) { g.pid = -1; return; }
    }
    bk_result r;
    memset(&r, 0, sizeof r);
    if (a.cfg.semantics != BK_SEM_ROLLOUT) {
        int best = -1000000;
        Quad sc{0, 0, 0, 0};
#pragma unroll 1
        for (int p = 0; p < 4; ++p) {
            const uint32_t* pl = slab.base + p * 20;
            const uint32_t r0 = pl[0], r19 = pl[19];
            int s = board_score(g, p);
            s += 5 * (int)((r0 & 1u) + ((r0 >> 19) & 1u) + (r19 & 1u) + ((r19 >> 19) & 1u));
            uint32_t centre = 0;
#pragma unroll
            for (int R = 8; R < 12; ++R) centre += __builtin_popcount(pl[R] & 0x00000F00u);
            s += 2 * (int)centre;
            sc.set(p, (uint32_t)s);
            best = s > best ? s : best;
        }
        uint8_t wm = 0;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            r.scores[p] = (int16_t)(int)sc.get(p);
            wm |= (uint8_t)(((int)sc.get(p) == best) << p);
        }
        r.winner_mask = wm;
        if (g.out == 0xFu || a.cfg.semantics != BK_SEM_ARENA) {
            // passes detected lazily after the final move are not counted by the
            // reference, whose game-over check runs right after each move
            // (engine/game.py:182-214)
            r.passes = (uint16_t)(g.passes - g.since_move);
            r.turns = (uint16_t)(g.turns - g.since_move);
        } else {
            // stopped by the turn cap (arena max_turns) before every player was known
            // to be stuck: the game may or may not be over.  Raw counts, the passes since
            // the last move in reserved[0]; the host decides with has_moves on the final
            // state (arena_runner.py:702), discounting them if the game is over.  (Or
            // stopped at a stop seat, BK_STATUS_STOP: the game goes on, counts are real.)
            r.passes = (uint16_t)g.passes;
            r.turns = (uint16_t)g.turns;
            r.reserved[0] = (uint32_t)g.since_move;
            if (!(g.status & BK_STATUS_STOP)) g.status |= BK_STATUS_CAP;
        }
    } else {
        int best = -1000000;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            r.scores[p] = (int16_t)board_score_q(g, p);
            best = r.scores[p] > best ? r.scores[p] : best;
        }
        r.reward = board_score(g, g.root_player) - g.root_score;
        r.turns = (uint16_t)g.turns;
    }
    r.plies = (uint16_t)g.plies;
    r.draws = g.draws;
    r.status = (uint8_t)g.status;
    a.out[g.pid] = r;
    g.pid = -1;
}

template <bool FR>
__device__ __forceinline__ void start_game(const RolloutArgs& a, Game& g, const Slab& slab, uint32_t slot, int32_t pid,
                                           const uint64_t* htab) {
    int32_t ri = a.root_index ? a.root_index[pid] : (pid % a.n_roots);
    bool bad_root = false;
    if (ri < 0 || ri >= a.n_roots) {  // device-path input error: flagged, never read out of bounds
        atomicOr(&a.counter[2], BK_STICKY_ROOT);
        ri = 0;
        bad_root = true;
    }
    const bk_state* s = a.roots + ri;
    g.pid = pid;
    uint32_t occ[20];
#pragma unroll
    for (int R = 0; R < 20; ++R) occ[R] = 0;
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {  // runtime loop: keeps only one player's words live
        uint32_t cells = 0;
        uint64_t w[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) w[k] = s->planes[p][k];
        uint32_t* dst = slab.base + p * 20;
#pragma unroll
        for (int R = 0; R < 20; ++R) {
            const uint32_t row = plane_row(w, R);
            dst[R] = row;
            occ[R] |= row;
            cells += __builtin_popcount(row);
        }
        g.cells.set(p, cells);
        g.used.set(p, s->used[p] & 0x1FFFFFu);
    }
#pragma unroll
    for (int R = 0; R < 20; ++R) slab.at(4, R) = occ[R];
    g.first = s->first_move & 0xFu;
    g.out = a.cfg.semantics != BK_SEM_ROLLOUT ? (s->out_mask & 0xFu) : 0u;
    g.move_count0 = s->move_count;
    g.cur = s->current_player & 3;
    g.plies = g.passes = g.turns = g.since_move = 0;
    g.root_player = g.cur;
    g.root_score = board_score(g, g.cur);
    g.draws = 0;
    g.pcount = 0;
    g.status = bad_root ? 4u : 0u;
    if constexpr (FR) {
        if (a.cfg.semantics == BK_SEM_ROLLOUT) {
            // MCTSAgent._rollout plays on sim = board.copy() (mcts/mcts_agent.py:470):
            // set.copy() re-lays the tables out
            bk_fset* d = &a.fslab[slot].s;
            const bk_fset* src = a.root_sets + ri;
#pragma unroll 1
            for (int q = 0; q < 4; ++q) {
                if (!fs_copy_dev(d, q, src, htab)) g.status |= 2u;
                uint16_t* hq = slab_hdr(slab, q);  // the header lives in the slab from here on
                hq[0] = d->mask[q];
                hq[1] = d->fill[q];
                hq[2] = d->used[q];
            }
        } else {
            copy_fset_in(&a.fslab[slot].s, slab, a.root_sets + ri);
        }
    }
    g.hmask = a.seat_masks ? (a.seat_masks[pid] & 0xFu) : (uint32_t)a.cfg.heuristic_seats;
    g.smask = a.seat_masks ? ((a.seat_masks[pid] >> 4) & 0xFu) : 0u;
    g.turns0 = a.seat_masks ? s->reserved[0] : 0u;
    g.passes0 = a.seat_masks ? s->reserved[1] : 0u;
    g.cap = a.cfg.max_plies - (int32_t)g.turns0;  // arena_runner max_turns over the whole game
    g.forced = a.forced ? a.forced[pid] : -1;
    if (a.rng_io) {  // seats' streams carried over from the previous call
        {  // 16-byte copies, loads first (the two pointers may alias as far as the compiler knows)
            uint4 t[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) t[q] = reinterpret_cast<const uint4*>(a.rng_io + (size_t)pid * 16)[q];
#pragma unroll
            for (int q = 0; q < 4; ++q) reinterpret_cast<uint4*>(&slab.word(SLAB_RNG_BASE))[q] = t[q];
        }
    } else if (a.cfg.rng == BK_RNG_NUMPY_MT) {
        const int nstreams = a.cfg.seats_share_stream ? 1 : 4;
        for (int q = 0; q < nstreams; ++q) {
            const MtCursor m = mt_cursor_init(a.compat_seeds[(size_t)pid * 4 + q]);
            slab.word(SLAB_RNG_BASE + 4 * q + 0) = m.i;
            slab.word(SLAB_RNG_BASE + 4 * q + 1) = m.a;
            slab.word(SLAB_RNG_BASE + 4 * q + 2) = m.b;
            slab.word(SLAB_RNG_BASE + 4 * q + 3) = m.c;
        }
    }
}

// uniform index in [0, n) for the current mover; numpy legacy masked rejection
__device__ __forceinline__ uint32_t draw_index(const RolloutArgs& a, Game& g, const Slab& slab, uint32_t slot,
                                               uint32_t n) {
    const uint32_t rng = n - 1u;
    if (rng == 0u) return 0u;  // randint(0, 1) consumes no draw
    const uint32_t mask = mask_for(rng);
    uint32_t v;
    if (a.cfg.rng == BK_RNG_NUMPY_MT) {
        const int q = a.cfg.seats_share_stream ? 0 : g.cur;
        uint32_t* base = slab.base + SLAB_RNG_BASE + 4 * q;
        MtCursor m;
        m.i = base[0]; m.a = base[1]; m.b = base[2]; m.c = base[3];
        bool ov = (g.status & 1u) != 0u;
        do {
            v = mt_cursor_next(m, ov) & mask;
            g.draws++;
        } while (v > rng && !ov);
        if (ov) g.status |= 1u;
        base[0] = m.i; base[1] = m.a; base[2] = m.b; base[3] = m.c;
        if (v > rng) v = 0;
    } else {
        do {
            v = philox_u32(g.pcount++, (uint32_t)g.pid + a.cfg.stream_base, a.cfg.seed) & mask;
            g.draws++;
        } while (v > rng);
    }
    return v;
}

// RandomState.random_sample() of the current mover's stream (genrand_res53: two 32-bit
// outputs), as rng.choice draws it (agents/heuristic_agent.py:65)
__device__ __forceinline__ double draw_double(const RolloutArgs& a, Game& g, const Slab& slab) {
    uint32_t x0, x1;
    if (a.cfg.rng == BK_RNG_NUMPY_MT) {
        const int q = a.cfg.seats_share_stream ? 0 : g.cur;
        uint32_t* base = slab.base + SLAB_RNG_BASE + 4 * q;
        MtCursor m;
        m.i = base[0]; m.a = base[1]; m.b = base[2]; m.c = base[3];
        bool ov = (g.status & 1u) != 0u;
        x0 = mt_cursor_next(m, ov);
        x1 = mt_cursor_next(m, ov);
        if (ov) g.status |= 1u;
        base[0] = m.i; base[1] = m.a; base[2] = m.b; base[3] = m.c;
    } else {
        x0 = philox_u32(g.pcount++, (uint32_t)g.pid + a.cfg.stream_base, a.cfg.seed);
        x1 = philox_u32(g.pcount++, (uint32_t)g.pid + a.cfg.stream_base, a.cfg.seed);
    }
    g.draws += 2;
    return ((double)(x0 >> 5) * 67108864.0 + (double)(x1 >> 6)) * (1.0 / 9007199254740992.0);
}

// bk_arena_step: the FastMCTSAgent root inputs of game g stopped at FastMCTS seat p
// (agents/fast_mcts_agent.py:260-298): the legal-move count, and _quick_move_evaluation --
// of the first 3 moves by piece id descending (a stable sort of the list: the first moves,
// in list order, of the largest pieces with moves), the first nearest the centre by
// |anchor_row - 9.5| + |anchor_col - 9.5| -- as its list index and its reward
// pid * 0.1 + (20 - dist) * 0.05 (CPython float ops, no fused multiply-add).  The counts
// are recomputed (the LDS area held other data since); locate overwrites the rows' C
// half, so the rows are rewritten before each of the (at most 3) locates.
__device__ __forceinline__ void stop_info(const RolloutArgs& a, const Game& g, const Planes& P, uint32_t* my, int lane,
                                       uint2* rows_lds, const bk_fset* fs, int fmask, int p, uint32_t avail,
                                       uint32_t total) {
    bk_stop_info si;
    si.n_legal = (int32_t)total;
    si.quick_index = 0;
    si.quick_reward = 0.0;
    if (a.quick_masks && ((a.quick_masks[g.pid] >> p) & 1u)) {
        (void)movegen_counts<true>(P, avail, my, lane);
        // list positions of the first 3 moves by piece descending: orientations are
        // piece-major, so piece P's moves are one run [s, s + c) of the list
        uint32_t k3[3] = {0u, 0u, 0u}, suf = 0u, cp = 0u;
        int n3 = 0;
#pragma unroll 1
        for (int gg = BK_NUM_ORIENTS - 1; gg >= 0 && n3 < 3; --gg) {
            cp += (my[(gg / 3) * WAVE + lane] >> (10 * (gg % 3))) & 0x3FFu;
            const uint32_t piece = kInfo[gg] & 0xFFu;
            if (gg == 0 || (kInfo[gg - 1] & 0xFFu) != piece) {  // first orientation of the piece
                const uint32_t s0 = total - suf - cp;
                for (uint32_t j = 0; j < cp && n3 < 3; ++j) k3[n3++] = s0 + j;
                suf += cp;
                cp = 0u;
            }
        }
        uint32_t kk3[3] = {0u, 0u, 0u};
        int g3[3] = {0, 0, 0};
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (i < n3) g3[i] = pick_orient(my, lane, k3[i], kk3[i]);  // before the rows overwrite the counts
        double best = 0.0;
        int q = -1;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (i >= n3) continue;
#pragma unroll
            for (int R = 0; R < 20; ++R) rows_lds[R * WAVE] = make_uint2(P.b(R), P.c(R));
            int ar, ac;
            locate_move_frontier(g3[i], kk3[i], rows_lds, fs->key[p], fmask, ar, ac);
            const double d = __dadd_rn(fabs((double)ar - 9.5), fabs((double)ac - 9.5));
            if (q < 0 || d < best) { best = d; q = i; }  // min(): the first nearest
        }
        if (q >= 0) {
            si.quick_index = (int32_t)k3[q];
            si.quick_reward = __dadd_rn(__dmul_rn((double)(kInfo[g3[q]] & 0xFFu), 0.1),
                                        __dmul_rn(__dadd_rn(20.0, -best), 0.05));
        }
    }
    a.stop_out[g.pid] = si;
}

// heuristic-policy kernels: 128-lane blocks, per lane 84 LDS dwords ({B, C} rows, then
// 21 per-piece e sums as doubles; the frontier-table staging reuses the area)
#define HBLOCK 128
#define HEUR_WORDS (84 * WAVE)
#define HEUR_PSUM 40  // dword offset of the per-piece sums in a wave's area

template <bool FR, bool HEUR = false>
__device__ __forceinline__ void rollout_body(const RolloutArgs& a) {
    constexpr int BLK = HEUR ? HBLOCK : BLOCK;
    constexpr int AREA = HEUR ? HEUR_WORDS : FR ? ROLL_WORDS_FR : ROLL_WORDS_PER_WAVE;
    constexpr int HS_WORDS = HEUR ? (int)(sizeof(HeurShared) + 7) / 4 : 0;
    // HEUR (k_rollout_fr_h): + the CPython cell hashes (shared by the block) for the
    // frontier tables and the policy's exp tables; k_rollout_fr reads the hashes from
    // global memory through the L1, so its LDS fits 4 blocks per CU
    constexpr bool HT_LDS = FR && HEUR;
    __shared__ __attribute__((aligned(16))) uint32_t lds[AREA * (BLK / WAVE) + (HT_LDS ? 2 * BK_CELLS : 0) + HS_WORDS];
    const int lane0 = threadIdx.x & (WAVE - 1), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    uint64_t* htab_lds = reinterpret_cast<uint64_t*>(lds + AREA * (BLK / WAVE));
    const uint64_t* htab = HT_LDS ? htab_lds : kCellHash;
    HeurShared* hs = reinterpret_cast<HeurShared*>(lds + AREA * (BLK / WAVE) + (HT_LDS ? 2 * BK_CELLS : 0));
    if constexpr (HT_LDS) {
        for (int i = threadIdx.x; i < BK_CELLS; i += BLK) htab_lds[i] = kCellHash[i];
    }
    if constexpr (HEUR) heur_shared_init(hs, threadIdx.x, BLK);
    if constexpr (HT_LDS || HEUR) __syncthreads();
    const uint32_t slot0 = blockIdx.x * BLK + threadIdx.x;
    // The lane's slot and lane index are laundered once per ply, so the addresses derived
    // from them (slab, frontier record, LDS columns) are recomputed in the loop instead of
    // being held in registers for the whole kernel (spilled across the stencil)
    uint32_t* const my = lds + wv * AREA;
    const bool arena = a.cfg.semantics != BK_SEM_ROLLOUT;  // passes allowed
    const bool advance = a.cfg.semantics == BK_SEM_ADVANCE;

    Game g;
    g.pid = -1;
    bool done = false;
    uint32_t handed = 0;  // playouts this slot has taken (handout 1, 2)
    SECT_DECL
    for (uint32_t iter = 0;; ++iter) {
        uint32_t slot = slot0;
        int lane = lane0;
        asm volatile("" : "+v"(slot), "+v"(lane));
        const Slab slab{a.slab + (size_t)slot * SLAB_WORDS};
        uint2* const rows_lds = reinterpret_cast<uint2*>(my) + lane;  // + R * WAVE
        double* const psum = reinterpret_cast<double*>(my + HEUR_PSUM * WAVE) + lane;  // + piece * WAVE
        SECT(0);
        // ---- make sure this lane has a game whose current player may still move
        for (int guard = 0; guard < 3 && !done; ++guard) {
            if (g.pid < 0) {
                int32_t next;
                if (a.handout == 0) {
                    next = (int32_t)atomicAdd(&a.counter[0], 1u);
                } else if (handed == 0u) {
                    next = (int32_t)slot;
                } else if (a.handout == 1) {
                    next = (int32_t)(slot + handed * a.nslots);
                } else {
                    next = slot < a.long_slots ? (int32_t)(a.nslots + atomicAdd(&a.counter[0], 1u)) : a.n_playouts;
                }
                ++handed;
                if (next >= a.n_playouts) { done = true; break; }
                // bk_arena_step: a game whose search is still running is left untouched
                if (HEUR && a.forced && a.forced[next] == BK_FORCE_SKIP) continue;
                start_game<FR>(a, g, slab, slot, next, htab);
            }
            if (arena) {
#pragma unroll 1
                for (int s = 0; s < 4 && ((g.out >> g.cur) & 1u) && g.out != 0xFu && (advance || g.turns < g.cap); ++s) {
                    g.passes++; g.turns++; g.since_move++;
                    g.cur = (g.cur + 1) & 3;
                }
                if (g.out == 0xFu || (advance ? g.plies : g.turns) >= g.cap) {
                    finish_game<FR>(a, g, slab, slot);
                    continue;
                }
            } else if (g.plies >= g.cap) {
                finish_game<FR>(a, g, slab, slot);
                continue;
            }
            break;
        }
        if (__ballot(!done) == 0ull) break;
        if (iter > a.max_iters) {  // safety valve: never spin forever
            if (lane == 0) { atomicOr(&a.counter[1], 1u); atomicOr(&a.counter[2], BK_STICKY_GUARD); }
            break;
        }
        SECT(1);
        // ---- derive + movegen for every active lane (uniform work)
        const bool idle = done || g.pid < 0;
        const int p = idle ? 0 : g.cur;
        Planes P;
        {
            uint32_t own[20], occ[20];
#pragma unroll
            for (int R = 0; R < 20; ++R) {
                own[R] = idle ? 0u : slab.at(p, R);
                occ[R] = idle ? 0u : slab.at(4, R);
            }
            derive_rows(own, occ, (g.first >> p) & 1u, p, P);
        }
        make_pairs(P);
        const uint32_t avail = idle ? 0u : (~g.used.get(p) & 0x1FFFFFu);
        uint32_t total;
        int gs = 0;
        uint32_t kk = 0;
        // heuristic policy (HEUR kernels): this lane's mover plays HeuristicAgent
        // bk_arena_step: this ply places the stop seat's chosen move (HEUR kernels only)
        const bool forced = HEUR && !idle && g.forced >= 0;
        const bool heur = HEUR && !idle && !forced && ((g.hmask >> p) & 1u);
        double h_target = 0.0, h_R = 0.0, h_total = 0.0;
        uint32_t h_ok[20];
        bool h_unc = false;
        if constexpr (HEUR) {
            total = 0;
            // uniform-random movers: counts, draw, orientation (before the area is reused)
            if (__builtin_amdgcn_ballot_w64(!idle && !heur)) {
                const uint32_t t = movegen_counts<true>(P, heur ? 0u : avail, my, lane);
                if (!idle && !heur) {
                    total = t;
                    // (a stop seat draws nothing: bk_arena_advance hands its turn back; a
                    // forced list index k picks its move as a draw of k would)
                    if (forced) {
                        gs = -1;
                        if ((g.forced & BK_FORCE_INDEX) && (uint32_t)(g.forced & ~BK_FORCE_INDEX) < t)
                            gs = pick_orient(my, lane, (uint32_t)(g.forced & ~BK_FORCE_INDEX), kk);
                    } else if (t > 0u && !((g.smask >> p) & 1u)) {
                        gs = pick_orient(my, lane, draw_index(a, g, slab, slot, t), kk);
                    }
                }
            }
            if (__builtin_amdgcn_ballot_w64(heur)) {
                const int edge_w = (g.move_count0 + g.plies) < 30 ? 6 : 3;  // move_count / 100.0 < 0.3
#pragma unroll
                for (int R = 0; R < 20; ++R) rows_lds[R * WAVE].x = P.b(R);
                const uint32_t t = heur_pass_a(P, heur ? avail : 0u, rows_lds, psum, hs, edge_w);
#pragma unroll
                for (int R = 0; R < 20; ++R) rows_lds[R * WAVE] = make_uint2(P.b(R), P.c(R));
                if (heur) {
                    total = t;
                    if (t > 0u) {
#pragma unroll 1
                        for (int q = 0; q < BK_PIECES; ++q) h_total += psum[q * WAVE];
                        h_target = draw_double(a, g, slab) * h_total;
                        gs = heur_pick_orient(psum, rows_lds, hs, edge_w, h_target, h_R, h_ok, h_unc);
                    }
                }
            }
        } else {
            total = movegen_counts<true>(P, avail, my, lane);
        }
        SECT(2);
        if (idle) continue;
        if (FR && total > 0u && ((g.smask >> p) & 1u) && !forced) {  // a search seat is to move: hand the game back
            if constexpr (HEUR) {
                if (a.stop_out)
                    stop_info(a, g, P, my, lane, rows_lds, &a.fslab[slot].s, (int)*slab_hdr(slab, p), p, avail, total);
            }
            g.status |= BK_STATUS_STOP;
            finish_game<FR>(a, g, slab, slot);
            continue;
        }
        bool fmove = false;  // forced as a move int (bk_mcts best_move): no pick, no locate
        if constexpr (HEUR) {
            if (forced) {
                fmove = !(g.forced & BK_FORCE_INDEX);
                // a move int must name an orientation of a piece the mover still holds (the
                // anchor's legality is checked against the orientation's legal set below)
                const int fg = g.forced / 400;
                const bool bad = total == 0u ||
                                 (fmove ? (fg >= BK_NUM_ORIENTS || !((avail >> ((kInfo[fg] & 0xFFu) - 1u)) & 1u))
                                        : gs < 0);
                if (bad) {
                    g.status |= BK_STATUS_BADFORCE;
                    finish_game<FR>(a, g, slab, slot);
                    continue;
                }
            }
        }
        if (total == 0u) {
            if (arena) {
                g.out |= 1u << p;
                g.passes++; g.turns++; g.since_move++;
                g.cur = (g.cur + 1) & 3;
            } else {
                finish_game<FR>(a, g, slab, slot);  // MCTSAgent._rollout breaks
            }
            continue;
        }
        if constexpr (!HEUR) {
            const uint32_t k = draw_index(a, g, slab, slot, total);
            gs = pick_orient(my, lane, k, kk);
        }
        // the picked orientation's table entries (loads issued before the rows' LDS writes)
        OrientRow orow = orient_row(gs < 0 ? 0 : gs);
        // counts are consumed: the area now takes the mover's rows for locate
#pragma unroll
        for (int R = 0; R < 20; ++R) rows_lds[R * WAVE] = make_uint2(P.b(R), P.c(R));
        SECT(3);
        int ar, ac;
        if constexpr (FR) {
            const bk_fset* fs = &a.fslab[slot].s;
            const int fmask = (int)*slab_hdr(slab, p);
            if (fmove) {  // the search's move: legal iff its anchor is in the orientation's legal set
                gs = g.forced / 400;
                ar = (g.forced % 400) / 20;
                ac = g.forced % 20;
                orow = orient_row(gs);
                locate_pass1(gs, rows_lds);
                if (!((rows_lds[ar * WAVE].y >> ac) & 1u)) ar = -1;
            } else if (heur && gs < 0) {
                ar = -1;
                ac = 0;
            } else if (heur) {
                const int edge_w = (g.move_count0 + g.plies) < 30 ? 6 : 3;
                heur_walk_frontier(gs, h_ok, rows_lds, fs->key[p], fmask, hs, edge_w, h_target, h_R, h_total,
                                   ar, ac, h_unc);
                if (h_unc) g.status |= BK_STATUS_UNCERT;
            } else {
                locate_move_frontier(orow, kk, rows_lds, fs->key[p], fmask, ar, ac);
            }
        } else {
            locate_move_lds(orow, kk, rows_lds, ar, ac);
        }
        if (HEUR && ar < 0) {  // cannot happen (counts > 0 means e sums > 0); never write off the board
            g.status |= forced ? BK_STATUS_BADFORCE : BK_STATUS_UNCERT;
            finish_game<FR>(a, g, slab, slot);
            continue;
        }
        if constexpr (HEUR) g.forced = -1;  // consumed
        SECT(4);
        // ---- apply (engine/board.py:515-555): own plane, occupancy, used, first, score
        const uint32_t info = orow.info;
        const int n = (int)((info >> 8) & 0xFFu);
        // per piece row d: one mask; all row loads issued before any store
        uint32_t m[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const uint32_t cell = orow.cell[q];
            const uint32_t bit = q < n ? (1u << (ac + (int)(cell & 0xFFu))) : 0u;
#pragma unroll
            for (int d = 0; d < 5; ++d) m[d] |= ((cell >> 8) == (uint32_t)d) ? bit : 0u;
        }
        {
            uint32_t ow[5], oc[5];
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                ow[d] = m[d] ? slab.at(p, ar + d) : 0u;
                oc[d] = m[d] ? slab.at(4, ar + d) : 0u;
            }
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                if (m[d]) {
                    slab.at(p, ar + d) = ow[d] | m[d];
                    slab.at(4, ar + d) = oc[d] | m[d];
                }
            }
        }
        SECT(5);
        if constexpr (FR) {  // the mover's frontier set (engine/board.py:548 -> :315-367)
            int32_t cells[5];
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                const uint32_t cell = q < n ? orow.cell[q] : orow.cell[0];
                cells[q] = (ar + (int)(cell >> 8)) * 20 + ac + (int)(cell & 0xFFu);
            }
            // before the table staging reuses the area
            const uint64_t real = frontier_ops(rows_lds, slab, p, (g.first >> p) & 1u, orow, ar, ac, m);
            SECT(7);
            int16_t* lk = reinterpret_cast<int16_t*>(lds + wv * AREA) + 2 * lane;
            // (HEUR: the area holds 84 dwords per lane, a 128-slot stage fits)
#ifdef BK_SECTION_PROF
            auto mark = [&](int i) { SECT(i); };
#else
            NoMark mark;
#endif
            // (staging every table of <= 128 slots in packed per-lane segments of the area,
            // so no lane probes its table in global memory, measured slower: 34.2 -> 31.7 M
            // playouts/s, profiles/r05/sweeps/r05i: the kernel is issue-bound, not waiting)
            // resize scratch: the area's dwords after the stage (FR: 32..39, HEUR: 64..83)
            constexpr int STG = HEUR ? 128 : BK_FS_STAGE_FR;
            static_assert(STG / 2 + STG / 8 <= AREA / WAVE, "the resize scratch fits the area");
            if (!place_frontier<STG>(&a.fslab[slot], p, lk, htab, cells, real, mark, slab_hdr(slab, p),
                                     lk + 2 * WAVE * (STG / 2)))
                g.status |= 2u;
        }
        SECT(6);
        g.cells.set(p, g.cells.get(p) + (uint32_t)n);
        g.used.set(p, g.used.get(p) | (1u << ((info & 0xFFu) - 1u)));
        g.first &= ~(1u << p);
        g.plies++; g.turns++; g.since_move = 0;
        g.cur = (g.cur + 1) & 3;
        if constexpr (FR) {
            if (g.status & 2u) finish_game<FR>(a, g, slab, slot);  // status 2: table overflow
        }
    }
    SECT_FLUSH;
}

// Two entry points over one body so profiles separate root generation (bk_advance)
// from the measured playouts (bk_rollout).
#if BK_DEF(BK_U_ROLLOUT)
__global__ __launch_bounds__(BLOCK, ROLL_BLOCKS_PER_CU) void k_rollout(RolloutArgs a) { rollout_body<false>(a); }
#else
__global__ void k_rollout(RolloutArgs a);
#endif
#if BK_DEF(BK_U_ROLLOUT)
__global__ __launch_bounds__(BLOCK, ROLL_BLOCKS_PER_CU) void k_advance(RolloutArgs a) { rollout_body<false>(a); }
#else
__global__ void k_advance(RolloutArgs a);
#endif
// reference frontier order (compat parity mode)
#if BK_DEF(BK_U_ROLLOUT_FR)
__global__ __launch_bounds__(BLOCK, FR_BLOCKS_PER_CU) void k_rollout_fr(RolloutArgs a) { rollout_body<true>(a); }
#else
__global__ void k_rollout_fr(RolloutArgs a);
#endif
// reference frontier order with HeuristicAgent seats (cfg.heuristic_seats)
#if BK_DEF(BK_U_ROLLOUT_FRH)
__global__ __launch_bounds__(HBLOCK, 2) void k_rollout_fr_h(RolloutArgs a) { rollout_body<true, true>(a); }
#else
__global__ void k_rollout_fr_h(RolloutArgs a);
#endif

// ------------------------------------------------------------------------------------
// FastMCTS simulate loop (agents/fast_mcts_agent.py:153-256): one wave per game
// ------------------------------------------------------------------------------------
#define FM_N 624
#define FM_M 397
// bit-exact with CPython floats: no a*b+c fusion anywhere below
#pragma clang fp contract(off)

__device__ __forceinline__ uint32_t mt_y(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// new mt[kk] = mt[kk + off] ^ twist(mt[kk], mt[kk+1]) for kk in [lo, hi), 64 lanes at a
// time; each chunk reads before it writes, and no chunk reads what a later chunk writes
__device__ __forceinline__ void twist_range(uint32_t* mt, int lo, int hi, int off, int lane) {
    for (int k0 = lo; k0 < hi; k0 += WAVE) {
        const int k = k0 + lane;
        uint32_t v = 0;
        if (k < hi) v = mt[k + off] ^ mt_y(mt[k], mt[k + 1]);
        __syncthreads();
        if (k < hi) mt[k] = v;
        __syncthreads();
    }
}

// CPython genrand_uint32's twist (Modules/_randommodule.c), parallel in four phases
__device__ void py_twist(uint32_t* mt, int lane) {
    twist_range(mt, 0, FM_N - FM_M, FM_M, lane);                            // old mt[kk+397]
    twist_range(mt, FM_N - FM_M, 2 * (FM_N - FM_M), FM_M - FM_N, lane);     // new mt[0..227)
    twist_range(mt, 2 * (FM_N - FM_M), FM_N - 1, FM_M - FM_N, lane);        // new mt[227..396)
    if (lane == 0) mt[FM_N - 1] = mt[FM_M - 1] ^ mt_y(mt[FM_N - 1], mt[0]);
    __syncthreads();
}

__device__ __forceinline__ uint32_t py_next(uint32_t* mt, int& idx, int lane) {
    if (idx >= FM_N) { py_twist(mt, lane); idx = 0; }
    uint32_t y = mt[idx++];
    y ^= y >> 11; y ^= (y << 7) & 0x9d2c5680u; y ^= (y << 15) & 0xefc60000u; y ^= y >> 18;
    return y;
}

__device__ __forceinline__ double py_random(uint32_t* mt, int& idx, int lane) {
    const uint32_t a = py_next(mt, idx, lane) >> 5, b = py_next(mt, idx, lane) >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}

// wave argmax of (value, index): larger value wins, ties -> smaller index (a total
// order, so any reduction order gives the same winner).  Inside each 16-lane row on DPP
// (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: ALU latency), then the
// four rows' winners by v_readlane -- where a __shfl_xor ladder is 18 dependent
// ds_bpermute round trips per reduction (FastMCTS runs one per iteration).  All 64 lanes
// active; every lane gets the result.
template <int CTRL>
__device__ __forceinline__ void argmax_dpp_step(double& v, int& j) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)b, (int)(uint32_t)b, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(b >> 32), (int)(uint32_t)(b >> 32), CTRL,
                                                              0xF, 0xF, false);
    const int oj = __builtin_amdgcn_update_dpp(j, j, CTRL, 0xF, 0xF, false);
    const double ov = __longlong_as_double((long long)(((uint64_t)hi << 32) | (uint64_t)lo));
    if (ov > v || (ov == v && oj < j)) { v = ov; j = oj; }
}
__device__ __forceinline__ void wave_argmax(double& v, int& j) {
    argmax_dpp_step<0xB1>(v, j);   // quad_perm [1, 0, 3, 2]
    argmax_dpp_step<0x4E>(v, j);   // quad_perm [2, 3, 0, 1]
    argmax_dpp_step<0x141>(v, j);  // row_half_mirror
    argmax_dpp_step<0x140>(v, j);  // row_mirror
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    double bv = v;
    int bj = j;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 16 * r);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 16 * r);
        const double ov = __longlong_as_double((long long)(((uint64_t)hi << 32) | (uint64_t)lo));
        const int oj = __builtin_amdgcn_readlane(j, 16 * r);
        if (r == 0 || ov > bv || (ov == bv && oj < bj)) { bv = ov; bj = oj; }
    }
    v = bv;
    j = bj;
}

struct PowFix {  // bk_pow_half_fix tables: CPython's (2 log N / v) ** 0.5 vs sqrt
    const int32_t* offsets;
    const int32_t* entries;
    int32_t rows;     // the tables cover N < rows
};

// c * x ** 0.5 with x = L2 / v, L2 = 2 * math.log(N) (fast_mcts_agent.py:52): the IEEE
// sqrt, moved one ulp where glibc's pow (what CPython calls) rounds the other way.  The
// few corrections of this N are scanned by every lane (N is wave-uniform).
__device__ __forceinline__ double fm_explore(double c, double L2, uint32_t v, uint32_t N, const PowFix& fx) {
    double s = sqrt(L2 / (double)v);
    if ((int32_t)N >= fx.rows) return c * s;
    const int32_t e0 = fx.offsets[N], e1 = fx.offsets[N + 1];
    for (int32_t e = e0; e < e1; ++e) {
        const int32_t w = fx.entries[e];
        if ((uint32_t)(w >> 1) == v) {
            const long long bits = __double_as_longlong(s);
            s = __longlong_as_double((w & 1) ? bits + 1 : bits - 1);  // s > 0 here (v < N)
        }
    }
    return c * s;
}

// UCB1 argmax over children [0, nch) (FastMCTSNode.select_child, fast_mcts_agent.py:55):
// the first child with the largest total/visits + explore; one wave
__device__ __forceinline__ int fm_select(const uint32_t* visits, const double* total, int nch, int lane,
                                         double L2, uint32_t N, double c, const PowFix& fx) {
    double best = -1.0 / 0.0;
    int bj = 0x7fffffff;
    for (int j = lane; j < nch; j += WAVE) {
        const uint32_t vi = visits[j];
        const double u = total[j] / (double)vi + fm_explore(c, L2, vi, N, fx);
        if (u > best) { best = u; bj = j; }
    }
    wave_argmax(best, bj);
    return bj;
}

#define FM_LOG_LDS 1024
struct FastMctsArgs {
    int32_t n_games;
    const int32_t* offset;
    const int32_t* iterations;
    const double* base;
    uint32_t* mt_state;
    const double* log_table;
    int32_t log_len;
    PowFix fix;
    double c;
    bk_fastmcts_out* out;
    int32_t* visits_out;  // optional: per legal index, flat by legal_offset
    uint32_t* err;
};

#if BK_DEF(BK_U_FASTMCTS)
__global__ __launch_bounds__(WAVE) void k_fastmcts(FastMctsArgs a) {
    __shared__ uint32_t visits[BK_FASTMCTS_MAX_CHILDREN];
    __shared__ double total[BK_FASTMCTS_MAX_CHILDREN];
    __shared__ uint32_t mt[FM_N];
    __shared__ double ltab[FM_LOG_LDS];  // the log table's first rows: one LDS read per iteration
    const int lane = threadIdx.x;
    const int game = blockIdx.x;
    if (game >= a.n_games) return;
    const int n = a.offset[game + 1] - a.offset[game];
    const int iters = a.iterations[game];
    const int nlt = iters + 1 < a.log_len ? (iters + 1 < FM_LOG_LDS ? iters + 1 : FM_LOG_LDS)
                                          : (a.log_len < FM_LOG_LDS ? a.log_len : FM_LOG_LDS);
    for (int k = lane; k < nlt; k += WAVE) ltab[k] = a.log_table[k];
    const double base = a.base[game];
    uint32_t* st = a.mt_state + (size_t)game * (FM_N + 1);
    for (int k = lane; k < FM_N; k += WAVE) mt[k] = st[k];
    int idx = (int)st[FM_N];
    for (int k = lane; k < n && k < BK_FASTMCTS_MAX_CHILDREN; k += WAVE) { visits[k] = 0; total[k] = 0.0; }
    __syncthreads();
    if (n > BK_FASTMCTS_MAX_CHILDREN || iters >= a.log_len) {
        if (lane == 0) { atomicOr(a.err, 1u); atomicOr(a.err + 1, BK_STICKY_FASTMCTS); }
        return;
    }
    int nch = 0;
    uint32_t root_visits = 0;
    int it = 0;
    if (n <= 2 * WAVE) {
        // Roots of <= 128 children (all of config 4's): child j's visits / total live in
        // lane j % 64's registers (slot j / 64), so an iteration is the UCB terms, the DPP
        // argmax and one register update by the child's lane -- no LDS round trip or
        // barrier.  The rewards do not depend on the selection: base + random() * 0.1 of
        // the stream's next two words each iteration, so they are drawn up to a twist ahead,
        // one per lane (fm_rew), and the generator's position is set back to what the
        // iterations actually consumed.
        __shared__ double fm_rew[FM_N / 2];
        const bool draw = base == base;  // NaN base: reward 0.0 and no draw (fast_mcts_agent.py:255-257)
        uint32_t v0 = 0u, v1 = 0u;
        double t0 = 0.0, t1 = 0.0;
        int rptr = 0, ravail = 0, ridx = idx;  // fm_rew[rptr..ravail) drawn from word ridx on
        for (; it < iters; ++it) {
            int sel;
            if (nch < n) {
                sel = nch++;  // expand: untried_moves.pop() -> child nch <-> legal[n - 1 - nch]
            } else {
                const double lg = (int)root_visits < nlt ? ltab[root_visits] : a.log_table[root_visits];
                const double L2 = 2.0 * lg;
                double best = -1.0 / 0.0;
                int bj = 0x7fffffff;
                if (lane < nch) { best = t0 / (double)v0 + fm_explore(a.c, L2, v0, root_visits, a.fix); bj = lane; }
                if (lane + WAVE < nch) {
                    const double u = t1 / (double)v1 + fm_explore(a.c, L2, v1, root_visits, a.fix);
                    if (u > best) { best = u; bj = lane + WAVE; }
                }
                wave_argmax(best, bj);
                sel = bj;
            }
            double reward = 0.0;
            if (draw) {
                if (rptr == ravail) {  // the next draws (py_random's order, lazy twist)
                    idx = ridx;
                    if (idx >= FM_N) { py_twist(mt, lane); idx = 0; }
                    const int m = (FM_N - idx) / 2;
                    __syncthreads();
                    if (m == 0) {  // one word left: this draw straddles the twist
                        const double r = py_random(mt, idx, lane);
                        if (lane == 0) fm_rew[0] = base + r * 0.1;
                        ravail = 1;
                    } else {
                        for (int l = lane; l < m; l += WAVE) {
                            uint32_t x = mt[idx + 2 * l], y = mt[idx + 2 * l + 1];
                            x ^= x >> 11; x ^= (x << 7) & 0x9d2c5680u; x ^= (x << 15) & 0xefc60000u; x ^= x >> 18;
                            y ^= y >> 11; y ^= (y << 7) & 0x9d2c5680u; y ^= (y << 15) & 0xefc60000u; y ^= y >> 18;
                            const double r = ((double)(x >> 5) * 67108864.0 + (double)(y >> 6)) *
                                             (1.0 / 9007199254740992.0);
                            fm_rew[l] = base + r * 0.1;
                        }
                        ravail = m;
                        idx += 2 * m;
                    }
                    ridx = idx;
                    rptr = 0;
                    __syncthreads();
                }
                reward = fm_rew[rptr++];
            }
            if (lane == (sel & (WAVE - 1))) {
                if (sel < WAVE) { v0 += 1u; t0 += reward; }
                else { v1 += 1u; t1 += reward; }
            }
            root_visits += 1u;
        }
        // the words the iterations consumed: the generator stops there (unused draws are
        // not taken)
        if (draw) idx = ridx - 2 * (ravail - rptr);  // (a straddling draw is always consumed)
        if (lane < n) { visits[lane] = v0; total[lane] = t0; }
        if (lane + WAVE < n) { visits[lane + WAVE] = v1; total[lane + WAVE] = t1; }
        __syncthreads();
    } else {
        for (; it < iters; ++it) {
            int sel;
            if (nch < n) {
                sel = nch++;  // expand: untried_moves.pop() -> child nch <-> legal[n - 1 - nch]
            } else {
                const double lg = (int)root_visits < nlt ? ltab[root_visits] : a.log_table[root_visits];
                sel = fm_select(visits, total, nch, lane, 2.0 * lg, root_visits, a.c, a.fix);
            }
            // NaN base: the cached legal list was empty -> reward 0.0 and no draw
            // (fast_mcts_agent.py:255-257)
            const double reward = (base == base) ? base + py_random(mt, idx, lane) * 0.1 : 0.0;
            if (lane == 0) {
                visits[sel] += 1u;
                total[sel] += reward;
            }
            __syncthreads();
            root_visits += 1u;
        }
    }
    if (a.visits_out) {
        int32_t* vo = a.visits_out + a.offset[game];
        for (int k = lane; k < n; k += WAVE) vo[k] = (n - 1 - k < nch) ? (int32_t)visits[n - 1 - k] : 0;
    }
    // hand the advanced generator state back (random.setstate on the host)
    for (int k = lane; k < FM_N; k += WAVE) st[k] = mt[k];
    if (lane == 0) st[FM_N] = (uint32_t)idx;
    // results
    bk_fastmcts_out* o = a.out + game;
    if (lane == 0) { o->iterations = it; o->n_children = nch; }
    // best = most visited child, first on ties
    {
        double bv = -1.0;
        int bj = 0x7fffffff;
        for (int j = lane; j < nch; j += WAVE)
            if ((double)visits[j] > bv) { bv = (double)visits[j]; bj = j; }
        wave_argmax(bv, bj);
        if (lane == 0) o->best_index = nch > 0 ? n - 1 - bj : 0;
    }
    // top moves: stable sort by visits desc (selection, marking picked children)
    int ntop = 0;
    for (int t = 0; t < BK_FASTMCTS_TOP && t < nch; ++t) {
        double bv = -1.0;
        int bj = 0x7fffffff;
        for (int j = lane; j < nch; j += WAVE)
            if (!(visits[j] & 0x80000000u) && (double)visits[j] > bv) { bv = (double)visits[j]; bj = j; }
        wave_argmax(bv, bj);
        if (lane == 0) {
            const uint32_t v = visits[bj];
            o->top_index[t] = n - 1 - bj;
            o->top_visits[t] = (int32_t)v;
            o->top_q[t] = total[bj] / (double)v;
            visits[bj] = v | 0x80000000u;
        }
        __syncthreads();
        ++ntop;
    }
    if (lane == 0) o->n_top = ntop;
}
#else
__global__ void k_fastmcts(FastMctsArgs a);
#endif

// bk_debug_fastmcts_select: one selection step of k_fastmcts on given child stats
#if BK_DEF(BK_U_FASTMCTS)
__global__ __launch_bounds__(WAVE) void k_fastmcts_select(const uint32_t* visits, const double* totals, int n,
                                                          uint32_t N, double L2, double c, PowFix fx, int32_t* out) {
    const int j = fm_select(visits, totals, n, threadIdx.x, L2, N, c, fx);
    if (threadIdx.x == 0) *out = j;
}
#else
__global__ void k_fastmcts_select(const uint32_t* visits, const double* totals, int n, uint32_t N, double L2, double c,
                                  PowFix fx, int32_t* out);
#endif

// ------------------------------------------------------------------------------------
// MCTSAgent searches (mcts/mcts_agent.py:19-582) with RandomAgent rollouts: one lane =
// one game's whole search.  The UCT tree lives in a per-game node pool in HBM, the
// Zobrist TT is a per-game open-addressing table in HBM, the rollout stream is the
// agent's numpy MT19937.  A node stores no board: the selected leaf's board is replayed
// from the root along the tree path with the reference's copy/place/copy sequence
// (frontier-set layouts, hence list orders, depend on it).  Every kernel step runs ONE
// movegen for each busy lane -- the expansion of its selected leaf or one rollout ply --
// and the divergent tree work (selection, replay, TT, backpropagation) in between.
// ------------------------------------------------------------------------------------
#define MC_FATAL(st) ((st) & ~BK_MCTS_EUNCERT)  // status bits that end a search
#define MC_SELECT 0
#define MC_EXPAND 1
#define MC_ROLLOUT 2
#define MC_PATH (BK_MCTS_MAX_DEPTH + 1)
#define MC_ZOB 2088
#define MC_TREE_BATCH WAVE

struct McLane {          // per-lane scratch record in HBM
    FsLane A;            // node.board tables of the node being worked on; the rollout's sim board
    bk_fset root;        // root.board (= board.copy(), made once per search)
    int32_t path[MC_PATH];
};
static_assert(sizeof(FsLane) % 16 == 0 && sizeof(bk_fset) % 16 == 0, "McLane tables are read as uint4");

struct MctsArgs {
    const bk_state* roots;
    const bk_fset* root_sets;
    const uint8_t* players;
    const uint64_t* root_hash;
    int32_t n_games;
    bk_mcts_cfg cfg;
    const uint64_t* zobrist;
    const int32_t* zidx;
    uint32_t* mt;
    uint64_t* tt_keys;
    double* tt_vals;
    int32_t* tt_count;
    const double* log_table;
    int32_t log_len;
    bk_mcts_node* nodes;
    double* rewards;
    uint8_t* hit_flags;
    bk_mcts_out* out;
    uint32_t* slab;
    McLane* lanes;
    uint32_t* counter;  // [0] next game, [1] step guard tripped
    uint64_t max_steps;
    uint64_t limit_ticks;  // cfg.time_limit_us in wall-clock (s_memrealtime) ticks
    int32_t tree_batch;    // tree phase once this many lanes of a wave wait for it (or no lane is busy)
    int32_t spread;        // only lanes with lane % spread == 0 take searches (more waves, fewer lanes each)
    int32_t coop_walk;     // k_mcts_coop(_h): frontier walk split over the wave (coop_walk), else serial
    int32_t coop_balanced; // k_mcts_coop_h: balanced HeuristicAgent pass (coop_heur_balanced), else per lane
    uint32_t* diag;        // the handle's failure record (BK_DIAG_WORDS; mc_diag), sticky until read
    uint32_t launch_seq;   // this launch's number on the handle (recorded in a failure record)
    uint32_t kernel_id;    // BK_DIAG_K_*: which search kernel runs (recorded in a failure record)
    uint32_t* started;     // one bit per search of the launch, set when a wave starts it (mc_mark_started)
    // BK_MCTS_STATE_ROWS: search g's agent state is row zidx[g] of mt_rows / tt_* (the
    // agent's own rows): the MT state is copied into mt[g] (the handle's scratch) at the
    // search's start and back at its end, the TT is probed and filled in place -- all
    // with system-scope loads and stores, which bypass the XCDs' L2s, so a search that
    // starts while an earlier launch still runs (on another XCD) sees the agent's rows as
    // that launch's finished search left them, with no L2 writeback
    int32_t state_rows;
    uint32_t* mt_rows;
    // bk_mcts_set_done: done[g] = the search's result word (mc_done_word) once its agent
    // rows are written back (bit 63 set; one 64-bit store to mapped host memory)
    uint64_t* done;
};

struct Mc {
    int32_t game;       // -1 = none
    int32_t it;         // iterations done
    int32_t mode;
    int32_t depth;      // path[depth] = node being expanded / simulated
    int32_t node;
    int32_t nodes_used, tt_cnt, hits, rollouts, rplies;
    int32_t root_player, root_cp;
    int32_t cur, player, plies, score0;
    uint32_t status, mt_pos, first, tt_slot;
    int32_t row;        // the search's MT / TT row (g, or zidx[g] with BK_MCTS_STATE_ROWS)
    bool tt_miss;
    Quad used, cells;
    uint64_t hash, t0;
};

__device__ __forceinline__ uint32_t mc_temper(uint32_t y) {
    y ^= y >> 11; y ^= (y << 7) & 0x9d2c5680u; y ^= (y << 15) & 0xefc60000u; y ^= y >> 18;
    return y;
}

// numpy mt19937_gen in place, 16 words per batch of loads (a batch only reads words an
// earlier batch wrote, or old words no batch has written yet)
__device__ void mc_twist(uint32_t* st) {
#pragma unroll 1
    for (int i0 = 0; i0 < FM_N; i0 += 16) {
        uint32_t x[16], y[16], z[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = i0 + j;
            x[j] = st[i];
            y[j] = st[i == FM_N - 1 ? 0 : i + 1];
            z[j] = st[i < FM_N - FM_M ? i + FM_M : i - (FM_N - FM_M)];
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) st[i0 + j] = z[j] ^ mt_y(x[j], y[j]);
    }
}

// RandomState.randint(0, n): masked rejection over 32-bit outputs; n == 1 draws nothing
__device__ __forceinline__ uint32_t mc_randint(uint32_t* st, uint32_t& pos, uint32_t n) {
    const uint32_t rng = n - 1u;
    if (rng == 0u) return 0u;
    const uint32_t mask = mask_for(rng);
    uint32_t v;
    do {
        if (pos >= FM_N) { mc_twist(st); pos = 0; }
        v = mc_temper(st[pos++]) & mask;
    } while (v > rng);
    return v;
}

__device__ __forceinline__ int mc_score(const Mc& m, int p) {  // Board.get_score, engine/board.py:562
    return (int)m.cells.get(p) + ((m.used.get(p) == 0x1FFFFFu) ? 15 : 0);
}

__device__ __forceinline__ bool mc_copy_tables(bk_fset* d, const bk_fset* s, const uint64_t* htab) {
    bool ok = true;
#pragma unroll 1
    for (int q = 0; q < 4; ++q) ok &= fs_copy_dev(d, q, s, htab);
    return ok;
}

// The placed piece's row masks (pm[d] = cells in row ar + d) and cell indices.
__device__ __forceinline__ void piece_cells(int gs, int ar, int ac, uint32_t (&pm)[5], int32_t (&cells)[5]) {
    const int n = (int)((kInfo[gs] >> 8) & 0xFFu);
#pragma unroll
    for (int d = 0; d < 5; ++d) pm[d] = 0u;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const uint32_t cell = kCells[gs][q < n ? q : 0];
        const int dr = (int)(cell >> 8), c = ac + (int)(cell & 0xFFu);
        cells[q] = (ar + dr) * 20 + c;
        const uint32_t bit = q < n ? (1u << c) : 0u;
#pragma unroll
        for (int d = 0; d < 5; ++d) pm[d] |= (dr == d) ? bit : 0u;
    }
}

// mc_place with the frontier update on the LDS-staged table (place_frontier).  pm /
// cells from piece_cells, real from frontier_ops -- computed by EVERY lane of the wave
// before any lane stages a table: the staged tables of some lanes overlay the LDS rows
// of others.
// RECOPY: the table then becomes its Board.copy() in place (expansion and replay edges:
// node boards are copies).
// stage_q (k_mcts_pair): the mover's table is already in the LDS-DMA stage at stage_q.
template <bool RECOPY, int RUN_U4 = DMA_RUN_DWORDS / 4, typename Mark = NoMark>
__device__ __forceinline__ bool mc_place_staged(Mc& m, const Slab& slab, int p, int gs, int ar, FsLane* T,
                                                const uint64_t* htab, const uint32_t (&pm)[5],
                                                const int32_t (&cells)[5], uint64_t real, int16_t* lk,
                                                int16_t* stage_q = nullptr, Mark mark = Mark(), bool inplace = false) {
    const uint32_t info = kInfo[gs];
    const int n = (int)((info >> 8) & 0xFFu);
    {  // every row load issued before any store (one memory latency, not one per row)
        uint32_t ow[5], oc[5];
#pragma unroll
        for (int d = 0; d < 5; ++d) {
            ow[d] = pm[d] ? slab.at(p, ar + d) : 0u;
            oc[d] = pm[d] ? slab.at(4, ar + d) : 0u;
        }
#pragma unroll
        for (int d = 0; d < 5; ++d) {
            if (pm[d]) {
                slab.at(p, ar + d) = ow[d] | pm[d];
                slab.at(4, ar + d) = oc[d] | pm[d];
            }
        }
    }
    mark(4);
    // (k_mcts_pair's DMA stage leaves this lane's LDS column free for the resize scratch;
    // the 128-slot stage in the column itself does not.  The cooperative kernels, RUN_U4
    // 2, resize through the record's tmp: the scratch measured 1-2 % slower there,
    // profiles/r05/sweeps/r05u)
    const bool ok = stage_q ? place_frontier_dma<RECOPY, RUN_U4>(T, p, stage_q, htab, cells, real, mark,
                                                                 RUN_U4 == 2 ? nullptr : lk, inplace)
                            : place_frontier<BK_FS_STAGE_MCTS, RECOPY>(T, p, lk, htab, cells, real);
    m.cells.set(p, m.cells.get(p) + (uint32_t)n);
    m.used.set(p, m.used.get(p) | (1u << ((info & 0xFFu) - 1u)));
    m.first &= ~(1u << p);
    return ok;
}

// Zobrist update for that placement (mcts/zobrist.py:70-99 terms that change)
__device__ __forceinline__ uint64_t mc_hash_step(const uint64_t* Z, uint64_t h, int p, int cp, int gs, int ar, int ac) {
    const uint32_t info = kInfo[gs];
    const int n = (int)((info >> 8) & 0xFFu);
    h ^= Z[2000 + cp] ^ Z[2000 + ((cp + 1) & 3)];
    for (int q = 0; q < n; ++q) {
        const uint32_t cell = kCells[gs][q];
        const int ci = (ar + (int)(cell >> 8)) * 20 + ac + (int)(cell & 0xFFu);
        h ^= Z[ci * 5] ^ Z[ci * 5 + p + 1];
    }
    return h ^ Z[2004 + p * 21 + (int)(info & 0xFFu) - 1];
}

__device__ __forceinline__ void mc_move_split(uint32_t mv, int& gs, int& ar, int& ac) {
    gs = (int)(mv / 400u);
    const int cell = (int)(mv % 400u);
    ar = cell / 20;
    ac = cell - 20 * ar;
}

// Failure record of a search whose tree breaks an invariant: a node
// visited more often than the log table allows (BK_MCTS_ELOG: a correct search of I
// iterations has every node's visits <= I < log_len), or a root whose visits differ from
// the iterations run (BK_MCTS_EINTERNAL: every iteration backpropagates through the root,
// mcts_agent.py:572-582).  Either means the search's node pool was written by something
// other than this search.  The first failing search of a launch writes what it saw into
// the handle's sticky buffer (atomicCAS on word 0; the cooperative kernels' 64 redundant
// lanes race for it and one wins); bk_synchronize reports it as BK_ECHECK and
// bk_debug_mcts_failure returns it.  Costs nothing unless it fires.  Words (BK_DIAG_*):
// 0 reason (BK_MCTS_ELOG / EINTERNAL), 1 kernel, 2 launch number on the handle, 3 the
// search's game index in the launch, 4 node, 5 node visits, 6 n_exp, 7 n_legal, 8 child0,
// 9 iterations done, 10 depth, 11 log_len, 12 the game hand-out counter when it fired,
// 13 node_cap, 14 nodes_used, 15 cfg.iterations, 16 path length recorded, 17 the
// search's first-touch wall clock (low word), 18..39 the path's nodes from the root,
// 40..61 their visits.
__device__ __forceinline__ void mc_diag(const MctsArgs& a, const Mc& m, const int32_t* path, int depth, uint32_t why,
                                     int32_t node, const bk_mcts_node& nd) {
    if (!a.diag || atomicCAS(&a.diag[0], 0u, why) != 0u) return;
    uint32_t* d = a.diag;
    const bk_mcts_node* pool = a.nodes + (size_t)m.game * a.cfg.node_cap;
    d[1] = a.kernel_id;
    d[2] = a.launch_seq;
    d[3] = (uint32_t)m.game;
    d[4] = (uint32_t)node;
    d[5] = nd.visits;
    d[6] = nd.n_exp;
    d[7] = nd.n_legal;
    d[8] = (uint32_t)nd.child0;
    d[9] = (uint32_t)m.it;
    d[10] = (uint32_t)depth;
    d[11] = (uint32_t)a.log_len;
    d[12] = __hip_atomic_load(&a.counter[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    d[13] = (uint32_t)a.cfg.node_cap;
    d[14] = (uint32_t)m.nodes_used;
    d[15] = (uint32_t)a.cfg.iterations;
    const int np = path ? (depth + 1 < 22 ? depth + 1 : 22) : 0;
    d[16] = (uint32_t)np;
    d[17] = (uint32_t)m.t0;
    for (int k = 0; k < np; ++k) {
        d[18 + k] = (uint32_t)path[k];
        d[40 + k] = pool[path[k]].visits;
    }
    __threadfence();
}

// root.board into the lane: rows from the state, tables = the search's root copy
__device__ __forceinline__ void mc_load_root(const MctsArgs& a, Mc& m, const Slab& slab, McLane* L) {
    const bk_state* s = a.roots + m.game;
    uint32_t occ[20];
#pragma unroll
    for (int R = 0; R < 20; ++R) occ[R] = 0;
#pragma unroll 1
    for (int p = 0; p < 4; ++p) {
        uint32_t cells = 0;
        uint64_t w[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) w[k] = s->planes[p][k];
#pragma unroll
        for (int R = 0; R < 20; ++R) {
            const uint32_t row = plane_row(w, R);
            slab.at(p, R) = row;
            occ[R] |= row;
            cells += __builtin_popcount(row);
        }
        m.cells.set(p, cells);
        m.used.set(p, s->used[p] & 0x1FFFFFu);
    }
#pragma unroll
    for (int R = 0; R < 20; ++R) slab.at(4, R) = occ[R];
    m.first = s->first_move & 0xFu;
    copy_fset(&L->A.s, &L->root);
}

// A search is started exactly once per launch.  The launch's bitmap takes one atomicOr
// per start (one lane per search); a bit already set means two waves / lanes were handed
// the same search, which would interleave two searches over one node pool: the second
// start writes a failure record (BK_DIAG_DOUBLE_START, with both hand-out values it can
// see) and the caller stops that search with BK_MCTS_EINTERNAL.
__device__ __forceinline__ bool mc_mark_started(const MctsArgs& a, int32_t g, uint32_t handed) {
    if (!a.started) return false;
    const uint32_t old = atomicOr(&a.started[(uint32_t)g >> 5], 1u << ((uint32_t)g & 31u));
    if (!((old >> ((uint32_t)g & 31u)) & 1u)) return false;
    if (a.diag && atomicCAS(&a.diag[0], 0u, BK_DIAG_DOUBLE_START) == 0u) {
        uint32_t* d = a.diag;
        d[1] = a.kernel_id;
        d[2] = a.launch_seq;
        d[3] = (uint32_t)g;
        d[12] = __hip_atomic_load(&a.counter[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        d[17] = handed;
        d[18] = (uint32_t)blockIdx.x;
        d[19] = (uint32_t)(threadIdx.x / WAVE);
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        d[20] = hw;
        d[21] = (uint32_t)a.n_games;
        __threadfence();
    }
    return true;
}

// System-scope (L2-bypassing) accesses of the agent rows under BK_MCTS_STATE_ROWS
template <typename T>
__device__ __forceinline__ T sys_ld(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ void sys_st(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t tt_key_ld(const MctsArgs& a, const uint64_t* p) {
    return a.state_rows ? sys_ld(p) : *p;
}
__device__ __forceinline__ double tt_val_ld(const MctsArgs& a, const double* p) {
    return a.state_rows ? __longlong_as_double((long long)sys_ld(reinterpret_cast<const uint64_t*>(p))) : *p;
}

// lane / nl: the lanes sharing the search (the cooperative kernels: 0..63 of 64), which
// split the agent row copies
__device__ __forceinline__ void mc_start_game(const MctsArgs& a, Mc& m, McLane* L, int32_t g, const uint64_t* htab,
                                              int lane = 0, int nl = 1) {
    m.game = g;
    m.mode = MC_SELECT;
    m.row = a.state_rows ? a.zidx[g] : g;
    if (a.state_rows) {  // the agent's MT state into the search's working copy
        const uint32_t* src = a.mt_rows + (size_t)m.row * (FM_N + 1);
        uint32_t* dst = a.mt + (size_t)g * (FM_N + 1);
        for (int i0 = lane; i0 < FM_N + 1; i0 += 8 * nl) {  // 8 loads in flight per lane
            uint32_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = i0 + j * nl < FM_N + 1 ? sys_ld(src + i0 + j * nl) : 0u;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (i0 + j * nl < FM_N + 1) dst[i0 + j * nl] = v[j];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the other lanes' copies are visible
        m.tt_cnt = a.cfg.use_tt ? sys_ld(a.tt_count + m.row) : 0;
    } else {
        m.tt_cnt = a.cfg.use_tt ? a.tt_count[g] : 0;
    }
    m.root_player = a.players[g] & 3;
    m.root_cp = a.roots[g].current_player & 3;
    m.mt_pos = a.mt[(size_t)g * (FM_N + 1) + FM_N];
    m.t0 = wall_clock64();
    if (a.cfg.resume) {  // a chunked search: carry on where the previous launch stopped
        const bk_mcts_out o = a.out[g];
        m.it = o.iterations_run;
        m.nodes_used = o.nodes_used;
        m.hits = o.tt_hits;
        m.rollouts = o.rollouts;
        m.rplies = o.rollout_plies;
        m.status = o.status;
    } else {
        m.it = 0;
        m.nodes_used = 1;
        m.hits = m.rollouts = m.rplies = 0;
        m.status = 0;
        bk_mcts_node* root = a.nodes + (size_t)g * a.cfg.node_cap;
        root->total = 0.0; root->visits = 0; root->child0 = -1;
        root->move = 0xFFFFu; root->n_exp = 0; root->n_legal = 0; root->flags = 0;
    }
    if (!mc_copy_tables(&L->root, a.root_sets + g, htab)) m.status |= BK_MCTS_EFSET;  // MCTSNode: board.copy()
}

// Slot for the next child of node nd (n_legal known, n_exp < n_legal).  The children
// block holds min(n_legal, 4) slots at the first expansion and moves to a block twice
// as large (capped at n_legal) whenever it is full, so a search of I iterations uses at
// most 4 * I + 1 slots.  Children keep their expansion order; nothing points into a
// block but its parent's child0 (paths are rebuilt from the root by every selection).
// -1: the pool is full.
__device__ __forceinline__ int32_t mc_child_slot(bk_mcts_node* pool, bk_mcts_node* nd, Mc& m, int32_t node_cap) {
    const uint32_t ne = nd->n_exp, nl = nd->n_legal;
    const bool grow = ne == 0u || (ne >= 4u && (ne & (ne - 1u)) == 0u);
    if (grow) {
        const uint32_t want = ne == 0u ? 4u : 2u * ne;
        const uint32_t ncap = want < nl ? want : nl;
        if ((uint64_t)m.nodes_used + ncap > (uint64_t)node_cap) return -1;
        const int32_t nb = m.nodes_used;
        m.nodes_used += (int32_t)ncap;
        const int32_t ob = nd->child0;
#pragma unroll 1
        for (uint32_t k = 0; k < ne; ++k) pool[nb + k] = pool[ob + k];
        nd->child0 = nb;
    }
    return nd->child0 + (int32_t)ne;
}

// the host's per-search result word (bk_mcts_set_done): best_move in bits 0..31,
// iterations_run in 32..55, status in 56..62, bit 63 set
__device__ __forceinline__ uint64_t mc_done_word(const bk_mcts_out& o) {
    return (uint64_t)(uint32_t)o.best_move | ((uint64_t)((uint32_t)o.iterations_run & 0xFFFFFFu) << 32) |
           ((uint64_t)(o.status & 0x7Fu) << 56) | (1ull << 63);
}

__device__ __forceinline__ void mc_finish_game(const MctsArgs& a, Mc& m, int lane = 0, int nl = 1) {
    const int32_t g = m.game;
    const bk_mcts_node* pool = a.nodes + (size_t)g * a.cfg.node_cap;
    const bk_mcts_node root = pool[0];
    if (root.visits != (uint32_t)m.it && !MC_FATAL(m.status)) {  // every iteration went through the root
        m.status |= BK_MCTS_EINTERNAL;
        mc_diag(a, m, nullptr, 0, BK_MCTS_EINTERNAL, 0, root);
    }
    int32_t best = -1;
    uint32_t bv = 0;
    for (int k = 0; k < (int)root.n_exp; ++k) {  // get_best_move: max visits, first on ties
        const bk_mcts_node c = pool[root.child0 + k];
        if (best < 0 || c.visits > bv) { bv = c.visits; best = c.move; }
    }
    bk_mcts_out o;
    o.best_move = best;
    o.iterations_run = m.it;
    o.tt_hits = m.hits;
    o.rollouts = m.rollouts;
    o.nodes_used = m.nodes_used;
    o.root_children = root.n_exp;
    o.status = m.status;
    o.rollout_plies = m.rplies;
    a.out[g] = o;
    if (a.state_rows) {  // the working MT state back into the agent's row, write-through
        uint32_t* mt = a.mt + (size_t)g * (FM_N + 1);
        if (lane == 0) mt[FM_N] = m.mt_pos;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        uint32_t* dst = a.mt_rows + (size_t)m.row * (FM_N + 1);
        for (int i0 = lane; i0 < FM_N + 1; i0 += 8 * nl) {
            uint32_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = i0 + j * nl < FM_N + 1 ? mt[i0 + j * nl] : 0u;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (i0 + j * nl < FM_N + 1) sys_st(dst + i0 + j * nl, v[j]);
        }
        if (a.cfg.use_tt) sys_st(a.tt_count + m.row, (int32_t)m.tt_cnt);
    } else {
        a.mt[(size_t)g * (FM_N + 1) + FM_N] = m.mt_pos;
        if (a.cfg.use_tt) a.tt_count[g] = m.tt_cnt;
    }
    if (a.done) {  // after every store above (and the TT's) has completed: the wave's vmcnt
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sys_st(a.done + g, mc_done_word(o));
    }
    m.game = -1;
}

// TT probe for m.hash: hit -> reward; miss -> remembers the free slot for the insert
__device__ __forceinline__ bool mc_tt_lookup(const MctsArgs& a, Mc& m, double& reward) {
    const uint64_t mask = (uint64_t)a.cfg.tt_cap - 1u;
    const uint64_t* keys = a.tt_keys + (size_t)m.row * a.cfg.tt_cap;
    const double* vals = a.tt_vals + (size_t)m.row * a.cfg.tt_cap;
    uint64_t i = m.hash & mask;
    for (;;) {
        const double v = tt_val_ld(a, vals + i);
        if (v != v) break;
        if (tt_key_ld(a, keys + i) == m.hash) { reward = v; return true; }
        i = (i + 1) & mask;
    }
    m.tt_slot = (uint32_t)i;
    return false;
}

// simulation result: TT insert on a miss, stats, backpropagation (mcts_agent.py:408-437,
// :572-582), next iteration
__device__ __forceinline__ void mc_complete(const MctsArgs& a, Mc& m, McLane* L, double reward, bool hit) {
    if (hit) {
        m.hits++;
    } else {
        m.rollouts++;
        if (a.cfg.use_tt) {
            if ((uint32_t)m.tt_cnt + 2u > (uint32_t)a.cfg.tt_cap) {
                m.status |= BK_MCTS_ETT;
            } else {
                uint64_t* kp = a.tt_keys + (size_t)m.row * a.cfg.tt_cap + m.tt_slot;
                double* vp = a.tt_vals + (size_t)m.row * a.cfg.tt_cap + m.tt_slot;
                if (a.state_rows) {
                    sys_st(kp, m.hash);
                    sys_st(reinterpret_cast<uint64_t*>(vp), (uint64_t)__double_as_longlong(reward));
                } else {
                    *kp = m.hash;
                    *vp = reward;
                }
                m.tt_cnt++;
            }
        }
    }
    if (a.rewards) {
        a.rewards[(size_t)m.game * a.cfg.iterations + m.it] = reward;
        a.hit_flags[(size_t)m.game * a.cfg.iterations + m.it] = hit ? 1u : 0u;
    }
    bk_mcts_node* pool = a.nodes + (size_t)m.game * a.cfg.node_cap;
    for (int d = 0; d <= m.depth; ++d) {
        bk_mcts_node* v = pool + L->path[d];
        v->visits += 1u;
        v->total += reward;
    }
    m.it++;
    m.mode = MC_SELECT;
}

// simulate the node in m.node / m.hash whose player has no legal move: the rollout
// breaks at once (reward 0.0, no draw)
__device__ __forceinline__ void mc_sim_terminal(const MctsArgs& a, Mc& m, McLane* L) {
    double reward = 0.0;
    bool hit = false;
    if (a.cfg.use_tt) hit = mc_tt_lookup(a, m, reward);
    if (!hit) reward = 0.0;
    mc_complete(a, m, L, reward, hit);
}

// best_child (mcts_agent.py:68-111): index of the first child with the largest UCB1
// total/visits + c * sqrt(log(parent visits) / visits) (unvisited: inf) among the n
// children at cb.  The (total, visits) pairs are loaded MC_UCB_BATCH children at a time
// before any is used, so a scan waits on ~n / MC_UCB_BATCH memory round trips instead of
// two dependent loads per child (a fully expanded root has hundreds of children, and a
// lane's child block is not cache-resident).  Same operations, same order: the argmax is
// the reference's.
#define MC_UCB_BATCH 16
__device__ __forceinline__ int mc_ucb_best(const bk_mcts_node* cb, int n, double lg, double c_explore) {
    int best = 0;
    double bv = 0.0;
#pragma unroll 1
    for (int k0 = 0; k0 < n; k0 += MC_UCB_BATCH) {
        double tot[MC_UCB_BATCH];
        uint32_t vis[MC_UCB_BATCH];
#pragma unroll
        for (int j = 0; j < MC_UCB_BATCH; ++j) {
            const int k = k0 + j < n ? k0 + j : n - 1;  // in bounds; unused past n
            tot[j] = cb[k].total;
            vis[j] = cb[k].visits;
        }
#pragma unroll
        for (int j = 0; j < MC_UCB_BATCH; ++j) {
            if (k0 + j < n) {
                double v;
                if (vis[j] == 0u) {
                    v = __builtin_inf();
                } else {
                    const double vd = (double)vis[j];
                    const double exploit = tot[j] / vd;
                    const double explore = c_explore * __builtin_sqrt(lg / vd);
                    v = exploit + explore;
                }
                if (k0 + j == 0 || v > bv) { bv = v; best = k0 + j; }
            }
        }
    }
    return best;
}

// selection (mcts_agent.py:384-406, UCB1 :68-111) from the root; leaves m.node at the
// node to expand or simulate, m.depth / path / m.hash for it.  Returns true when that
// node is evaluated terminal (no untried move, no child).
__device__ __forceinline__ bool mc_select(const MctsArgs& a, Mc& m, McLane* L, const uint64_t* Z) {
    const bk_mcts_node* pool = a.nodes + (size_t)m.game * a.cfg.node_cap;
    int u = 0, depth = 0;
    uint64_t h = a.root_hash[m.game];
    L->path[0] = 0;
    for (;;) {
        const bk_mcts_node nd = pool[u];
        if (!(nd.flags & BK_MCTS_NODE_EVALUATED) || nd.n_legal > nd.n_exp) break;  // expand it
        if (nd.n_exp == 0) { m.node = u; m.depth = depth; m.hash = h; return true; }
        if ((int32_t)nd.visits >= a.log_len) {
            m.status |= BK_MCTS_ELOG;
            mc_diag(a, m, L->path, depth, BK_MCTS_ELOG, u, nd);
            break;
        }
        if (depth >= BK_MCTS_MAX_DEPTH) { m.status |= BK_MCTS_EPATH; break; }
        const double lg = a.log_table[nd.visits];
        const int best = nd.child0 + mc_ucb_best(pool + nd.child0, (int)nd.n_exp, lg, a.cfg.exploration);
        int gs, ar, ac;
        mc_move_split(pool[best].move, gs, ar, ac);
        h = mc_hash_step(Z, h, (m.root_player + depth) & 3, (m.root_cp + depth) & 3, gs, ar, ac);
        u = best;
        L->path[++depth] = u;
    }
    m.node = u;
    m.depth = depth;
    m.hash = h;
    return false;
}

// node.board of path[depth] into the lane (slab rows + table A): root, then per edge
// new_board = board.copy(); place; MCTSNode(new_board) copies again (mcts_agent.py:113-145).
// Every node board is a copy, and a copy of a copy is slot-for-slot the same table
// (set_merge's same-size path), so the first copy is skipped and the second only
// changes the mover's table: place on A (the ops that change the set, frontier_ops from
// the slab, on the LDS-staged table) and replace that table by its copy in place.  lk:
// this lane's LDS column (free in the tree phase: every lane of the wave is at the same
// point of this loop, and the rows of a step are rebuilt after it).
__device__ __forceinline__ void mc_replay(const MctsArgs& a, Mc& m, const Slab& slab, McLane* L, const uint64_t* htab,
                                          int16_t* lk) {
    mc_load_root(a, m, slab, L);
    const bk_mcts_node* pool = a.nodes + (size_t)m.game * a.cfg.node_cap;
    bool ok = true;
    for (int d = 1; d <= m.depth; ++d) {
        int gs, ar, ac;
        mc_move_split(pool[L->path[d]].move, gs, ar, ac);
        const int p = (m.root_player + d - 1) & 3;
        uint32_t pm[5];
        int32_t cells[5];
        piece_cells(gs, ar, ac, pm, cells);
        const uint64_t real = frontier_ops<true>(nullptr, slab, p, (m.first >> p) & 1u, gs, ar, ac, pm);
        ok &= mc_place_staged<true>(m, slab, p, gs, ar, &L->A, htab, pm, cells, real, lk);
    }
    if (!ok) m.status |= BK_MCTS_EFSET;
}

// numpy RandomState.random_sample() (genrand_res53) from a per-game stream
__device__ __forceinline__ double mc_random_sample(uint32_t* st, uint32_t& pos) {
    if (pos >= FM_N) { mc_twist(st); pos = 0; }
    const uint32_t a0 = mc_temper(st[pos++]);
    if (pos >= FM_N) { mc_twist(st); pos = 0; }
    const uint32_t a1 = mc_temper(st[pos++]);
    return ((double)(a0 >> 5) * 67108864.0 + (double)(a1 >> 6)) * (1.0 / 9007199254740992.0);
}

// HEUR: rollouts play HeuristicAgent (MCTSAgent's default rollout_agent,
// mcts/mcts_agent.py:275-281) instead of RandomAgent
// PAIR (k_mcts_pair, spread 2, random rollouts): the idle odd lane of each pair counts
// half of the even lane's stencil entries (count_class_pair).
template <bool HEUR, bool PAIR = false>
__device__ __forceinline__ void mcts_body(const MctsArgs& a) {
    static_assert(!(HEUR && PAIR), "the heuristic pass is not split");
    constexpr int BLK = HEUR ? HBLOCK : BLOCK;
    // PAIR: + the LDS-DMA stage of the pairs' mover tables after the 40 dwords per lane of
    // counts / rows (2 blocks of 77 KB per CU)
    constexpr int AREA = HEUR ? HEUR_WORDS : PAIR ? 40 * WAVE + DMA_RUNS * DMA_RUN_DWORDS
                                                  : ROLL_WORDS_STAGE(BK_FS_STAGE_MCTS);
    static_assert(AREA >= ROLL_WORDS_STAGE(BK_FS_STAGE_MCTS) || HEUR, "the replay's 128-slot stage fits");
    constexpr int HS_WORDS = HEUR ? (int)(sizeof(HeurShared) + 7) / 4 : 0;
    // per wave: counts / B,C rows (+ HEUR: per-piece e sums) / the staged frontier table
    __shared__ __attribute__((aligned(16))) uint32_t lds[AREA * (BLK / WAVE) + 2 * BK_CELLS + HS_WORDS];
    const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
    uint32_t* my = lds + wv * AREA;
    uint32_t* dstage = my + 40 * WAVE;  // PAIR: run r of pair q at dstage + r * DMA_RUN_DWORDS + 8 q
    int16_t* stage_q = reinterpret_cast<int16_t*>(dstage + 8 * (lane >> 1));
    uint2* rows_lds = reinterpret_cast<uint2*>(my) + lane;
    int16_t* lk = reinterpret_cast<int16_t*>(my) + 2 * lane;
    uint64_t* htab = reinterpret_cast<uint64_t*>(lds + AREA * (BLK / WAVE));
    HeurShared* hs = reinterpret_cast<HeurShared*>(lds + AREA * (BLK / WAVE) + 2 * BK_CELLS);
    double* psum = reinterpret_cast<double*>(my + HEUR_PSUM * WAVE) + lane;
    for (int i = threadIdx.x; i < BK_CELLS; i += BLK) htab[i] = kCellHash[i];
    if constexpr (HEUR) heur_shared_init(hs, threadIdx.x, BLK);
    __syncthreads();
    const uint32_t slot = blockIdx.x * BLK + threadIdx.x;
    const Slab slab{a.slab + (size_t)slot * SLAB_WORDS};
    McLane* L = a.lanes + slot;
    Mc m;
    m.game = -1;
    m.mode = MC_SELECT;
    bool done = (lane % a.spread) != 0;
    SECT_DECL
    for (uint64_t step = 0;; ++step) {
        SECT(13);
        // ---- tree work until this lane needs a movegen (divergent).  The wave runs it
        // once a.tree_batch lanes wait for it (or none is mid-simulation): selection,
        // replay and backpropagation of one lane cost the whole wave about one ply, so
        // batching them beats letting every finished rollout stall the other 63 lanes.
        // Lanes play independent searches: the order changes no result.
        // PAIR: the tree phase stages tables in LDS over the DMA stage, so no DMA of the
        // previous step may still be landing (a step that ended before locate never waited)
        if constexpr (PAIR) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t waiting = __ballot(!done && m.mode == MC_SELECT);
        const bool tree_now = __popcll(waiting) >= a.tree_batch || __ballot(!done && m.mode != MC_SELECT) == 0ull;
        while (tree_now && !done && m.mode == MC_SELECT) {
            if (m.game < 0) {
                const int32_t next = (int32_t)atomicAdd(&a.counter[0], 1u);
                if (next >= a.n_games) { done = true; break; }
                const bool twice = mc_mark_started(a, next, (uint32_t)next);
                mc_start_game(a, m, L, next, htab);
                if (twice) m.status |= BK_MCTS_EINTERNAL;
            }
            const bool timed_out = a.cfg.time_limit_us > 0 &&
                                   wall_clock64() - m.t0 >= a.limit_ticks;
            const bool chunk_end = a.cfg.iter_stop > 0 && m.it >= a.cfg.iter_stop;
            if (m.it >= a.cfg.iterations || chunk_end || timed_out || MC_FATAL(m.status)) { mc_finish_game(a, m); continue; }
            const uint64_t* Z = a.zobrist + (size_t)a.zidx[m.game] * MC_ZOB;
            SECT(2);
            const bool term = mc_select(a, m, L, Z);
            SECT(0);
            if (term) { mc_sim_terminal(a, m, L); continue; }
            if (MC_FATAL(m.status)) continue;
            mc_replay(a, m, slab, L, htab, lk);
            SECT(1);
            m.mode = MC_EXPAND;
        }
        if (__ballot(!done) == 0ull) break;
        if (step > a.max_steps) {  // safety valve: never spin forever
            if (lane == 0) { atomicOr(&a.counter[1], 1u); atomicOr(&a.counter[2], BK_STICKY_GUARD); }
            break;
        }
        SECT(8);
        // ---- one movegen per busy lane (uniform work)
        const bool idle = done || m.mode == MC_SELECT;
        const int p = idle ? 0 : (m.mode == MC_EXPAND ? ((m.root_player + m.depth) & 3) : m.cur);
        // the board-player this lane counts: its own, or (PAIR, odd lane) its even neighbour's
        bool c_idle = idle;
        int cp = p;
        uint32_t c_first = (m.first >> p) & 1u, c_used = m.used.get(p);
        uint32_t* c_base = slab.base;
        const bk_fset* ofs = nullptr;  // PAIR: the pair's node / sim tables and the mover's mask
        uint32_t omask = 0xFFFFu;
        if constexpr (PAIR) {
            c_idle = pair_even((int)idle) != 0;
            cp = pair_even(p);
            c_first = (uint32_t)pair_even((int)c_first);
            c_used = (uint32_t)pair_even((int)c_used);
            c_base = a.slab + (size_t)(slot & ~1u) * SLAB_WORDS;
            ofs = &a.lanes[slot & ~1u].A.s;
            omask = ofs->mask[cp];
        }
        const Slab cslab{c_base};
        Planes P;
        {
            uint32_t own[20], occ[20];
#pragma unroll
            for (int R = 0; R < 20; ++R) {
                own[R] = c_idle ? 0u : cslab.at(cp, R);
                occ[R] = c_idle ? 0u : cslab.at(4, R);
            }
            derive_rows(own, occ, c_first, cp, P);
        }
        make_pairs(P);
        // PAIR: the mover's table (<= 128 slots) goes to the pair's LDS-DMA stage while the
        // stencil runs: the lanes of a pair load alternate 16-byte halves of each 16-slot run
        bool staged = false;
        if constexpr (PAIR) {
            staged = !c_idle && omask < 16u * DMA_RUNS;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the table's last stores have landed
            const int16_t* src = ofs->key[cp] + 8 * (lane & 1);
#pragma unroll
            for (int r = 0; r < DMA_RUNS; ++r) {
                const bool need = staged && omask >= 16u * (uint32_t)r;
                if (__builtin_amdgcn_ballot_w64(need) == 0ull) break;
                if (need)
                    __builtin_amdgcn_global_load_lds((const void*)(src + 16 * r), (void*)(dstage + r * DMA_RUN_DWORDS),
                                                     16, 0, 0);
            }
        }
        const uint32_t avail = c_idle ? 0u : (~c_used & 0x1FFFFFu);
        uint32_t total = movegen_counts<true, PAIR>(P, avail, my, lane);
        if constexpr (PAIR) total += (uint32_t)pair_other((int)total);
        SECT(9);
        // PAIR: the odd lane of a busy pair stays for the pair's locate (below)
        if (!PAIR && idle) continue;
        bool act = !idle;
        bk_mcts_node* pool = a.nodes + (size_t)(act ? m.game : 0) * a.cfg.node_cap;
        uint32_t k = 0;
        if (act) {
            if (m.mode == MC_EXPAND) {
                bk_mcts_node* nd = pool + m.node;
                uint32_t n_legal = nd->n_legal, n_exp = nd->n_exp;
                if (!(nd->flags & BK_MCTS_NODE_EVALUATED)) {  // MCTSNode._initialize_untried_moves
                    n_legal = total;
                    nd->n_legal = (uint16_t)n_legal;
                    nd->child0 = -1;
                    nd->flags = BK_MCTS_NODE_EVALUATED;
                }
                if (n_legal != total) {  // an evaluated node's list cannot change
                    m.status |= BK_MCTS_EINTERNAL;
                    m.mode = MC_SELECT;
                    act = false;
                } else if (n_legal == n_exp) {  // no legal move: terminal leaf
                    mc_sim_terminal(a, m, L);
                    act = false;
                } else {
                    k = n_legal - n_exp - 1u;  // untried_moves.pop(): the last list entry
                }
            } else if (total == 0u) {  // _rollout: no legal move -> break
                mc_complete(a, m, L, (double)(mc_score(m, m.player) - m.score0), false);
                act = false;
            } else {
                k = HEUR ? 0u : mc_randint(a.mt + (size_t)m.game * (FM_N + 1), m.mt_pos, total);
            }
        }
        if (!PAIR && !act) continue;
        uint32_t kk = 0;
        int gs = act ? pick_orient<PAIR>(my, lane, k, kk) : 0;
        // HEUR: a rollout ply's move is HeuristicAgent.select_action's (heur_* above)
        const bool hroll = HEUR && m.mode == MC_ROLLOUT;
        double h_target = 0.0, h_R = 0.0, h_total = 0.0;
        uint32_t h_ok[20];
        bool h_unc = false;
        int edge_w = 6;
        if constexpr (HEUR) {
            if (__builtin_amdgcn_ballot_w64(hroll)) {
                // Board.move_count of the rollout board: placements on the way from the root
                edge_w = (int)(a.roots[m.game].move_count + m.depth + m.plies) < 30 ? 6 : 3;
#pragma unroll
                for (int R = 0; R < 20; ++R) rows_lds[R * WAVE].x = P.b(R);
                heur_pass_a(P, hroll ? avail : 0u, rows_lds, psum, hs, edge_w);
#pragma unroll
                for (int R = 0; R < 20; ++R) rows_lds[R * WAVE] = make_uint2(P.b(R), P.c(R));
                if (hroll) {
#pragma unroll 1
                    for (int q = 0; q < BK_PIECES; ++q) h_total += psum[q * WAVE];
                    h_target = mc_random_sample(a.mt + (size_t)m.game * (FM_N + 1), m.mt_pos) * h_total;
                    gs = heur_pick_orient(psum, rows_lds, hs, edge_w, h_target, h_R, h_ok, h_unc);
                }
            }
        }
#pragma unroll
        for (int R = 0; R < 20; ++R) rows_lds[R * WAVE] = make_uint2(P.b(R), P.c(R));
        FsLane* T = &L->A;  // the node board at expansion, the rollout's sim board after it
        int ar = -1, ac = 0;
        SECT(10);
        if constexpr (PAIR) {
            // both lanes of a busy pair: the even lane's orientation, rank and table
            const int o = lane & ~1;  // the pair's even lane (its LDS column)
            const bool pact = pair_even((int)act) != 0;
            const int pgs = pair_even(gs);
            const uint32_t pkk = (uint32_t)pair_even((int)kk);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA stage has landed
            if (pact) {
                uint2* prow = reinterpret_cast<uint2*>(my) + o;
                if (staged) locate_frontier_pair<DMA_RUN_DWORDS / 4>(pgs, pkk, prow, stage_q, (int)omask, (lane & 1) != 0, ar, ac);
                else locate_frontier_pair(pgs, pkk, prow, ofs->key[cp], (int)omask, (lane & 1) != 0, ar, ac);
            }
            if (!act) continue;
        } else if (hroll) {
            if (gs < 0) {
                ar = -1;
                ac = 0;
            } else {
                heur_walk_frontier(gs, h_ok, rows_lds, T->s.key[p], T->s.mask[p], hs, edge_w, h_target, h_R, h_total,
                                   ar, ac, h_unc);
            }
            if (h_unc) m.status |= BK_MCTS_EUNCERT;
        } else {
            locate_move_frontier(gs, kk, rows_lds, T->s.key[p], T->s.mask[p], ar, ac);
        }
        SECT(11);
        if (ar < 0) {  // the table does not list the move: counts and tables disagree
            m.status |= BK_MCTS_EINTERNAL;
            m.mode = MC_SELECT;
            continue;
        }
        uint32_t pm[5];
        int32_t cells[5];
        piece_cells(gs, ar, ac, pm, cells);
        // all lanes, before any table staging
        const uint64_t real = frontier_ops(rows_lds, slab, p, (m.first >> p) & 1u, gs, ar, ac, pm);
        SECT(3);
#ifdef BK_SECTION_PROF
        {  // diagnostic counts (not cycles): [6] placements (wave steps), [7] their real ops
            uint32_t cs = (uint32_t)__popcll(real);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) cs += (uint32_t)__shfl_xor((int)cs, o);
            sect_acc[6] += 1;
            sect_acc[7] += cs;
        }
#endif
        // MCTSNode.expand (mcts_agent.py:113-145) places on new_board = board.copy() (B),
        // a rollout ply on sim (B): one place call site for both
        const bool expand = m.mode == MC_EXPAND;
        uint32_t c = 0;
        bool ok = true;
        if (expand) {
            bk_mcts_node* nd = pool + m.node;
            const int32_t cs = mc_child_slot(pool, nd, m, a.cfg.node_cap);
            if (cs < 0) { m.status |= BK_MCTS_EPOOL; m.mode = MC_SELECT; continue; }
            c = (uint32_t)cs;
            nd->n_exp = (uint16_t)(nd->n_exp + 1u);
            bk_mcts_node ch;
            ch.total = 0.0; ch.visits = 0; ch.child0 = -1;
            ch.move = (uint16_t)(gs * 400 + ar * 20 + ac);
            ch.n_exp = 0; ch.n_legal = 0; ch.flags = 0;
            pool[c] = ch;
            if (m.depth >= BK_MCTS_MAX_DEPTH) { m.status |= BK_MCTS_EPATH; m.mode = MC_SELECT; continue; }
        }
        // expand: new_board = board.copy() is table A itself (A is a copy, see mc_replay),
        // and MCTSNode(new_board)'s copy replaces the mover's table in place; the rollout's
        // sim = node.board.copy() is that copy again (A), and its plies place on A
        int16_t* sq = (PAIR && staged) ? stage_q : nullptr;
#ifdef BK_SECTION_PROF
        auto mark = [&](int i) { SECT(i); };
#else
        NoMark mark;
#endif
        if (expand) ok &= mc_place_staged<true>(m, slab, p, gs, ar, &L->A, htab, pm, cells, real, lk, sq, mark);
        else ok &= mc_place_staged<false>(m, slab, p, gs, ar, &L->A, htab, pm, cells, real, lk, sq, mark);
        if (expand) {
            if (!ok) { m.status |= BK_MCTS_EFSET; m.mode = MC_SELECT; continue; }
            const uint64_t* Z = a.zobrist + (size_t)a.zidx[m.game] * MC_ZOB;
            m.hash = mc_hash_step(Z, m.hash, p, (m.root_cp + m.depth) & 3, gs, ar, ac);
            L->path[++m.depth] = (int32_t)c;
            m.node = (int32_t)c;
            double reward = 0.0;
            if (a.cfg.use_tt && mc_tt_lookup(a, m, reward)) {
                mc_complete(a, m, L, reward, true);
                continue;
            }
            // _rollout (mcts_agent.py:470-554) on sim = node.board.copy(): the copy of the
            // copy in B is B
            m.player = m.cur = (m.root_player + m.depth) & 3;
            m.score0 = mc_score(m, m.player);
            m.plies = 0;
            m.mode = MC_ROLLOUT;
            SECT(12);
        } else {
            if (!ok) { m.status |= BK_MCTS_EFSET; m.mode = MC_SELECT; continue; }
            m.plies++;
            m.rplies++;
            m.cur = (m.cur + 1) & 3;
            if (m.plies >= a.cfg.max_rollout_moves)
                mc_complete(a, m, L, (double)(mc_score(m, m.player) - m.score0), false);
            SECT(14);
        }
    }
    SECT_FLUSH;
}

#if BK_DEF(BK_U_MCTS)
__global__ __launch_bounds__(BLOCK, MCTS_BLOCKS_PER_CU) void k_mcts(MctsArgs a) { mcts_body<false>(a); }
// ZobristHash.hash_board (mcts/zobrist.py:70-99) of each root, one lane per root: the
// cell keys (cell * 5 + occupant, 0 = empty), the side to move, the used pieces -- what
// mcts/zobrist.py hash_states computes on the host (bk_mcts with root_hash NULL)
__global__ __launch_bounds__(BLOCK) void k_root_hash(const bk_state* roots, const uint64_t* zob,
                                                     const int32_t* zidx, uint64_t* out, int32_t n) {
    const int32_t g = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (g >= n) return;
    const bk_state* s = roots + g;
    const uint64_t* Z = zob + (size_t)zidx[g] * MC_ZOB;
    uint64_t h = 0;
#pragma unroll 1
    for (int w = 0; w < 7; ++w) {
        const uint64_t p0 = s->planes[0][w], p1 = s->planes[1][w], p2 = s->planes[2][w], p3 = s->planes[3][w];
        const int nb = w < 6 ? 64 : BK_CELLS - 6 * 64;
#pragma unroll 1
        for (int b = 0; b < nb; ++b) {
            const int o = ((p0 >> b) & 1u) ? 1 : ((p1 >> b) & 1u) ? 2 : ((p2 >> b) & 1u) ? 3 : ((p3 >> b) & 1u) ? 4 : 0;
            h ^= Z[(w * 64 + b) * 5 + o];
        }
    }
    h ^= Z[2000 + (s->current_player & 3)];
#pragma unroll 1
    for (int p = 0; p < 4; ++p)
#pragma unroll 1
        for (int i = 0; i < BK_PIECES; ++i)
            if ((s->used[p] >> i) & 1u) h ^= Z[2004 + p * BK_PIECES + i];
    out[g] = h;
}
#else
__global__ void k_mcts(MctsArgs a);
__global__ void k_root_hash(const bk_state* roots, const uint64_t* zob, const int32_t* zidx, uint64_t* out,
                            int32_t n);
#endif
#if BK_DEF(BK_U_MCTS_PAIR)
__global__ __launch_bounds__(BLOCK, MCTS_BLOCKS_PER_CU) void k_mcts_pair(MctsArgs a) { mcts_body<false, true>(a); }
#else
__global__ void k_mcts_pair(MctsArgs a);
#endif
#if BK_DEF(BK_U_MCTS_H)
__global__ __launch_bounds__(HBLOCK, 2) void k_mcts_h(MctsArgs a) { mcts_body<true>(a); }
#else
__global__ void k_mcts_h(MctsArgs a);
#endif

// ------------------------------------------------------------------------------------
// Cooperative MCTSAgent searches: ONE 64-lane wave per search, for batches too small to
// fill the chip with one search per lane (config 4: ~500 MCTS seats to move per arena
// round, i.e. 8 waves on 1,024 SIMDs; single MCTSAgent.select_action calls: 1 lane).
// Every lane of the wave holds the same search: the same registers, the same data in its
// own LDS column, and the wave's slab / McLane / node pool / TT / MT state in HBM.  The
// serial parts (tree select / replay / backprop, TT, the frontier tables, locate, place)
// therefore run unchanged and redundantly -- identical stores to identical addresses --
// and the one atomic (the game counter) is lane 0's.  The per-ply work that is parallel
// is split over the lanes: lane l evaluates orientations l and l + 64 with data-driven
// cell terms from the B/C rows in its column (lane_ok_rows), the per-orientation counts
// are wave-scanned for the pick (naive order: g ascending), and the HeuristicAgent's e
// sums (lane_orient_sum) go to a wave-shared array and are summed per piece in
// orientation order.  The searches are the reference's, as in k_mcts / k_mcts_h (tests
// run both kernels on the same batches).
// ------------------------------------------------------------------------------------
#define COOP_WAVES 2                             // searches (waves) per block
// k_mcts_coop_h keeps the search's McLane in LDS, both cooperative kernels the search's
// slab.  k_mcts_coop_h runs one wave per SIMD (a 2-wave build, <= 256 registers, spills:
// 755 vs 832 games/s, profiles/r05/sweeps/r05g).
#define COOP_AREA ROLL_WORDS_STAGE(BK_FS_STAGE_MCTS)  // per-wave per-lane area (rows / staged table)

// Wave-wide scans and broadcasts of the cooperative kernels (all 64 lanes active).  The
// inclusive prefix sum runs on DPP: row_shr 1 / 2 / 4 / 8 inside each 16-lane row, then
// row_bcast 15 and row_bcast 31 add the earlier rows' totals -- six ALU-latency steps,
// where a __shfl_up ladder is six dependent ds_bpermute round trips through the LDS
// crossbar (two per step for a double).  Lanes whose DPP source is outside the row, or
// whose row is masked off, read the identity (old = 0).  A broadcast from a uniform lane
// (found by a ballot) is a v_readlane into a scalar register, not a ds_bpermute.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = dpp_u32<CTRL, ROWS>((uint32_t)b), hi = dpp_u32<CTRL, ROWS>((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | (uint64_t)lo));
}
#define DPP_ROW_SHR(n) (0x110 + (n))
#define DPP_ROW_BCAST15 0x142
#define DPP_ROW_BCAST31 0x143
#define DPP_WAVE_SHR1 0x138

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int) {
    v += dpp_u32<DPP_ROW_SHR(1), 0xF>(v);
    v += dpp_u32<DPP_ROW_SHR(2), 0xF>(v);
    v += dpp_u32<DPP_ROW_SHR(4), 0xF>(v);
    v += dpp_u32<DPP_ROW_SHR(8), 0xF>(v);
    v += dpp_u32<DPP_ROW_BCAST15, 0xA>(v);
    v += dpp_u32<DPP_ROW_BCAST31, 0xC>(v);
    return v;
}

__device__ __forceinline__ uint32_t lane_bcast(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ int lane_bcast(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double lane_bcast(double v, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | (uint64_t)lo));
}

// legal-move counts (and with E the e sums, HeuristicAgent pass A) of this lane's
// orientations g = lane + 64 h; 0 for g >= 91 or a used piece.  rows = {B, C} in the
// lane's column.
// The wave's live orientations (pieces the mover still holds), compacted onto its lanes:
// lane k takes the k-th live orientation in g order for pass 0 and the (64 + k)-th for
// pass 1 (og[h], -1 none), so a ply with <= 64 live orientations -- most rollout plies once
// a few pieces are down -- runs ONE pass of the per-lane orientation work instead of two.
// The order is g ascending, so scans over (pass 0 lanes, pass 1 lanes) run in the
// reference's list order.  otab: 91 int16 of wave-private LDS (the walk's rank array,
// which coop_walk re-initialises before use).  Returns the live count.
__device__ __forceinline__ uint32_t coop_live_orients(uint32_t avail, int lane, int16_t* otab, int (&og)[2]) {
    bool live[2];
    uint64_t msk[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int g = lane + WAVE * h;
        live[h] = g < BK_NUM_ORIENTS && ((avail >> ((kInfo[g < BK_NUM_ORIENTS ? g : 0] & 0xFFu) - 1u)) & 1u);
        msk[h] = __ballot(live[h]);
    }
    const uint32_t n0 = (uint32_t)__popcll(msk[0]), n = n0 + (uint32_t)__popcll(msk[1]);
    const uint64_t lt = (1ull << lane) - 1ull;
    if (live[0]) otab[__popcll(msk[0] & lt)] = (int16_t)lane;
    if (live[1]) otab[n0 + (uint32_t)__popcll(msk[1] & lt)] = (int16_t)(lane + WAVE);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    og[0] = (uint32_t)lane < n ? (int)otab[lane] : -1;
    og[1] = (uint32_t)(lane + WAVE) < n ? (int)otab[lane + WAVE] : -1;
    return n;
}

template <bool E>
__device__ __forceinline__ void coop_orients(const uint2* rows, const int (&og)[2], uint32_t nlive,
                                             const HeurShared* hs, int edge_w, uint32_t (&cnt)[2],
                                             double (&es)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        cnt[h] = 0u;
        es[h] = 0.0;
        if (h == 1 && nlive <= (uint32_t)WAVE) continue;  // (uniform) one pass holds them all
        const int g = og[h];
        if (g >= 0) {
            uint32_t ok[20];
            lane_ok_rows(g, rows, ok);
#pragma unroll
            for (int r = 0; r < 20; ++r) cnt[h] += __builtin_popcount(ok[r]);
            if constexpr (E) es[h] = lane_orient_sum(g, ok, rows, hs, edge_w);
        }
    }
}

__device__ __forceinline__ double wave_incl_scan_f64(double v, int) {
    v += dpp_f64<DPP_ROW_SHR(1), 0xF>(v);
    v += dpp_f64<DPP_ROW_SHR(2), 0xF>(v);
    v += dpp_f64<DPP_ROW_SHR(4), 0xF>(v);
    v += dpp_f64<DPP_ROW_SHR(8), 0xF>(v);
    v += dpp_f64<DPP_ROW_BCAST15, 0xA>(v);
    v += dpp_f64<DPP_ROW_BCAST31, 0xC>(v);
    return v;
}

struct CoopScan {
    uint32_t i0, i1, c0, c1;  // inclusive prefix counts of this lane's two orientations
    uint32_t total;
};

__device__ __forceinline__ CoopScan coop_scan(const uint32_t (&cnt)[2], int lane) {
    CoopScan s;
    s.c0 = cnt[0];
    s.c1 = cnt[1];
    s.i0 = wave_incl_scan(cnt[0], lane);
    const uint32_t t0 = lane_bcast(s.i0, WAVE - 1);
    s.i1 = wave_incl_scan(cnt[1], lane) + t0;
    s.total = lane_bcast(s.i1, WAVE - 1);
    return s;
}

// pick_orient for the wave's search: the orientation holding the k-th legal move (g
// ascending) and the move's rank kk in it
__device__ __forceinline__ int coop_find(const CoopScan& s, const int (&og)[2], uint32_t k, uint32_t& kk) {
    const uint64_t b0 = __ballot(k < s.i0 && k >= s.i0 - s.c0);
    const uint64_t b1 = __ballot(k < s.i1 && k >= s.i1 - s.c1);
    int g = BK_NUM_ORIENTS - 1;
    uint32_t before = k;
    if (b0) {
        const int L = __ffsll((unsigned long long)b0) - 1;
        g = lane_bcast(og[0], L);
        before = lane_bcast(s.i0 - s.c0, L);
    } else if (b1) {
        const int L = __ffsll((unsigned long long)b1) - 1;
        g = lane_bcast(og[1], L);
        before = lane_bcast(s.i1 - s.c1, L);
    }
    kk = k - before;
    return g;
}

// heur_pick_orient for the wave's search from the lanes' e sums (es[h] of orientation
// lane + 64 h): the orientation (list order: g ascending) whose cumulative e crosses
// target, by a wave scan; R = cumulative e before it, total = the sum of all.  The sums
// differ from the per-piece serial ones by rounding only (the walk certifies the draw
// against HEUR_MARGIN).  Uncertain when no crossing is found (rounding at the total).
__device__ __forceinline__ int coop_heur_pick(const double (&es)[2], const int (&og)[2], int lane, const uint32_t* st,
                                              uint32_t& pos,
                                              uint32_t pre0, uint32_t pre1, double& target, double& R,
                                              double& total, bool& uncertain) {
    const double i0 = wave_incl_scan_f64(es[0], lane);
    const double i1 = wave_incl_scan_f64(es[1], lane) + lane_bcast(i0, WAVE - 1);
    total = lane_bcast(i1, WAVE - 1);
    // HeuristicAgent's draw (random_sample): the two words were loaded ahead (pre) when
    // the state holds them without a twist
    double u;
    if (pos + 2u <= (uint32_t)FM_N) {
        u = ((double)(mc_temper(pre0) >> 5) * 67108864.0 + (double)(mc_temper(pre1) >> 6)) *
            (1.0 / 9007199254740992.0);
        pos += 2u;
    } else {
        u = mc_random_sample(const_cast<uint32_t*>(st), pos);
    }
    target = u * total;
    const uint64_t b0 = __ballot(es[0] > 0.0 && i0 > target);
    const uint64_t b1 = __ballot(es[1] > 0.0 && i1 > target);
    int L = -1, h = 0;
    if (b0) { L = __ffsll((unsigned long long)b0) - 1; }
    else if (b1) { L = __ffsll((unsigned long long)b1) - 1; h = 1; }
    else {
        uncertain = true;
        const uint64_t l1 = __ballot(es[1] > 0.0), l0 = __ballot(es[0] > 0.0);
        if (l1) { L = 63 - __clzll((unsigned long long)l1); h = 1; }
        else if (l0) { L = 63 - __clzll((unsigned long long)l0); }
    }
    if (L < 0) { R = 0.0; return -1; }
    R = lane_bcast(h ? i1 - es[1] : i0 - es[0], L);
    return lane_bcast(h ? og[1] : og[0], L);
}

// legal anchor rows and counts of this lane's orientations g = lane + 64 h (rows = {B, C}
// in the lane's column); 0 rows for g >= 91 or a used piece.  The rows stay in registers
// for the balanced heuristic pass.
__device__ __forceinline__ uint32_t coop_ok_count1(const uint2* rows, int g, uint32_t (&ok)[20]) {
    if (g >= 0) {
        lane_ok_rows(g, rows, ok);
    } else {
#pragma unroll
        for (int r = 0; r < 20; ++r) ok[r] = 0u;
    }
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < 20; ++r) c += __builtin_popcount(ok[r]);
    return c;
}

__device__ __forceinline__ void coop_ok_counts(const uint2* rows, const int (&og)[2], uint32_t nlive,
                                               uint32_t (&ok0)[20], uint32_t (&ok1)[20], uint32_t (&cnt)[2]) {
    cnt[0] = coop_ok_count1(rows, og[0], ok0);
    if (nlive > (uint32_t)WAVE) {  // (uniform) a second pass only for > 64 live orientations
        cnt[1] = coop_ok_count1(rows, og[1], ok1);
    } else {
        cnt[1] = 0u;
#pragma unroll
        for (int r = 0; r < 20; ++r) ok1[r] = 0u;
    }
}

// orientation g's legal moves (rows ok) into the move list from index idx: naive order
// The 20 rows are packed into seven 64-bit words of cell bits (r * 20 + c) first, so the
// divergent bit loops run 7 times (each as long as its busiest lane) instead of 20
__device__ __forceinline__ void coop_list_moves(uint16_t* ml, uint32_t idx, uint32_t g, const uint32_t (&ok)[20]) {
    uint64_t P[7] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
#pragma unroll
    for (int r = 0; r < 20; ++r) {
        const int off = 20 * r, q = off / 64, sh = off % 64;
        P[q] |= (uint64_t)ok[r] << sh;
        if (sh > 44) P[q + 1] |= (uint64_t)ok[r] >> (64 - sh);
    }
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        uint64_t w = P[q];
        while (w) {
            const uint32_t x = (uint32_t)__builtin_ctzll(w);
            w &= w - 1ull;
            ml[idx++] = (uint16_t)(g * 400u + 64u * (uint32_t)q + x);
        }
    }
}

// lane_ok_rows / locate_pass1 for the wave's ONE orientation gs (every lane's column holds
// the same {B, C} rows): lane r < 20 computes anchor row r from its own column (5 LDS
// reads, conflict-free), and the 20 rows are broadcast with v_readlane, so ok[] is
// wave-uniform -- instead of every lane computing all 20 rows (100 LDS reads and ~240
// VALU per lane).  All 64 lanes must be active (the cooperative kernels' uniform flow).
__device__ __forceinline__ void coop_ok_rows(int gs, const uint2* rows, int lane, uint32_t (&ok)[20]) {
    const uint32_t info = kInfo[gs];
    const int n = (int)((info >> 8) & 0xFFu);
    const int rlim = 20 - (int)((info >> 16) & 0xFFu);
    const int r = lane < 20 ? lane : 0;
    const int rr = r < rlim ? r : rlim;
    uint2 v[5];
    uint32_t sh[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t cell = kCells[gs][k < n ? k : 0];
        sh[k] = cell & 0xFFu;
        v[k] = rows[(rr + (int)(cell >> 8)) * WAVE];
    }
    uint32_t ab = BITOP3(v[0].x >> sh[0], v[1].x >> sh[1], v[2].x >> sh[2], LUT_OR3);
    uint32_t ac = BITOP3(v[0].y >> sh[0], v[1].y >> sh[1], v[2].y >> sh[2], LUT_OR3);
    ab = BITOP3(ab, v[3].x >> sh[3], v[4].x >> sh[4], LUT_OR3);
    ac = BITOP3(ac, v[3].y >> sh[3], v[4].y >> sh[4], LUT_OR3);
    const uint32_t mine = r <= rlim ? (ac & ~ab) : 0u;
#pragma unroll
    for (int q = 0; q < 20; ++q) ok[q] = (uint32_t)__builtin_amdgcn_readlane((int)mine, q);
}

// Balanced HeuristicAgent pass A for the wave's search (k_mcts_coop_h): instead of each
// lane summing e over its own two orientations' moves (the wave then iterates the
// largest orientation's move count, ~1 legal move per lane-iteration), the ply's legal
// moves go to a list in LDS in naive order (orientation ascending, anchors row-major:
// orientation g at [s_g, s_g + c_g) from the count scan), and the wave evaluates
// e = exp(score) 64 moves at a time, with a running prefix sum.  The lane holding the
// first / last move of an orientation records the cumulative e before / after it; the
// crossing of target = u * total is then found at orientation level by a ballot, exactly
// what coop_heur_pick decides from per-orientation sums (the sums differ by rounding only;
// the walk certifies the draw against HEUR_MARGIN).  area = the wave's LDS area (the move
// list and the cumulative sums after the {B, C} rows).  false: more than COOP_MOVE_CAP
// legal moves (nothing done; the caller runs coop_orients<true> + coop_heur_pick).
#define COOP_MOVE_CAP 2048
#define COOP_ML_DWORD (40 * WAVE)                        // after the rows' 40 dwords per lane
#define COOP_CUM_DWORD (COOP_ML_DWORD + COOP_MOVE_CAP / 2)  // cumE[91], cumS[91] (doubles)
template <typename Mark = NoMark>
__device__ __forceinline__ bool coop_heur_balanced(const uint2* rows, uint32_t* area, int lane, const HeurShared* hs,
                                                   int edge_w, const int (&og)[2], const uint32_t (&ok0)[20],
                                                   const uint32_t (&ok1)[20],
                                                   const uint32_t (&cnt)[2], const CoopScan& sc, const uint32_t* st,
                                                   uint32_t& pos, uint32_t pre0, uint32_t pre1, double& target,
                                                   double& R, double& total, bool& uncertain, int& gs,
                                                   uint32_t (&gok)[20], Mark mark = Mark()) {
    const uint32_t n_moves = sc.total;
    if (n_moves > COOP_MOVE_CAP) return false;
    uint16_t* ml = reinterpret_cast<uint16_t*>(area + COOP_ML_DWORD);
    double* cumE = reinterpret_cast<double*>(area + COOP_CUM_DWORD);
    double* cumS = cumE + BK_NUM_ORIENTS;
    mark(3);
    coop_list_moves(ml, sc.i0 - sc.c0, (uint32_t)(og[0] < 0 ? 0 : og[0]), ok0);  // (no moves when og < 0)
    coop_list_moves(ml, sc.i1 - sc.c1, (uint32_t)(og[1] < 0 ? 0 : og[1]), ok1);
    mark(6);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double carry = 0.0;
    // the B rows through this lane's own column: lanes read different rows, and column 0's
    // rows all sit in one LDS bank (a 20-way conflict per read)
    const uint2* const own = rows + lane;
#pragma unroll 1
    for (uint32_t k0 = 0; k0 < n_moves; k0 += WAVE) {
        const uint32_t k = k0 + (uint32_t)lane;
        const bool in = k < n_moves;
        const uint32_t mv = in ? ml[k] : 0u;
        const int g = (int)(mv / 400u), cell = (int)(mv % 400u);
        const int gn = k + 1u < n_moves ? (int)(ml[k + 1u] / 400u) : -1;
        const int gp = in && k > 0u ? (int)(ml[k - 1u] / 400u) : -1;
        double e = 0.0;
        if (in) {
            int n;
            uint32_t cd[5], cc[5];
            orient_cells(g, n, cd, cc);
            e = heur_e(n, cd, cc, cell / 20, cell % 20, own, hs, edge_w);
        }
        const double incl = wave_incl_scan_f64(e, lane) + carry;
        const double up = dpp_f64<DPP_WAVE_SHR1, 0xF>(incl);
        const double excl = lane ? up : carry;
        if (in && gn != g) cumE[g] = incl;
        if (in && gp != g) cumS[g] = excl;
        carry = lane_bcast(incl, WAVE - 1);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    mark(7);
    total = carry;
    // the HeuristicAgent's draw (random_sample), as coop_heur_pick
    double u;
    if (pos + 2u <= (uint32_t)FM_N) {
        u = ((double)(mc_temper(pre0) >> 5) * 67108864.0 + (double)(mc_temper(pre1) >> 6)) *
            (1.0 / 9007199254740992.0);
        pos += 2u;
    } else {
        u = mc_random_sample(const_cast<uint32_t*>(st), pos);
    }
    target = u * total;
    const double e0 = cnt[0] ? cumE[og[0]] : 0.0;
    const double e1 = cnt[1] ? cumE[og[1]] : 0.0;
    const uint64_t b0 = __ballot(cnt[0] != 0u && e0 > target);
    const uint64_t b1 = __ballot(cnt[1] != 0u && e1 > target);
    int L = -1, h = 0;
    if (b0) { L = __ffsll((unsigned long long)b0) - 1; }
    else if (b1) { L = __ffsll((unsigned long long)b1) - 1; h = 1; }
    else {
        uncertain = true;
        const uint64_t l1 = __ballot(cnt[1] != 0u), l0 = __ballot(cnt[0] != 0u);
        if (l1) { L = 63 - __clzll((unsigned long long)l1); h = 1; }
        else if (l0) { L = 63 - __clzll((unsigned long long)l0); }
    }
    if (L < 0) { R = 0.0; gs = -1; return true; }
    gs = lane_bcast(h ? og[1] : og[0], L);
    R = cumS[gs];
    // the chosen orientation's legal rows, recomputed from the {B, C} rows (coop_ok_rows,
    // every lane's column holds the same rows): ok0 / ok1 then die once the moves are
    // listed instead of staying live through the e pass (registers)
    coop_ok_rows(gs, own, lane, gok);
    return true;
}

// Cooperative pass 2 of locate_move_frontier / heur_walk_frontier (one wave = one search;
// the legal anchors of gs in rows[r * WAVE].y, identical in every lane's column).  Lane j
// takes the table's slots j and j + 64.  The anchor a = f - cell_k of the key f at slot s
// is NEW there -- the serial walk counts it at s -- iff no key of an earlier slot is
// another cell of the piece placed at a: rank[a + cell_q] > s for every q != k, where
// rank holds each key's slot (0x7FFF elsewhere; wave-private LDS).  Count mode (E =
// false): the kk-th new anchor in (slot, cell) order.  E: the anchor whose cumulative e
// from R first exceeds target, certified as in heur_walk_frontier (the prefix sums differ
// from the serial ones by rounding only, far inside the margin): the new anchors are
// listed in (slot, cell) order in `list` (wave-private LDS), their e values computed one
// per lane and wave-scanned from R -- one heur_e per lane for a list of <= 64 anchors,
// where the per-slot sums cost the busiest lane one heur_e per anchor of its two slots,
// and resolving the chosen slot up to five more.  Tables of more than 128 slots return
// false: the caller walks serially.
template <bool E>
__device__ __forceinline__ bool coop_walk(int gs, uint32_t kk, const uint2* rows, const int16_t* key, int mask,
                                          int16_t* rank, int lane, const HeurShared* hs, int edge_w, double target,
                                          double R, double total, int& out_r, int& out_c, bool& uncertain,
                                          uint16_t* list = nullptr) {
    if (mask > 2 * WAVE - 1) return false;
    int n;
    uint32_t cd[5], cc[5];
    orient_cells(gs, n, cd, cc);
#pragma unroll
    for (int t = 0; t < 7; ++t)
        if (lane + WAVE * t < BK_CELLS) rank[lane + WAVE * t] = 0x7FFF;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int f[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int sl = lane + WAVE * h;
        f[h] = sl <= mask ? (int)key[sl] : -1;
        if (f[h] >= 0) rank[f[h]] = (int16_t)sl;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t cnt[2] = {0u, 0u}, newk[2] = {0u, 0u};  // newk bit k: cell k's anchor is new here
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (f[h] < 0) continue;
        const int sl = lane + WAVE * h, fr = f[h] / 20, fc = f[h] - 20 * (f[h] / 20);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (k >= n) continue;
            const int ar = fr - (int)cd[k], acl = fc - (int)cc[k];
            if (ar < 0 || acl < 0 || !((rows[ar * WAVE].y >> acl) & 1u)) continue;
            bool fresh = true;
#pragma unroll
            for (int q = 0; q < 5; ++q)
                if (q < n && q != k && rank[(ar + (int)cd[q]) * 20 + acl + (int)cc[q]] < sl) fresh = false;
            if (!fresh) continue;
            newk[h] |= 1u << k;
            ++cnt[h];
        }
    }
    if constexpr (E) {
        const CoopScan sc = coop_scan(cnt, lane);
        const uint32_t na = sc.total;
        if (na == 0u) { out_r = -1; out_c = 0; return true; }
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // this lane's new anchors at their list positions
            uint32_t pos = h ? sc.i1 - sc.c1 : sc.i0 - sc.c0;
            if (!newk[h]) continue;
            const int fr = f[h] / 20, fc = f[h] - 20 * (f[h] / 20);
#pragma unroll
            for (int k = 0; k < 5; ++k)
                if ((newk[h] >> k) & 1u) list[pos++] = (uint16_t)((fr - (int)cd[k]) * 20 + fc - (int)cc[k]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double carry = R, lo = R, e_hit = 0.0;
        int cell_hit = -1;
#pragma unroll 1
        for (uint32_t b0 = 0; b0 < na; b0 += WAVE) {
            const uint32_t j = b0 + (uint32_t)lane;
            int cell = 0;
            double e = 0.0;
            if (j < na) {
                cell = list[j];
                e = heur_e(n, cd, cc, cell / 20, cell - 20 * (cell / 20), rows, hs, edge_w);
            }
            const double incl = wave_incl_scan_f64(e, lane) + carry;
            const double up = dpp_f64<DPP_WAVE_SHR1, 0xF>(incl);
            const double excl = lane ? up : carry;
            const uint64_t b = __ballot(j < na && incl > target);
            if (b) {
                const int L = __ffsll((unsigned long long)b) - 1;
                cell_hit = lane_bcast(cell, L);
                e_hit = lane_bcast(e, L);
                lo = lane_bcast(excl, L);
                break;
            }
            carry = lane_bcast(incl, WAVE - 1);
            if (b0 + WAVE >= na) {  // rounding put the target past the last anchor: the last one, uncertified
                const int L = (int)((na - 1u) & (WAVE - 1));
                cell_hit = lane_bcast(cell, L);
                e_hit = lane_bcast(e, L);
                lo = lane_bcast(excl, L);
                uncertain = true;
            }
        }
        if (!(target - lo > HEUR_MARGIN * total && lo + e_hit - target > HEUR_MARGIN * total)) uncertain = true;
        out_r = cell_hit / 20;
        out_c = cell_hit - 20 * (cell_hit / 20);
        return true;
    }
    // the slot holding the answer, then the anchor inside it in cell order
    int hit = -1, hh = 0;
    uint32_t before = 0;
    {
        const CoopScan sc = coop_scan(cnt, lane);
        const uint64_t b0 = __ballot(kk < sc.i0 && kk >= sc.i0 - sc.c0);
        const uint64_t b1 = __ballot(kk < sc.i1 && kk >= sc.i1 - sc.c1);
        if (b0) { hit = __ffsll((unsigned long long)b0) - 1; before = lane_bcast(sc.i0 - sc.c0, hit); }
        else if (b1) { hit = __ffsll((unsigned long long)b1) - 1; hh = 1; before = lane_bcast(sc.i1 - sc.c1, hit); }
    }
    if (hit < 0) { out_r = -1; out_c = 0; return true; }
    // every lane resolves the chosen slot (identical work and result)
    const int fh = lane_bcast(hh ? f[1] : f[0], hit);
    const uint32_t nk = lane_bcast(hh ? newk[1] : newk[0], hit);
    const int fr = fh / 20, fc = fh - 20 * (fh / 20);
    int found_r = -1, found_c = 0;
    uint32_t rem = kk - before;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        if (found_r >= 0 || !((nk >> k) & 1u)) continue;
        if (rem == 0u) { found_r = fr - (int)cd[k]; found_c = fc - (int)cc[k]; } else { --rem; }
    }
    out_r = found_r;
    out_c = found_c;
    return true;
}

static_assert(COOP_CUM_DWORD + 4 * BK_NUM_ORIENTS <= COOP_AREA, "the move list and sums fit a wave's area");

template <bool HEUR>
__device__ __forceinline__ void mcts_coop_body(const MctsArgs& a) {
    constexpr int BLK = COOP_WAVES * WAVE;
    constexpr int HS_WORDS = HEUR ? (int)(sizeof(HeurShared) + 7) / 4 : 0;
    __shared__ __attribute__((aligned(16))) uint32_t lds[COOP_AREA * COOP_WAVES + 2 * BK_CELLS + HS_WORDS];
    __shared__ int16_t coop_rank[COOP_WAVES][448];  // coop_walk: slot of each frontier key
    // the mover's table (<= 128 slots), one copy per wave, loaded by LDS-DMA while the
    // orientations are evaluated: locate / walk read it and the set operations run on it
    __shared__ __attribute__((aligned(16))) int16_t coop_stage[COOP_WAVES][16 * DMA_RUNS];
    __shared__ __attribute__((aligned(16))) uint32_t coop_slab[COOP_WAVES][SLAB_WORDS];
    // k_mcts_coop_h: the search's McLane (frontier tables of the node / sim board, the
    // root's tables, the path) lives in LDS too -- it is rebuilt at every search start,
    // so no launch leaves anything in it for the next -- and the mover's table is then
    // used in place (no LDS-DMA stage, no write-back).  (k_mcts_coop keeps it in HBM: the
    // 4.9 KB per wave would cost it a block per CU.)
    constexpr bool ML_LDS = HEUR;
    __shared__ __attribute__((aligned(16))) McLane coop_ml[ML_LDS ? COOP_WAVES : 1];
    const bool coop_walk_on = a.coop_walk != 0;
    // the wave index is uniform (readfirstlane): the wave's LDS area, slab and McLane
    // addresses live in scalar registers
    const int lane0 = threadIdx.x & (WAVE - 1), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
    uint32_t* my = lds + wv * COOP_AREA;
    uint64_t* htab = reinterpret_cast<uint64_t*>(lds + COOP_AREA * COOP_WAVES);
    HeurShared* hs = reinterpret_cast<HeurShared*>(lds + COOP_AREA * COOP_WAVES + 2 * BK_CELLS);
    for (int i = threadIdx.x; i < BK_CELLS; i += BLK) htab[i] = kCellHash[i];
    if constexpr (HEUR) heur_shared_init(hs, threadIdx.x, BLK);
    __syncthreads();
    const uint32_t slot = blockIdx.x * COOP_WAVES + wv;  // one slab / McLane per search
    // the search's board (the slab: planes, occupancy) lives in LDS, one per wave: it
    // is rebuilt from the root at every iteration, so nothing outside the wave reads it
    const Slab slab{coop_slab[wv]};
    McLane* L = ML_LDS ? &coop_ml[ML_LDS ? wv : 0] : a.lanes + slot;
    Mc m{};
    m.game = -1;
    m.mode = MC_SELECT;
    int root_mc = 0;  // Board.move_count of the search's root
    // section timers (-DBK_SECTION_PROF): 0 tree, 1 derive + rows, 2 lane orientations +
    // scan, 3 draw + pick, 4 locate / heuristic walk, 5 frontier ops + place + expansion
    SECT_DECL
    for (uint64_t step = 0;; ++step) {
        // An opaque per-step copy of the lane index: every lane-dependent address (LDS
        // columns, table entries of this lane's orientations) is recomputed inside the
        // loop, not hoisted out of it into registers held for the whole kernel (~60 such
        // addresses kept k_mcts_coop_h at one wave per SIMD)
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        uint2* rows_lds = reinterpret_cast<uint2*>(my) + lane;
        int16_t* lk = reinterpret_cast<int16_t*>(my) + 2 * lane;
        SECT(5);
        // ---- tree work until the search needs a movegen (uniform over the wave)
        bool done = false;
        while (m.mode == MC_SELECT) {
            if (m.game < 0) {
                int32_t next = 0;
                if (lane == 0) next = (int32_t)atomicAdd(&a.counter[0], 1u);
                next = __shfl(next, 0);
                if (next >= a.n_games) { done = true; break; }
                uint32_t twice = 0;
                if (lane == 0) twice = mc_mark_started(a, next, (uint32_t)next) ? 1u : 0u;
                twice = __shfl(twice, 0);
                mc_start_game(a, m, L, next, htab, lane, WAVE);
                if (twice) m.status |= BK_MCTS_EINTERNAL;
                root_mc = (int)a.roots[next].move_count;  // (constant for the search)
            }
            const bool timed_out = a.cfg.time_limit_us > 0 && wall_clock64() - m.t0 >= a.limit_ticks;
            const bool chunk_end = a.cfg.iter_stop > 0 && m.it >= a.cfg.iter_stop;
            if (m.it >= a.cfg.iterations || chunk_end || timed_out || MC_FATAL(m.status)) { mc_finish_game(a, m, lane, WAVE); continue; }
            const uint64_t* Z = a.zobrist + (size_t)a.zidx[m.game] * MC_ZOB;
            if (mc_select(a, m, L, Z)) { mc_sim_terminal(a, m, L); continue; }
            if (MC_FATAL(m.status)) continue;
            mc_replay(a, m, slab, L, htab, lk);
            m.mode = MC_EXPAND;
        }
        SECT(0);
        if (done) break;
        if (step > a.max_steps) {  // safety valve: never spin forever
            if (lane == 0) { atomicOr(&a.counter[1], 1u); atomicOr(&a.counter[2], BK_STICKY_GUARD); }
            break;
        }
        // ---- one movegen, split over the lanes
        const int p = m.mode == MC_EXPAND ? ((m.root_player + m.depth) & 3) : m.cur;
        const uint32_t tmask = L->A.s.mask[p];  // (loaded with the slab rows)
        Planes P;
        {
            uint32_t own[20], occ[20];
#pragma unroll
            for (int R = 0; R < 20; ++R) {
                own[R] = slab.at(p, R);
                occ[R] = slab.at(4, R);
            }
            derive_rows(own, occ, (m.first >> p) & 1u, p, P);
        }
#pragma unroll
        for (int R = 0; R < 20; ++R) rows_lds[R * WAVE] = make_uint2(P.b(R), P.c(R));
        const bool staged = tmask < 16u * DMA_RUNS;  // uniform: one search per wave
        if (!ML_LDS && staged) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the table's last stores have landed
            if (lane < 16)  // 16 lanes x 16 bytes = the 128-slot table
                __builtin_amdgcn_global_load_lds((const void*)(L->A.s.key[p] + 8 * lane), (void*)coop_stage[wv], 16, 0, 0);
        }
        // (ML_LDS: the table itself, in LDS, is the stage)
        int16_t* const stage_w = ML_LDS ? L->A.s.key[p] : coop_stage[wv];
        const uint32_t avail = ~m.used.get(p) & 0x1FFFFFu;
        const bool hroll = HEUR && m.mode == MC_ROLLOUT;
        // Board.move_count of the rollout board: placements on the way from the root
        const int edge_w = root_mc + m.depth + m.plies < 30 ? 6 : 3;
        uint32_t h_pre0 = 0u, h_pre1 = 0u;  // the heuristic draw's two MT words, loaded early
        if (hroll && m.mt_pos + 2u <= (uint32_t)FM_N) {
            const uint32_t* st = a.mt + (size_t)m.game * (FM_N + 1);
            h_pre0 = st[m.mt_pos];
            h_pre1 = st[m.mt_pos + 1u];
        }
        SECT(1);
        uint32_t cnt[2];
        double es[2];
        uint32_t okA[20], okB[20];  // hroll: this lane's orientations' legal rows (balanced pass)
        int og[2];
        const uint32_t nlive = coop_live_orients(avail, lane, coop_rank[wv], og);
        if (hroll) coop_ok_counts(rows_lds, og, nlive, okA, okB, cnt);
        else coop_orients<false>(rows_lds, og, nlive, hs, edge_w, cnt, es);
        const CoopScan sc = coop_scan(cnt, lane);
        const uint32_t total = sc.total;
        SECT(2);
        bk_mcts_node* pool = a.nodes + (size_t)m.game * a.cfg.node_cap;
        uint32_t k = 0;
        if (m.mode == MC_EXPAND) {
            bk_mcts_node* nd = pool + m.node;
            uint32_t n_legal = nd->n_legal, n_exp = nd->n_exp;
            if (!(nd->flags & BK_MCTS_NODE_EVALUATED)) {  // MCTSNode._initialize_untried_moves
                n_legal = total;
                nd->n_legal = (uint16_t)n_legal;
                nd->child0 = -1;
                nd->flags = BK_MCTS_NODE_EVALUATED;
            }
            if (n_legal != total) {  // an evaluated node's list cannot change
                m.status |= BK_MCTS_EINTERNAL;
                m.mode = MC_SELECT;
                continue;
            }
            if (n_legal == n_exp) {  // no legal move: terminal leaf
                mc_sim_terminal(a, m, L);
                continue;
            }
            k = n_legal - n_exp - 1u;  // untried_moves.pop(): the last list entry
        } else {
            if (total == 0u) {  // _rollout: no legal move -> break
                mc_complete(a, m, L, (double)(mc_score(m, m.player) - m.score0), false);
                continue;
            }
            if (!hroll) k = mc_randint(a.mt + (size_t)m.game * (FM_N + 1), m.mt_pos, total);
        }
        uint32_t kk = 0;
        int gs;
        double h_target = 0.0, h_R = 0.0, h_total = 0.0;
        uint32_t h_ok[20];
        bool h_unc = false;
        if (hroll) {
            uint32_t* st = a.mt + (size_t)m.game * (FM_N + 1);
#ifdef BK_SECTION_PROF
            auto cmark = [&](int i) { SECT(i); };
#else
            NoMark cmark;
#endif
            if (!a.coop_balanced ||
                !coop_heur_balanced(rows_lds - lane, my, lane, hs, edge_w, og, okA, okB, cnt, sc, st, m.mt_pos,
                                    h_pre0, h_pre1, h_target, h_R, h_total, h_unc, gs, h_ok, cmark)) {
                // more legal moves than the list holds: per-lane orientation sums
                es[0] = cnt[0] ? lane_orient_sum(og[0], okA, rows_lds, hs, edge_w) : 0.0;
                es[1] = cnt[1] ? lane_orient_sum(og[1], okB, rows_lds, hs, edge_w) : 0.0;
                gs = coop_heur_pick(es, og, lane, st, m.mt_pos, h_pre0, h_pre1, h_target, h_R, h_total, h_unc);
                if (gs >= 0) coop_ok_rows(gs, rows_lds, lane, h_ok);
            }
        } else {
            gs = coop_find(sc, og, k, kk);
        }
        FsLane* T = &L->A;  // the node board at expansion, the rollout's sim board after it
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA stage has landed
        const int16_t* tkey = staged ? stage_w : T->s.key[p];
        int ar, ac;
        SECT(3);
        int16_t* rank = coop_rank[wv];
        if (hroll) {
            if (gs < 0) {
                ar = -1;
                ac = 0;
            } else if (coop_walk_on) {
#pragma unroll
                for (int r = 0; r < 20; ++r) rows_lds[r * WAVE].y = h_ok[r];
                if (!coop_walk<true>(gs, 0u, rows_lds, tkey, (int)tmask, rank, lane, hs, edge_w, h_target,
                                     h_R, h_total, ar, ac, h_unc, reinterpret_cast<uint16_t*>(my + COOP_ML_DWORD)))
                    heur_walk_frontier(gs, h_ok, rows_lds, tkey, (int)tmask, hs, edge_w, h_target, h_R,
                                       h_total, ar, ac, h_unc);
            } else {
                heur_walk_frontier(gs, h_ok, rows_lds, tkey, (int)tmask, hs, edge_w, h_target, h_R, h_total,
                                   ar, ac, h_unc);
            }
            if (h_unc) m.status |= BK_MCTS_EUNCERT;
        } else {
            bool walked = false;
            if (coop_walk_on && tmask <= 2 * WAVE - 1) {
                bool unc_unused = false;
                uint32_t okr[20];
                coop_ok_rows(gs, rows_lds, lane, okr);  // locate_pass1 for the wave's one orientation
#pragma unroll
                for (int r = 0; r < 20; ++r) rows_lds[r * WAVE].y = okr[r];
                walked = coop_walk<false>(gs, kk, rows_lds, tkey, (int)tmask, rank, lane, hs, 0, 0.0, 0.0,
                                          0.0, ar, ac, unc_unused);
            }
            if (!walked) locate_move_frontier(gs, kk, rows_lds, tkey, (int)tmask, ar, ac);
        }
        if (ar < 0) {  // the table does not list the move: counts and tables disagree
            m.status |= BK_MCTS_EINTERNAL;
            m.mode = MC_SELECT;
            continue;
        }
        SECT(4);
        uint32_t pm[5];
        int32_t cells[5];
        piece_cells(gs, ar, ac, pm, cells);
        const uint64_t real = frontier_ops(rows_lds, slab, p, (m.first >> p) & 1u, gs, ar, ac, pm);
        SECT(8);
        const bool expand = m.mode == MC_EXPAND;
        uint32_t c = 0;
        bool ok = true;
        if (expand) {
            bk_mcts_node* nd = pool + m.node;
            const int32_t cs = mc_child_slot(pool, nd, m, a.cfg.node_cap);
            if (cs < 0) { m.status |= BK_MCTS_EPOOL; m.mode = MC_SELECT; continue; }
            c = (uint32_t)cs;
            nd->n_exp = (uint16_t)(nd->n_exp + 1u);
            bk_mcts_node ch;
            ch.total = 0.0; ch.visits = 0; ch.child0 = -1;
            ch.move = (uint16_t)(gs * 400 + ar * 20 + ac);
            ch.n_exp = 0; ch.n_legal = 0; ch.flags = 0;
            pool[c] = ch;
            if (m.depth >= BK_MCTS_MAX_DEPTH) { m.status |= BK_MCTS_EPATH; m.mode = MC_SELECT; continue; }
        }
        int16_t* sq = staged ? stage_w : nullptr;
        bool inpl = false;
        if constexpr (ML_LDS) {
            if (staged && expand) {  // the expansion's copy needs the table as a separate stage
                if (lane < 16)
                    reinterpret_cast<uint4*>(coop_stage[wv])[lane] = reinterpret_cast<const uint4*>(T->s.key[p])[lane];
                sq = coop_stage[wv];
            } else {
                inpl = staged;
            }
        }
#ifdef BK_SECTION_PROF
        // 9 slab rows, 10 set ops, 11 write-back / copy
        auto pmark = [&](int i) { SECT(i == 4 ? 9 : 10); };
#else
        NoMark pmark;
#endif
        if (expand) ok &= mc_place_staged<true, 2>(m, slab, p, gs, ar, &L->A, htab, pm, cells, real, lk, sq, pmark, inpl);
        else ok &= mc_place_staged<false, 2>(m, slab, p, gs, ar, &L->A, htab, pm, cells, real, lk, sq, pmark, inpl);
        SECT(11);
        if (expand) {
            if (!ok) { m.status |= BK_MCTS_EFSET; m.mode = MC_SELECT; continue; }
            const uint64_t* Z = a.zobrist + (size_t)a.zidx[m.game] * MC_ZOB;
            m.hash = mc_hash_step(Z, m.hash, p, (m.root_cp + m.depth) & 3, gs, ar, ac);
            L->path[++m.depth] = (int32_t)c;
            m.node = (int32_t)c;
            double reward = 0.0;
            if (a.cfg.use_tt && mc_tt_lookup(a, m, reward)) {
                mc_complete(a, m, L, reward, true);
                continue;
            }
            m.player = m.cur = (m.root_player + m.depth) & 3;
            m.score0 = mc_score(m, m.player);
            m.plies = 0;
            m.mode = MC_ROLLOUT;
        } else {
            if (!ok) { m.status |= BK_MCTS_EFSET; m.mode = MC_SELECT; continue; }
            m.plies++;
            m.rplies++;
            m.cur = (m.cur + 1) & 3;
            if (m.plies >= a.cfg.max_rollout_moves)
                mc_complete(a, m, L, (double)(mc_score(m, m.player) - m.score0), false);
        }
    }
    SECT_FLUSH;
}

#if BK_DEF(BK_U_COOP)
__global__ __launch_bounds__(COOP_WAVES * WAVE) void k_mcts_coop(MctsArgs a) { mcts_coop_body<false>(a); }
#else
__global__ void k_mcts_coop(MctsArgs a);
#endif
#if BK_DEF(BK_U_COOP_H)
__global__ __launch_bounds__(COOP_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(1)))
void k_mcts_coop_h(MctsArgs a) { mcts_coop_body<true>(a); }
#else
__global__ void k_mcts_coop_h(MctsArgs a);
#endif

#if BK_DEF(BK_U_HOST)
// ------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------
struct bk_handle_s {
    int device = 0;
    hipStream_t own = nullptr, cur = nullptr;
    std::vector<hipStream_t> extra;  // bk_stream_create's streams, destroyed with the handle
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    char err[512] = {0};
    // device staging / scratch
    void* d_in = nullptr; size_t d_in_cap = 0;
    void* d_out = nullptr; size_t d_out_cap = 0;
    void* d_aux = nullptr; size_t d_aux_cap = 0;
    void* d_aux2 = nullptr; size_t d_aux2_cap = 0;
    void* d_slab = nullptr; size_t d_slab_cap = 0;
    void* d_fin = nullptr; size_t d_fin_cap = 0;     // frontier: root tables
    void* d_fout = nullptr; size_t d_fout_cap = 0;   // frontier: advanced tables
    void* d_fslab = nullptr; size_t d_fslab_cap = 0; // frontier: per-slot records
    void* d_mc = nullptr; size_t d_mc_cap = 0;       // bk_mcts: staged inputs/outputs
    void* d_mclane = nullptr; size_t d_mclane_cap = 0; // bk_mcts: per-slot records
    void* d_rh = nullptr; size_t d_rh_cap = 0;       // bk_mcts: root hashes computed on the device
    void* d_step = nullptr; size_t d_step_cap = 0;   // bk_arena_step: staged extras
    uint32_t* d_counter = nullptr;
    uint32_t* d_diag = nullptr;        // bk_mcts failure record (mc_diag), sticky until reported
    void* d_started = nullptr; size_t d_started_cap = 0;  // bk_mcts: searches started (mc_mark_started)
    uint64_t* mcts_done = nullptr;  // bk_mcts_set_done: per-search result words
    void* d_mtwork = nullptr; size_t d_mtwork_cap = 0;  // BK_MCTS_STATE_ROWS: the searches' MT copies
    uint32_t diag_host[BK_DIAG_WORDS] = {0};  // the last record bk_synchronize reported
    bool diag_seen = false;
    uint32_t mcts_launches = 0;
    int num_cu = 0;
    int rollout_blocks_per_cu = 0;
    int fr_blocks_per_cu = 0;    // k_rollout_fr
    int mcts_blocks_per_cu = 0;  // k_mcts
    const char* last_kernel = "";  // name of the kernel the last timed call launched
    // tuning / test overrides (bk_set_tuning; read from the environment once, in bk_create)
    int64_t tune[BK_TUNE_COUNT];
    // an asynchronous bk_mcts search is running on `busy_stream` with this handle's scratch
    bool busy = false;
    hipStream_t busy_stream = nullptr;
    bool capturing = false;  // the current launch goes into a graph being captured (untimed)
};

static const char* const kTuneNames[BK_TUNE_COUNT] = {
    "BK_MG_GROUPS", "BK_MG_STAGE", "BK_MG_PARTS", "BK_MG_PART_WAVES", "BK_DEBUG_MAX_ITERS", "BK_HANDOUT",
    "BK_MCTS_COOP", "BK_COOP_BLOCKS_PER_CU", "BK_MCTS_SPREAD", "BK_TREE_BATCH", "BK_COOP_WALK", "BK_COOP_BAL",
    "BK_MCTS_PAIR"};

// the tuning value for key, or dflt when automatic (-1)
static inline int64_t tune_or(const bk_handle_s* h, int key, int64_t dflt) {
    return h->tune[key] < 0 ? dflt : h->tune[key];
}

#ifdef BK_SECTION_PROF
static std::vector<int (*)(unsigned long long*, int)>& sect_readers() {
    static std::vector<int (*)(unsigned long long*, int)> v;
    return v;
}
void bk_register_sections(int (*rd)(unsigned long long*, int)) { sect_readers().push_back(rd); }
#endif

static int set_err(bk_handle h, int code, const char* fmt, const char* detail) {
    if (h) snprintf(h->err, sizeof h->err, fmt, detail ? detail : "");
    return code;
}

#define HIPCHK(h, call)                                                                 \
    do {                                                                                \
        hipError_t _e = (call);                                                         \
        if (_e != hipSuccess) return set_err((h), BK_EHIP, #call ": %s", hipGetErrorString(_e)); \
    } while (0)

// A host-memory launch reports its own device error synchronously, so it clears only its
// own sticky bit (`own`): any other bit still pending from an earlier device-path launch on
// the handle (BK_STICKY_GUARD / _ROOT / _FASTMCTS) stays for bk_synchronize to report
// (clearing the whole word lost them).
static int clear_own_sticky(bk_handle h, uint32_t sticky, uint32_t own) {
    if (!(sticky & own)) return BK_OK;
    const uint32_t rest = sticky & ~own;
    HIPCHK(h, hipMemcpyAsync(h->d_counter + 2, &rest, sizeof rest, hipMemcpyHostToDevice, h->cur));
    HIPCHK(h, hipStreamSynchronize(h->cur));
    return BK_OK;
}

// every launching entry point: the handle's scratch may be in use by an asynchronous
// bk_mcts search (BK_MCTS_ASYNC) until bk_synchronize
#define BK_IDLE(h, name)                                                                \
    do {                                                                                \
        if ((h)->busy)                                                                  \
            return set_err((h), BK_EINVAL, name ": an asynchronous bk_mcts search is still running on " \
                                           "this handle (bk_synchronize first)%s", "");  \
    } while (0)

// A pending bk_mcts failure record (mc_diag) moves to the host copy and is reported once
// as BK_ECHECK; bk_debug_mcts_failure returns it afterwards.
static int take_diag(bk_handle h) {
    uint32_t rec[BK_DIAG_WORDS];
    HIPCHK(h, hipMemcpyAsync(rec, h->d_diag, sizeof rec, hipMemcpyDeviceToHost, h->cur));
    HIPCHK(h, hipStreamSynchronize(h->cur));
    if (!rec[0]) return BK_OK;
    HIPCHK(h, hipMemsetAsync(h->d_diag, 0, sizeof rec, h->cur));
    HIPCHK(h, hipStreamSynchronize(h->cur));
    memcpy(h->diag_host, rec, sizeof rec);
    h->diag_seen = true;
    char msg[256];
    if (rec[0] == BK_DIAG_DOUBLE_START)
        snprintf(msg, sizeof msg, "search %u of launch %u (kernel %u) was started twice (second start by block %u wave "
                 "%u, hw_id 0x%x, hand-out counter %u, %u searches)", rec[3], rec[2], rec[1], rec[18], rec[19], rec[20],
                 rec[12], rec[21]);
    else
        snprintf(msg, sizeof msg, "search %u of launch %u (kernel %u) broke a tree invariant (status %u): node %u has "
                 "%u visits after %u iterations (log_len %u, n_exp %u, n_legal %u)", rec[3], rec[2], rec[1], rec[0],
                 rec[4], rec[5], rec[9], rec[11], rec[6], rec[7]);
    return set_err(h, BK_ECHECK, "bk_mcts: %s; bk_debug_mcts_failure has the record", msg);
}

// A handle's scratch grows in stream order on the handle's current stream
// (hipFreeAsync / hipMallocAsync): hipFree would wait for the whole device, stalling
// every other stream's launches (the arena's search streams regrow as job sizes vary).
static int grow(bk_handle h, void** p, size_t* cap, size_t need) {
    if (need <= *cap) return BK_OK;
    if (*p) (void)hipFreeAsync(*p, h->cur);
    *p = nullptr; *cap = 0;
    size_t n = need + need / 2 + 256;
    HIPCHK(h, hipMallocAsync(p, n, h->cur));
    *cap = n;
    return BK_OK;
}

extern "C" {

int bk_abi_version(void) { return BK_ABI_VERSION; }
int bk_tables_version(void) { return BK_TABLES_VERSION; }

int bk_orient_info(int g, int32_t* piece_id, int32_t* orient, int32_t* ncells, int32_t* offs) {
    if (g < 0 || g >= BK_NUM_ORIENTS || !piece_id || !orient || !ncells || !offs) return BK_EINVAL;
    *piece_id = (int32_t)(kOrientInfoHost[g] & 0xFF);
    *orient = kOrientIndexHost[g];
    *ncells = (int32_t)((kOrientInfoHost[g] >> 8) & 0xFF);
    for (int k = 0; k < 5; ++k) {
        offs[2 * k] = (int32_t)(kOrientCellsHost[g][k] >> 8);
        offs[2 * k + 1] = (int32_t)(kOrientCellsHost[g][k] & 0xFF);
    }
    return BK_OK;
}

int bk_create(int device, uint32_t flags, bk_handle* out) {
    (void)flags;
    if (!out) return BK_EINVAL;
    *out = nullptr;
    bk_handle h = new (std::nothrow) bk_handle_s();
    if (!h) return BK_ENOMEM;
    h->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&h->ev0);
    if (e == hipSuccess) e = hipEventCreate(&h->ev1);
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_counter, 4 * sizeof(uint32_t));
    // The handle's device words are zeroed on its own stream and waited for HERE.  A plain
    // hipMemset runs on the legacy null stream, which is not ordered with the
    // non-blocking streams launches go to (torch's, bk_set_stream): under load it could
    // land after the handle's first kernel had started and reset its hand-out counter
    // mid-launch, handing searches out twice (the round-4 / round-6 BK_MCTS_ELOG failures,
    // DESIGN.md 4).  No entry point touches device memory on the null stream.
    if (e == hipSuccess) e = hipMemsetAsync(h->d_counter, 0, 4 * sizeof(uint32_t), h->own);
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_diag, BK_DIAG_WORDS * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemsetAsync(h->d_diag, 0, BK_DIAG_WORDS * sizeof(uint32_t), h->own);
    if (e == hipSuccess) e = hipStreamSynchronize(h->own);
    hipDeviceProp_t prop;
    if (e == hipSuccess) e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) {
        fprintf(stderr, "bk_create: %s\n", hipGetErrorString(e));
        delete h;
        return BK_EHIP;
    }
    h->num_cu = prop.multiProcessorCount;
    for (int k = 0; k < BK_TUNE_COUNT; ++k) {  // the only place the environment is read
        const char* env = getenv(kTuneNames[k]);
        h->tune[k] = env && *env ? (int64_t)strtoll(env, nullptr, 10) : -1;
    }
    int bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k_rollout, BLOCK, 0) != hipSuccess || bpc < 1) bpc = 1;
    h->rollout_blocks_per_cu = bpc;
    if (const char* env = getenv("BK_BLOCKS_PER_CU")) {  // tuning override
        const int v = atoi(env);
        if (v > 0 && v < bpc) h->rollout_blocks_per_cu = v;
    }
    // resident blocks of the frontier-order kernels, from their real register / LDS use
    bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k_rollout_fr, BLOCK, 0) != hipSuccess || bpc < 1) bpc = 1;
    h->fr_blocks_per_cu = bpc;
    bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k_mcts, BLOCK, 0) != hipSuccess || bpc < 1) bpc = 1;
    h->mcts_blocks_per_cu = bpc;
    if (const char* env = getenv("BK_FR_BLOCKS_PER_CU")) {  // tuning override (both kernels)
        const int v = atoi(env);
        if (v > 0 && v < h->fr_blocks_per_cu) h->fr_blocks_per_cu = v;
        if (v > 0 && v < h->mcts_blocks_per_cu) h->mcts_blocks_per_cu = v;
    }
    h->cur = h->own;
    *out = h;
    return BK_OK;
}

int bk_destroy(bk_handle h) {
    if (!h) return BK_EINVAL;
    (void)hipSetDevice(h->device);
    if (h->busy) (void)hipStreamSynchronize(h->busy_stream);
    if (h->own) (void)hipStreamSynchronize(h->own);
    void* bufs[] = {h->d_in, h->d_out, h->d_aux, h->d_aux2, h->d_slab, h->d_fin, h->d_fout, h->d_fslab,
                    h->d_mc, h->d_mclane, h->d_step, h->d_counter, h->d_rh, h->d_diag, h->d_started, h->d_mtwork};
    for (void* b : bufs) if (b) (void)hipFree(b);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->own) (void)hipStreamDestroy(h->own);
    for (hipStream_t x : h->extra) (void)hipStreamDestroy(x);
    delete h;
    return BK_OK;
}

int bk_stream_create(bk_handle h, const uint32_t* cu_mask, int32_t mask_words, void** out_stream) {
    if (!h || !out_stream || mask_words < 0 || (mask_words > 0 && !cu_mask))
        return set_err(h, BK_EINVAL, "bk_stream_create: invalid arguments%s", "");
    HIPCHK(h, hipSetDevice(h->device));
    hipStream_t st = nullptr;
    if (mask_words > 0) {
        HIPCHK(h, hipExtStreamCreateWithCUMask(&st, (uint32_t)mask_words, cu_mask));
    } else {
        HIPCHK(h, hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    }
    h->extra.push_back(st);
    *out_stream = (void*)st;
    return BK_OK;
}

int bk_set_stream(bk_handle h, void* stream) {
    if (!h) return BK_EINVAL;
    h->cur = (stream == BK_STREAM_OWN) ? h->own : (hipStream_t)stream;
    return BK_OK;
}

int bk_synchronize(bk_handle h) {
    if (!h) return BK_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    if (h->busy) {  // the asynchronous search's stream (bk_set_stream may have moved h->cur)
        HIPCHK(h, hipStreamSynchronize(h->busy_stream));
        h->busy = false;
        h->busy_stream = nullptr;
    }
    HIPCHK(h, hipStreamSynchronize(h->cur));
    if (int rc = take_diag(h)) return rc;
    uint32_t sticky = 0;
    HIPCHK(h, hipMemcpyAsync(&sticky, h->d_counter + 2, sizeof sticky, hipMemcpyDeviceToHost, h->cur));
    HIPCHK(h, hipStreamSynchronize(h->cur));
    if (sticky) {
        HIPCHK(h, hipMemsetAsync(h->d_counter + 2, 0, sizeof sticky, h->cur));
        HIPCHK(h, hipStreamSynchronize(h->cur));
        if (sticky & BK_STICKY_GUARD)
            return set_err(h, BK_EOVERFLOW, "device-path launch: iteration guard tripped, results incomplete%s", "");
        if (sticky & BK_STICKY_FASTMCTS)
            return set_err(h, BK_EINVAL, "device-path bk_fastmcts: a root with more than BK_FASTMCTS_MAX_CHILDREN "
                                         "children or iterations past the log table (its output is not set)%s", "");
        return set_err(h, BK_EINVAL, "device-path launch: root_index entry outside [0, n_roots)%s", "");
    }
    return BK_OK;
}

int bk_debug_mcts_failure(bk_handle h, uint32_t* out, int32_t n) {
    if (!h || !out || n < 1) return BK_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    if (!h->busy) {  // a record still on the device (nobody synchronized since): take it now
        HIPCHK(h, hipStreamSynchronize(h->cur));
        (void)take_diag(h);
    }
    const int32_t k = n < BK_DIAG_WORDS ? n : BK_DIAG_WORDS;
    for (int32_t i = 0; i < n; ++i) out[i] = i < k && h->diag_seen ? h->diag_host[i] : 0u;
    return h->diag_seen ? 1 : 0;
}

int bk_mcts_set_done(bk_handle h, uint64_t* done) {
    if (!h) return BK_EINVAL;
    h->mcts_done = done;
    return BK_OK;
}

void* bk_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0 || hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
    memset(p, 0, bytes);
    return p;
}

int bk_host_free(void* p) {
    if (!p) return BK_OK;
    return hipHostFree(p) == hipSuccess ? BK_OK : BK_EHIP;
}

int bk_last_error(bk_handle h, char* buf, size_t len) {
    if (!h || !buf || len == 0) return BK_EINVAL;
    snprintf(buf, len, "%s", h->err);
    return BK_OK;
}

int bk_set_tuning(bk_handle h, int32_t key, int64_t value) {
    if (!h || key < 0 || key >= BK_TUNE_COUNT || value < -1)
        return set_err(h, BK_EINVAL, "bk_set_tuning: unknown key or value < -1%s", "");
    h->tune[key] = value;
    return BK_OK;
}

int bk_get_tuning(bk_handle h, int32_t key, int64_t* value) {
    if (!h || !value || key < 0 || key >= BK_TUNE_COUNT) return set_err(h, BK_EINVAL, "bk_get_tuning: bad key%s", "");
    *value = h->tune[key];
    return BK_OK;
}

int bk_debug_sections(bk_handle h, uint64_t* out, int32_t n, int32_t reset) {
    if (!h || !out || n < 1) return BK_EINVAL;
#ifdef BK_SECTION_PROF
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->cur));
    unsigned long long v[BK_NSECT] = {0};
    for (auto rd : sect_readers())  // every unit's own counters, summed
        if (rd(v, reset) != 0) return set_err(h, BK_EHIP, "bk_debug_sections: counter copy failed%s", "");
    for (int i = 0; i < n; ++i) out[i] = i < BK_NSECT ? (uint64_t)v[i] : 0u;
    return BK_OK;
#else
    (void)reset;
    for (int i = 0; i < n; ++i) out[i] = 0u;
    return set_err(h, BK_EINVAL, "bk_debug_sections: library built without -DBK_SECTION_PROF%s", "");
#endif
}

const char* bk_last_kernel(bk_handle h) { return h ? h->last_kernel : ""; }

int bk_last_kernel_ms(bk_handle h, float* ms) {
    if (!h || !ms) return BK_EINVAL;
    if (!h->timed) return set_err(h, BK_EINVAL, "no timed kernel on this handle%s", "");
    HIPCHK(h, hipEventSynchronize(h->ev1));
    HIPCHK(h, hipEventElapsedTime(ms, h->ev0, h->ev1));
    return BK_OK;
}

// HIP events around a launch (bk_last_kernel_ms).  Not while the stream is being captured
// into a graph (hipStreamBeginCapture: the caller times the graph's replays itself): the
// launches then go into the graph untimed, and bk_last_kernel_ms reports the last timed one.
static hipError_t mark_start(bk_handle h) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    const hipError_t e = hipStreamIsCapturing(h->cur, &st);
    if (e != hipSuccess) return e;
    h->capturing = st != hipStreamCaptureStatusNone;
    return h->capturing ? hipSuccess : hipEventRecord(h->ev0, h->cur);
}
static hipError_t mark_end(bk_handle h) {
    if (h->capturing) return hipSuccess;
    const hipError_t e = hipEventRecord(h->ev1, h->cur);
    if (e == hipSuccess) h->timed = true;
    return e;
}

static int stage_in(bk_handle h, const void* src, size_t bytes, int mem, void** dev, void** buf, size_t* cap) {
    if (mem == BK_MEM_DEVICE) { *dev = const_cast<void*>(src); return BK_OK; }
    int rc = grow(h, buf, cap, bytes);
    if (rc) return rc;
    HIPCHK(h, hipMemcpyAsync(*buf, src, bytes, hipMemcpyHostToDevice, h->cur));
    *dev = *buf;
    return BK_OK;
}

int bk_movegen(bk_handle h, const bk_state* states, const uint8_t* players, int32_t n, uint32_t* out_rows,
               uint32_t* out_count, int mem) {
    if (!h || !states || !players || n < 0 || (mem != BK_MEM_HOST && mem != BK_MEM_DEVICE))
        return set_err(h, BK_EINVAL, "bk_movegen: invalid arguments%s", "");
    if (n == 0) return BK_OK;
    HIPCHK(h, hipSetDevice(h->device));
    BK_IDLE(h, "bk_movegen");
    void *d_states, *d_players;
    int rc = stage_in(h, states, sizeof(bk_state) * (size_t)n, mem, &d_states, &h->d_in, &h->d_in_cap);
    if (rc) return rc;
    rc = stage_in(h, players, (size_t)n, mem, &d_players, &h->d_aux, &h->d_aux_cap);
    if (rc) return rc;
    uint32_t* d_rows = out_rows;
    uint32_t* d_count = out_count;
    const size_t rows_bytes = sizeof(uint32_t) * (size_t)n * BK_NUM_ORIENTS * 20;
    if (mem == BK_MEM_HOST) {
        rc = grow(h, &h->d_out, &h->d_out_cap, (out_rows ? rows_bytes : 0) + sizeof(uint32_t) * (size_t)n);
        if (rc) return rc;
        d_count = (uint32_t*)h->d_out;
        d_rows = out_rows ? (uint32_t*)((char*)h->d_out + sizeof(uint32_t) * (size_t)n + 0) : nullptr;
        // keep 16-byte alignment of the rows block
        if (d_rows) d_rows = (uint32_t*)(((uintptr_t)d_rows + 15) & ~(uintptr_t)15);
        if (d_rows) { rc = grow(h, &h->d_out, &h->d_out_cap, rows_bytes + sizeof(uint32_t) * (size_t)n + 16);
                      if (rc) return rc;
                      d_count = (uint32_t*)h->d_out;
                      d_rows = (uint32_t*)(((uintptr_t)((char*)h->d_out + sizeof(uint32_t) * (size_t)n) + 15) & ~(uintptr_t)15); }
    } else if (out_rows && ((uintptr_t)out_rows & 15)) {
        return set_err(h, BK_EINVAL, "bk_movegen: out_rows must be 16-byte aligned%s", "");
    }
    // orientation groups: about 4 waves per CU, at least 8 groups (measured best at 4,096
    // and 16,384 board-players, profiles/r02/sweeps/movegen_groups.jsonl)
    const int waves = (n + WAVE - 1) / WAVE;
    int groups = (4 * h->num_cu + waves - 1) / waves;
    groups = groups < 8 ? 8 : (groups > MG_GROUPS_DEFAULT_MAX ? MG_GROUPS_DEFAULT_MAX : groups);
    groups = (int)tune_or(h, BK_TUNE_MG_GROUPS, groups);
    if (groups < 1) groups = 1;
    if (groups > MG_GROUPS_MAX) groups = MG_GROUPS_MAX;
    MovegenArgs a{(const bk_state*)d_states, (const uint8_t*)d_players, n, d_rows, d_count, nullptr, groups, nullptr};
    if (d_count) HIPCHK(h, hipMemsetAsync(d_count, 0, sizeof(uint32_t) * (size_t)n, h->cur));  // atomics add in
    const int grid = waves * groups;
    HIPCHK(h, mark_start(h));
    h->last_kernel = "k_movegen_g";
    hipLaunchKernelGGL(k_movegen_g, dim3(grid), dim3(WAVE), 0, h->cur, a);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, mark_end(h));
    if (mem == BK_MEM_HOST) {
        if (out_count) HIPCHK(h, hipMemcpyAsync(out_count, d_count, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, h->cur));
        if (out_rows) HIPCHK(h, hipMemcpyAsync(out_rows, d_rows, rows_bytes, hipMemcpyDeviceToHost, h->cur));
        HIPCHK(h, hipStreamSynchronize(h->cur));
    }
    return BK_OK;
}

int bk_movegen_mask(bk_handle h, const bk_state* states, const uint8_t* players, int32_t n, uint64_t* out_mask,
                    uint32_t* out_count, int mem) {
    if (!h || !states || !players || n < 0 || (mem != BK_MEM_HOST && mem != BK_MEM_DEVICE))
        return set_err(h, BK_EINVAL, "bk_movegen_mask: invalid arguments%s", "");
    if (n == 0) return BK_OK;
    if (mem == BK_MEM_DEVICE && out_mask && ((uintptr_t)out_mask & 7))
        return set_err(h, BK_EINVAL, "bk_movegen_mask: out_mask must be 8-byte aligned%s", "");
    HIPCHK(h, hipSetDevice(h->device));
    BK_IDLE(h, "bk_movegen_mask");
    void *d_states, *d_players;
    int rc = stage_in(h, states, sizeof(bk_state) * (size_t)n, mem, &d_states, &h->d_in, &h->d_in_cap);
    if (rc) return rc;
    rc = stage_in(h, players, (size_t)n, mem, &d_players, &h->d_aux, &h->d_aux_cap);
    if (rc) return rc;
    uint64_t* d_mask = out_mask;
    uint32_t* d_count = out_count;
    const size_t mask_bytes = sizeof(uint64_t) * 7 * BK_NUM_ORIENTS * (size_t)n;
    if (mem == BK_MEM_HOST) {
        const size_t cb = (sizeof(uint32_t) * (size_t)n + 15) & ~(size_t)15;
        rc = grow(h, &h->d_out, &h->d_out_cap, cb + (out_mask ? mask_bytes : 0));
        if (rc) return rc;
        d_count = (uint32_t*)h->d_out;
        d_mask = out_mask ? (uint64_t*)((char*)h->d_out + cb) : nullptr;
    }
    // groups as bk_movegen; sets of 64 board-players rounded up to a multiple of the XCDs
    const int waves = (n + WAVE - 1) / WAVE;
    int groups = (4 * h->num_cu + waves - 1) / waves;
    groups = groups < 8 ? 8 : (groups > MG_GROUPS_DEFAULT_MAX ? MG_GROUPS_DEFAULT_MAX : groups);
    groups = (int)tune_or(h, BK_TUNE_MG_GROUPS, groups);
    if (groups < 1) groups = 1;
    if (groups > MG_GROUPS_MAX) groups = MG_GROUPS_MAX;
    const int sets = ((waves + MG_XCDS - 1) / MG_XCDS) * MG_XCDS;
    MovegenArgs a{(const bk_state*)d_states, (const uint8_t*)d_players, n, nullptr, d_count, nullptr, groups, d_mask};
    if (d_count) HIPCHK(h, hipMemsetAsync(d_count, 0, sizeof(uint32_t) * (size_t)n, h->cur));  // atomics add in
    HIPCHK(h, mark_start(h));
    // LDS-staged whole-line writes (k_movegen_ml): the groups' waves split over MG_PARTS
    // orientation ranges of one set each; BK_MG_STAGE=0 keeps the per-lane stores
    bool staged = out_mask != nullptr;
    staged = staged && tune_or(h, BK_TUNE_MG_STAGE, 1) != 0;
    if (staged) {
        int parts = (int)tune_or(h, BK_TUNE_MG_PARTS, 4);  // 4, 5, 7 or 13
        if (parts != 5 && parts != 7 && parts != 13) parts = 4;
        int wp = (int)tune_or(h, BK_TUNE_MG_PART_WAVES, groups / parts);
        wp = wp < 1 ? 1 : (wp > MG_PART_WAVES_MAX ? MG_PART_WAVES_MAX : wp);
        const dim3 grid(sets * parts), blk(wp * WAVE);
        static const uint32_t kClassHost[BK_NUM_ORIENTS][2] = BK_CLASS_TABLE_INIT;
        memset(a.part_masks, 0, sizeof a.part_masks);
        for (int i = 0; i < BK_NUM_ORIENTS; ++i) {
            const int g = (int)(kClassHost[i][0] >> 8);
            int q = 0;
            while ((q + 1) * BK_NUM_ORIENTS / parts <= g) ++q;  // range q: [q 91 / parts, (q + 1) 91 / parts)
            a.part_masks[q][i >> 5] |= 1u << (i & 31);
        }
        if (parts == 4) {
            h->last_kernel = "k_movegen_ml4";
            hipLaunchKernelGGL(k_movegen_ml4, grid, blk, 0, h->cur, a);
        } else if (parts == 5) {
            h->last_kernel = "k_movegen_ml5";
            hipLaunchKernelGGL(k_movegen_ml5, grid, blk, 0, h->cur, a);
        } else if (parts == 7) {
            h->last_kernel = "k_movegen_ml7";
            hipLaunchKernelGGL(k_movegen_ml7, grid, blk, 0, h->cur, a);
        } else {
            h->last_kernel = "k_movegen_ml13";
            hipLaunchKernelGGL(k_movegen_ml13, grid, blk, 0, h->cur, a);
        }
    } else {
        h->last_kernel = "k_movegen_m";
        hipLaunchKernelGGL(k_movegen_m, dim3(sets * groups), dim3(WAVE), 0, h->cur, a);
    }
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, mark_end(h));
    if (mem == BK_MEM_HOST) {
        if (out_count) HIPCHK(h, hipMemcpyAsync(out_count, d_count, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost, h->cur));
        if (out_mask) HIPCHK(h, hipMemcpyAsync(out_mask, d_mask, mask_bytes, hipMemcpyDeviceToHost, h->cur));
        HIPCHK(h, hipStreamSynchronize(h->cur));
    }
    return BK_OK;
}

int bk_has_moves(bk_handle h, const bk_state* states, int32_t n, uint8_t* out_mask4, int mem) {
    if (!h || !states || !out_mask4 || n < 0 || (mem != BK_MEM_HOST && mem != BK_MEM_DEVICE))
        return set_err(h, BK_EINVAL, "bk_has_moves: invalid arguments%s", "");
    if (n == 0) return BK_OK;
    HIPCHK(h, hipSetDevice(h->device));
    BK_IDLE(h, "bk_has_moves");
    void* d_states;
    int rc = stage_in(h, states, sizeof(bk_state) * (size_t)n, mem, &d_states, &h->d_in, &h->d_in_cap);
    if (rc) return rc;
    uint8_t* d_mask = out_mask4;
    if (mem == BK_MEM_HOST) {
        rc = grow(h, &h->d_out, &h->d_out_cap, (size_t)n);
        if (rc) return rc;
        d_mask = (uint8_t*)h->d_out;
    }
    MovegenArgs a{(const bk_state*)d_states, nullptr, n, nullptr, nullptr, d_mask, 0, nullptr};
    HIPCHK(h, mark_start(h));
    h->last_kernel = "k_has_moves";
    hipLaunchKernelGGL(k_has_moves, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, h->cur, a);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, mark_end(h));
    if (mem == BK_MEM_HOST) {
        HIPCHK(h, hipMemcpyAsync(out_mask4, d_mask, (size_t)n, hipMemcpyDeviceToHost, h->cur));
        HIPCHK(h, hipStreamSynchronize(h->cur));
    }
    return BK_OK;
}

static int launch_playouts(bk_handle h, const bk_state* roots, int32_t n_roots, const int32_t* root_index,
                           int32_t n_playouts, const bk_rollout_cfg* cfg, const uint32_t* compat_seeds,
                           bk_result* out, bk_state* out_states, int mem, const bk_fset* root_sets = nullptr,
                           bk_fset* out_sets = nullptr, const uint8_t* seat_masks = nullptr,
                           uint32_t* rng_io = nullptr, const uint8_t* quick_masks = nullptr,
                           const int32_t* forced = nullptr, bk_stop_info* stop_out = nullptr) {
    if (!h || !roots || !cfg || n_roots <= 0 || n_playouts < 0 || (mem != BK_MEM_HOST && mem != BK_MEM_DEVICE))
        return set_err(h, BK_EINVAL, "bk_rollout: invalid arguments%s", "");
    if (cfg->semantics != BK_SEM_ARENA && cfg->semantics != BK_SEM_ROLLOUT && cfg->semantics != BK_SEM_ADVANCE)
        return set_err(h, BK_EINVAL, "bk_rollout: unknown semantics%s", "");
    if ((cfg->semantics == BK_SEM_ADVANCE && !out_states) || (cfg->semantics == BK_SEM_ROLLOUT && out_states))
        return set_err(h, BK_EINVAL, "bk_rollout: out_states goes with BK_SEM_ADVANCE (or BK_SEM_ARENA)%s", "");
    if (!out && !out_states) return set_err(h, BK_EINVAL, "bk_rollout: no output%s", "");
    const bool fr = cfg->order == BK_ORDER_FRONTIER;
    if (cfg->order != BK_ORDER_NAIVE && !fr) return set_err(h, BK_EINVAL, "bk_rollout: unknown order%s", "");
    if (fr != (root_sets != nullptr))
        return set_err(h, BK_EINVAL, "bk_rollout: BK_ORDER_FRONTIER goes with root frontier sets "
                                     "(bk_rollout_frontier)%s", "");
    if (fr && (out_states != nullptr) != (out_sets != nullptr))
        return set_err(h, BK_EINVAL, "bk_rollout_frontier: out_sets goes with out_states%s", "");
    if (cfg->rng != BK_RNG_PHILOX && cfg->rng != BK_RNG_NUMPY_MT)
        return set_err(h, BK_EINVAL, "bk_rollout: unknown rng%s", "");
    if (cfg->rng == BK_RNG_NUMPY_MT && !compat_seeds && !rng_io)
        return set_err(h, BK_EINVAL, "bk_rollout: compat rng needs compat_seeds%s", "");
    if (cfg->max_plies <= 0) return set_err(h, BK_EINVAL, "bk_rollout: max_plies must be > 0%s", "");
    if ((cfg->heuristic_seats & ~0xF) || (cfg->heuristic_seats && !fr))
        return set_err(h, BK_EINVAL, "bk_rollout: heuristic_seats (4 bits) needs BK_ORDER_FRONTIER%s", "");
    if (n_playouts == 0) return BK_OK;
    HIPCHK(h, hipSetDevice(h->device));
    BK_IDLE(h, "bk_rollout");
    void *d_roots, *d_idx = nullptr, *d_seeds = nullptr;
    int rc = stage_in(h, roots, sizeof(bk_state) * (size_t)n_roots, mem, &d_roots, &h->d_in, &h->d_in_cap);
    if (rc) return rc;
    if (root_index) {
        if (mem == BK_MEM_HOST)
            for (int32_t i = 0; i < n_playouts; ++i)
                if (root_index[i] < 0 || root_index[i] >= n_roots)
                    return set_err(h, BK_EINVAL, "bk_rollout: root_index entry outside [0, n_roots)%s", "");
        rc = stage_in(h, root_index, sizeof(int32_t) * (size_t)n_playouts, mem, &d_idx, &h->d_aux, &h->d_aux_cap);
        if (rc) return rc;
    }
    if (cfg->rng == BK_RNG_NUMPY_MT && compat_seeds) {  // (bk_arena_advance carries cursors instead)
        rc = stage_in(h, compat_seeds, sizeof(uint32_t) * 4 * (size_t)n_playouts, mem, &d_seeds, &h->d_aux2,
                      &h->d_aux2_cap);
        if (rc) return rc;
    }
    void* d_rsets = nullptr;
    if (fr) {
        rc = stage_in(h, root_sets, sizeof(bk_fset) * (size_t)n_roots, mem, &d_rsets, &h->d_fin, &h->d_fin_cap);
        if (rc) return rc;
    }
    void *d_masks = nullptr, *d_rng = nullptr, *d_quick = nullptr, *d_forced = nullptr;
    bk_stop_info* d_stop = stop_out;
    if (seat_masks) {  // bk_arena_advance / bk_arena_step
        rc = stage_in(h, seat_masks, (size_t)n_playouts, mem, &d_masks, &h->d_aux, &h->d_aux_cap);
        if (rc) return rc;
        rc = stage_in(h, rng_io, sizeof(uint32_t) * 16 * (size_t)n_playouts, mem, &d_rng, &h->d_aux2, &h->d_aux2_cap);
        if (rc) return rc;
        // bk_arena_step's extras share one staging buffer (host mode): quick masks,
        // forced moves, stop infos at 16-byte aligned offsets
        const size_t qb = quick_masks ? ((size_t)n_playouts + 15) & ~(size_t)15 : 0;
        const size_t fb = forced ? (sizeof(int32_t) * (size_t)n_playouts + 15) & ~(size_t)15 : 0;
        const size_t sb = stop_out ? sizeof(bk_stop_info) * (size_t)n_playouts : 0;
        if (mem == BK_MEM_HOST && (qb + fb + sb)) {
            rc = grow(h, &h->d_step, &h->d_step_cap, qb + fb + sb);
            if (rc) return rc;
            char* base = (char*)h->d_step;
            if (quick_masks) {
                d_quick = base;
                HIPCHK(h, hipMemcpyAsync(d_quick, quick_masks, (size_t)n_playouts, hipMemcpyHostToDevice, h->cur));
            }
            if (forced) {
                d_forced = base + qb;
                HIPCHK(h, hipMemcpyAsync(d_forced, forced, sizeof(int32_t) * (size_t)n_playouts,
                                         hipMemcpyHostToDevice, h->cur));
            }
            if (stop_out) d_stop = (bk_stop_info*)(base + qb + fb);
        } else {
            d_quick = const_cast<uint8_t*>(quick_masks);
            d_forced = const_cast<int32_t*>(forced);
        }
    }
    bk_result* d_out = out;
    bk_state* d_states = out_states;
    bk_fset* d_osets = out_sets;
    if (mem == BK_MEM_HOST) {
        const size_t rb = out ? sizeof(bk_result) * (size_t)n_playouts : 0;
        const size_t sb = out_states ? sizeof(bk_state) * (size_t)n_playouts : 0;
        rc = grow(h, &h->d_out, &h->d_out_cap, rb + sb);
        if (rc) return rc;
        d_out = out ? (bk_result*)h->d_out : nullptr;
        d_states = out_states ? (bk_state*)((char*)h->d_out + rb) : nullptr;
        if (out_sets) {
            rc = grow(h, &h->d_fout, &h->d_fout_cap, sizeof(bk_fset) * (size_t)n_playouts);
            if (rc) return rc;
            d_osets = (bk_fset*)h->d_fout;
        }
    }
    // persistent grid: every resident slot pulls playouts from the counter
    const bool heur = fr && ((cfg->heuristic_seats & 0xF) != 0 || seat_masks != nullptr);
    const int blk = heur ? HBLOCK : BLOCK;
    int blocks = h->num_cu * (heur ? 3 : fr ? h->fr_blocks_per_cu : h->rollout_blocks_per_cu);
    const int need = (n_playouts + blk - 1) / blk;
    if (blocks > need) blocks = need;
    if (blocks < 1) blocks = 1;
    const uint32_t nslots = (uint32_t)blocks * blk;
    rc = grow(h, &h->d_slab, &h->d_slab_cap, sizeof(uint32_t) * SLAB_WORDS * (size_t)nslots);
    if (rc) return rc;
    if (fr) {
        rc = grow(h, &h->d_fslab, &h->d_fslab_cap, sizeof(FsLane) * (size_t)nslots);
        if (rc) return rc;
    }
    HIPCHK(h, hipMemsetAsync(h->d_counter, 0, 2 * sizeof(uint32_t), h->cur));  // [2] is sticky
    const uint64_t per_lane = ((uint64_t)n_playouts + nslots - 1) / nslots + 1;
    const uint64_t per_game = (cfg->semantics == BK_SEM_ROLLOUT ? (uint64_t)cfg->max_plies + 2u : 100u);
    uint64_t iters = 2 * per_lane * per_game + 64u;  // 2x: uneven hand-outs (handout 2)
    iters = (uint64_t)tune_or(h, BK_TUNE_DEBUG_MAX_ITERS, (int64_t)iters);  // tests: force the guard
    RolloutArgs a{(const bk_state*)d_roots, n_roots, (const int32_t*)d_idx, n_playouts, *cfg,
                  (const uint32_t*)d_seeds, d_out, (uint32_t*)h->d_slab, nslots, h->d_counter,
                  (uint32_t)(iters > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : iters), d_states,
                  (const bk_fset*)d_rsets, d_osets, fr ? (FsLane*)h->d_fslab : nullptr,
                  (const uint8_t*)d_masks, (uint32_t*)d_rng, fr ? 0 : 2, 0u};
    a.quick_masks = (const uint8_t*)d_quick;
    a.forced = (const int32_t*)d_forced;
    a.stop_out = d_stop;
    // Playout hand-out.  Config 3 has 1.33 playouts per resident slot: pulled per lane
    // from one counter (handout 0), the extra third lands on lanes of EVERY wave, and each
    // wave then runs a second playout length with a third of its lanes; given to whole
    // waves (2: slot s plays s first, then only the first slots -- whole waves, one per
    // SIMD -- pull the rest), the other waves finish and free their SIMD time.  57.0 M ->
    // 60.2 M playouts/s (profiles/r03/sweeps/handout.jsonl).  The frontier-order kernels
    // keep 0 (22.4 vs 21.5 M: their playout lengths vary more).  Results depend only on the
    // playout id, not on the slot (tests/test_gpu_parity.py slot independence).
    a.handout = (int)tune_or(h, BK_TUNE_HANDOUT, a.handout);
    if (a.handout < 0 || a.handout > 2) a.handout = 0;
    {
        const int64_t rest = (int64_t)n_playouts - (int64_t)nslots;
        int64_t ls = rest <= 0 ? 0 : rest >= (int64_t)nslots ? (int64_t)nslots : ((rest + WAVE - 1) / WAVE) * WAVE;
        a.long_slots = (uint32_t)ls;
    }
    HIPCHK(h, mark_start(h));
    if (heur) {
        h->last_kernel = "k_rollout_fr_h";
        hipLaunchKernelGGL(k_rollout_fr_h, dim3(blocks), dim3(HBLOCK), 0, h->cur, a);
    } else if (fr) {
        h->last_kernel = "k_rollout_fr";
        hipLaunchKernelGGL(k_rollout_fr, dim3(blocks), dim3(BLOCK), 0, h->cur, a);
    } else if (cfg->semantics == BK_SEM_ADVANCE) {
        h->last_kernel = "k_advance";
        hipLaunchKernelGGL(k_advance, dim3(blocks), dim3(BLOCK), 0, h->cur, a);
    } else {
        h->last_kernel = "k_rollout";
        hipLaunchKernelGGL(k_rollout, dim3(blocks), dim3(BLOCK), 0, h->cur, a);
    }
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, mark_end(h));
    if (mem == BK_MEM_HOST) {
        if (out)
            HIPCHK(h, hipMemcpyAsync(out, d_out, sizeof(bk_result) * (size_t)n_playouts, hipMemcpyDeviceToHost, h->cur));
        if (out_states)
            HIPCHK(h, hipMemcpyAsync(out_states, d_states, sizeof(bk_state) * (size_t)n_playouts,
                                     hipMemcpyDeviceToHost, h->cur));
        if (out_sets)
            HIPCHK(h, hipMemcpyAsync(out_sets, d_osets, sizeof(bk_fset) * (size_t)n_playouts,
                                     hipMemcpyDeviceToHost, h->cur));
        if (rng_io)
            HIPCHK(h, hipMemcpyAsync(rng_io, d_rng, sizeof(uint32_t) * 16 * (size_t)n_playouts,
                                     hipMemcpyDeviceToHost, h->cur));
        if (stop_out)
            HIPCHK(h, hipMemcpyAsync(stop_out, d_stop, sizeof(bk_stop_info) * (size_t)n_playouts,
                                     hipMemcpyDeviceToHost, h->cur));
        uint32_t ctr[4];
        HIPCHK(h, hipMemcpyAsync(ctr, h->d_counter, sizeof ctr, hipMemcpyDeviceToHost, h->cur));
        HIPCHK(h, hipStreamSynchronize(h->cur));
        if (int rc = clear_own_sticky(h, ctr[2], BK_STICKY_GUARD)) return rc;  // reported here
        if (ctr[1]) return set_err(h, BK_EOVERFLOW, "bk_rollout: iteration guard tripped%s", "");
    }
    return BK_OK;
}

int bk_rollout(bk_handle h, const bk_state* roots, int32_t n_roots, const int32_t* root_index, int32_t n_playouts,
               const bk_rollout_cfg* cfg, const uint32_t* compat_seeds, bk_result* out, int mem) {
    if (!out) return set_err(h, BK_EINVAL, "bk_rollout: out is NULL%s", "");
    if (cfg && cfg->semantics == BK_SEM_ADVANCE) return set_err(h, BK_EINVAL, "bk_rollout: use bk_advance%s", "");
    return launch_playouts(h, roots, n_roots, root_index, n_playouts, cfg, compat_seeds, out, nullptr, mem);
}

int bk_advance(bk_handle h, const bk_state* roots, int32_t n_roots, const int32_t* root_index, int32_t n_playouts,
               const bk_rollout_cfg* cfg, const uint32_t* compat_seeds, bk_state* out_states, int mem) {
    if (!out_states || !cfg || cfg->semantics != BK_SEM_ADVANCE)
        return set_err(h, BK_EINVAL, "bk_advance: needs out_states and BK_SEM_ADVANCE%s", "");
    return launch_playouts(h, roots, n_roots, root_index, n_playouts, cfg, compat_seeds, nullptr, out_states, mem);
}

int bk_mt_cursor_init(uint32_t seed, uint32_t* out4) {
    if (!out4) return BK_EINVAL;
    uint32_t x = seed, b = 0;
    for (uint32_t j = 1; j <= 397; ++j) {
        x = 1812433253u * (x ^ (x >> 30)) + j;
        if (j == 1) b = x;
    }
    out4[0] = 0; out4[1] = seed; out4[2] = b; out4[3] = x;
    return BK_OK;
}

int bk_arena_advance(bk_handle h, bk_state* states, bk_fset* sets, int32_t n, const bk_rollout_cfg* cfg,
                     const uint8_t* seat_masks, uint32_t* rng_state, bk_result* out, int mem) {
    if (!h || !states || !sets || !cfg || !seat_masks || !rng_state || !out || n < 0)
        return set_err(h, BK_EINVAL, "bk_arena_advance: invalid arguments%s", "");
    if (cfg->semantics != BK_SEM_ARENA || cfg->order != BK_ORDER_FRONTIER || cfg->rng != BK_RNG_NUMPY_MT ||
        cfg->seats_share_stream)
        return set_err(h, BK_EINVAL, "bk_arena_advance: needs ARENA, FRONTIER order, NUMPY_MT per-seat streams%s", "");
    if (mem == BK_MEM_DEVICE && ((uintptr_t)rng_state & 15))
        return set_err(h, BK_EINVAL, "bk_arena_advance: rng_state must be 16-byte aligned%s", "");
    if (n == 0) return BK_OK;
    return launch_playouts(h, states, n, nullptr, n, cfg, nullptr, out, states, mem, sets, sets, seat_masks,
                           rng_state);
}

int bk_arena_step(bk_handle h, bk_state* states, bk_fset* sets, int32_t n, const bk_rollout_cfg* cfg,
                  const uint8_t* seat_masks, const uint8_t* quick_masks, const int32_t* forced, uint32_t* rng_state,
                  bk_result* out, bk_stop_info* stop_out, int mem) {
    if (!h || !states || !sets || !cfg || !seat_masks || !rng_state || !out || n < 0)
        return set_err(h, BK_EINVAL, "bk_arena_step: invalid arguments%s", "");
    if (cfg->semantics != BK_SEM_ARENA || cfg->order != BK_ORDER_FRONTIER || cfg->rng != BK_RNG_NUMPY_MT ||
        cfg->seats_share_stream)
        return set_err(h, BK_EINVAL, "bk_arena_step: needs ARENA, FRONTIER order, NUMPY_MT per-seat streams%s", "");
    if (quick_masks && !stop_out)
        return set_err(h, BK_EINVAL, "bk_arena_step: quick_masks goes with stop_out%s", "");
    if (mem == BK_MEM_DEVICE && ((uintptr_t)rng_state & 15))
        return set_err(h, BK_EINVAL, "bk_arena_step: rng_state must be 16-byte aligned%s", "");
    if (mem == BK_MEM_HOST && forced)
        for (int32_t i = 0; i < n; ++i)
            if (forced[i] < BK_FORCE_SKIP || (forced[i] >= 0 && !(forced[i] & BK_FORCE_INDEX) && forced[i] >= BK_NUM_ORIENTS * 400))
                return set_err(h, BK_EINVAL, "bk_arena_step: forced move out of range%s", "");
    if (n == 0) return BK_OK;
    return launch_playouts(h, states, n, nullptr, n, cfg, nullptr, out, states, mem, sets, sets, seat_masks,
                           rng_state, quick_masks, forced, stop_out);
}

int bk_rollout_frontier(bk_handle h, const bk_state* roots, const bk_fset* root_sets, int32_t n_roots,
                        const int32_t* root_index, int32_t n_playouts, const bk_rollout_cfg* cfg,
                        const uint32_t* compat_seeds, bk_result* out, bk_state* out_states, bk_fset* out_sets,
                        int mem) {
    if (!cfg || cfg->order != BK_ORDER_FRONTIER || !root_sets)
        return set_err(h, BK_EINVAL, "bk_rollout_frontier: needs BK_ORDER_FRONTIER and root_sets%s", "");
    if ((cfg->semantics == BK_SEM_ADVANCE && !out_states) || (cfg->semantics == BK_SEM_ROLLOUT && out_states))
        return set_err(h, BK_EINVAL, "bk_rollout_frontier: out_states goes with BK_SEM_ADVANCE / BK_SEM_ARENA%s", "");
    if (cfg->semantics != BK_SEM_ADVANCE && !out)
        return set_err(h, BK_EINVAL, "bk_rollout_frontier: out is NULL%s", "");
    return launch_playouts(h, roots, n_roots, root_index, n_playouts, cfg, compat_seeds, out, out_states, mem,
                           root_sets, out_sets);
}

// ---- host-side frontier tables (no GPU) ---------------------------------------------
static const int32_t kCornerCell[4] = {0, 19, 399, 380};  // engine/board.py:57-61

int bk_fset_init(bk_fset* s) {
    if (!s) return BK_EINVAL;
    memset(s, 0, sizeof *s);
    for (int p = 0; p < 4; ++p) {
        FsetRef t = fs_ref(s, p, kCellHashHost);
        fs_clear(t);
        int16_t tmp[BK_FSET_SLOTS];
        fs_add(t, tmp, (int16_t)kCornerCell[p]);  // init_frontier_for_player :385-405
    }
    return BK_OK;
}

int bk_fset_place(bk_fset* s, const bk_state* after, int32_t player, const int32_t* cells, int32_t n) {
    if (!s || !after || player < 0 || player > 3 || !cells || n < 0 || n > 5) return BK_EINVAL;
    for (int i = 0; i < n; ++i)
        if (cells[i] < 0 || cells[i] >= BK_CELLS) return BK_EINVAL;
    auto bit = [&](int q, int r, int c) {
        const int b = r * 20 + c;
        return ((after->planes[q][b >> 6] >> (b & 63)) & 1ull) != 0ull;
    };
    int16_t tmp[BK_FSET_SLOTS];
    const bool ok = fs_place(fs_ref(s, player, kCellHashHost), tmp, cells, n,
                             [&](int r, int c) { return bit(0, r, c) || bit(1, r, c) || bit(2, r, c) || bit(3, r, c); },
                             [&](int r, int c) { return bit(player, r, c); });
    return ok ? BK_OK : BK_EOVERFLOW;
}

int bk_fset_copy(bk_fset* dst, const bk_fset* src) {
    if (!dst || !src) return BK_EINVAL;
    if (dst == src) return BK_OK;
    for (int p = 0; p < 4; ++p) {
        if (src->mask[p] + 1u > BK_FSET_SLOTS) return BK_EINVAL;
        if (!fs_copy(fs_ref(dst, p, kCellHashHost), src->key[p], src->mask[p], src->fill[p], src->used[p]))
            return BK_EINVAL;
    }
    return BK_OK;
}

int bk_debug_fset_op(bk_fset* s, int32_t player, int32_t key, int32_t add) {
    if (!s || player < 0 || player > 3 || key < 0 || key >= BK_CELLS || s->mask[player] + 1u > BK_FSET_SLOTS)
        return BK_EINVAL;
    int16_t tmp[BK_FSET_SLOTS];
    // add bit 1: the staged kernels' resize (fs_resize_lds, tables of <= 128 slots) with a
    // 32-key scratch, k_mcts_pair's (k_rollout_fr's holds 16: lds_tmp callers).  A resize of
    // up to 32 active keys then goes through fs_resize_lds (fs_resize_any's choice), and the
    // call returns 1 so the test can count that the path really ran.
    FsetRef t = fs_ref(s, player, kCellHashHost), lt{};
    if (add & 2) {
        t.cap = 128;
        lt.key = tmp;
        lt.cap = 32;
    }
    // fs_op_h, spelled out: the op, then the resize it asked for (fs_resize_any's choice)
    if (!fs_op_nr(t, (int16_t)key, (add & 1) != 0, kCellHashHost[key])) return BK_OK;
    const bool lds_path = lt.key && *t.used <= lt.cap;
    if (!fs_resize_any(t, tmp, lt)) return BK_EOVERFLOW;
    return lds_path ? 1 : BK_OK;
}

int bk_fset_list(const bk_fset* s, int32_t player, int32_t* out, int32_t cap) {
    if (!s || player < 0 || player > 3 || (cap > 0 && !out) || s->mask[player] + 1u > BK_FSET_SLOTS)
        return BK_EINVAL;
    int n = 0;
    for (int i = 0; i <= s->mask[player]; ++i)
        if (s->key[player][i] >= 0) {
            if (n < cap) out[n] = s->key[player][i];
            ++n;
        }
    return n;
}

// Rows [N] of the pow corrections: v in [1, N] where libm pow(x, 0.5) != sqrt(x),
// x = (2.0 * log_table[N]) / v.  false: pow and sqrt more than one ulp apart.
static bool pow_fix_row(const double* log_table, int32_t N, double (*powp)(double, double), std::vector<int32_t>& out) {
    const double L2 = 2.0 * log_table[N];
    for (int32_t v = 1; v <= N; ++v) {
        const double x = L2 / (double)v;
        const double q = sqrt(x);
        if (!(q > 0.0)) continue;
        // sqrt is correctly rounded: |sqrt_exact - q| = d ulp with d <= 0.5.  glibc's pow is
        // within 0.54 ulp of exact (the bound stated in its e_pow.c), so it can return the
        // other neighbour only when d >= 0.46; pow is called for d >= 0.45 alone (~10 %).
        // d from the residual q*q - x, q*q exact by Dekker's product (no fma needed).
        const double c = 134217729.0 * q, qh = c - (c - q), ql = q - qh;
        const double pq = q * q;
        const double err = ((qh * qh - pq) + 2.0 * qh * ql) + ql * ql;
        const double r = (pq - x) + err;  // pq - x is exact (Sterbenz)
        uint64_t b;
        memcpy(&b, &q, sizeof b);
        b &= 0x7FF0000000000000ull;
        double ulp;
        memcpy(&ulp, &b, sizeof ulp);
        ulp *= 2.220446049250313e-16;  // 2^-52: one ulp of q (q normal)
        if (fabs(r) < 0.90 * q * ulp) continue;  // d = |r| / (2 q ulp) < 0.45
        const double p = powp(x, 0.5);
        if (p == q) continue;
        if (p != nextafter(q, INFINITY) && p != nextafter(q, -INFINITY)) return false;
        out.push_back((v << 1) | (p > q ? 1 : 0));
    }
    return true;
}

int bk_pow_half_fix(const double* log_table, int32_t log_len, int32_t* offsets, int32_t* entries, int32_t cap,
                    int32_t* n_entries) {
    if (!log_table || log_len < 1 || !offsets || cap < 0 || (cap > 0 && !entries) || !n_entries) return BK_EINVAL;
    // through a volatile pointer: the call must reach libm's pow (what CPython's float
    // ** calls), never a compiler rewrite of pow(x, 0.5) into sqrt(x)
    double (*volatile powp)(double, double) = pow;
    double (*const pw)(double, double) = powp;
    std::vector<std::vector<int32_t>> rows((size_t)log_len);
    unsigned nt = std::thread::hardware_concurrency();
    cpu_set_t aff;  // the CPUs this process may run on (a bench rank's share of the host)
    if (sched_getaffinity(0, sizeof aff, &aff) == 0 && CPU_COUNT(&aff) > 0) nt = (unsigned)CPU_COUNT(&aff);
    nt = nt < 1 ? 1 : nt > 16 ? 16 : nt;  // the GPU box's CPU share is 16
    if ((int64_t)log_len * log_len < 4000000) nt = 1;
    std::vector<char> ok(nt, 1);
    auto work = [&](unsigned t) {  // rows interleaved: row N costs N
        for (int32_t N = (int32_t)t; N < log_len; N += (int32_t)nt)
            if (!pow_fix_row(log_table, N, pw, rows[(size_t)N])) ok[t] = 0;
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (char o : ok)
        if (!o) return BK_EINVAL;
    int32_t k = 0;
    for (int32_t N = 0; N < log_len; ++N) {
        offsets[N] = k;
        for (int32_t w : rows[(size_t)N]) {
            if (k < cap) entries[k] = w;
            ++k;
        }
    }
    offsets[log_len] = k;
    *n_entries = k;
    return k > cap ? BK_EOVERFLOW : BK_OK;
}

int bk_debug_fastmcts_select(bk_handle h, int32_t n, const uint32_t* visits, const double* totals,
                             uint32_t root_visits, const double* log_table, int32_t log_len,
                             const int32_t* pow_fix_offsets, const int32_t* pow_fix_entries, int32_t pow_fix_rows,
                             double exploration, int32_t* out_best) {
    if (!h || n < 1 || !visits || !totals || !log_table || (int64_t)root_visits >= log_len || !pow_fix_offsets ||
        pow_fix_rows < 0 || pow_fix_rows > log_len || !out_best ||
        (pow_fix_offsets[pow_fix_rows] > 0 && !pow_fix_entries))
        return set_err(h, BK_EINVAL, "bk_debug_fastmcts_select: invalid arguments%s", "");
    const int32_t pow_fix_len = pow_fix_offsets[pow_fix_rows];
    for (int32_t j = 0; j < n; ++j)
        if (visits[j] == 0) return set_err(h, BK_EINVAL, "bk_debug_fastmcts_select: visits must be > 0%s", "");
    HIPCHK(h, hipSetDevice(h->device));
    BK_IDLE(h, "bk_debug_fastmcts_select");
    const size_t bv = sizeof(uint32_t) * n, bt = sizeof(double) * n, bo = sizeof(int32_t) * (size_t)(pow_fix_rows + 1),
                 be = sizeof(int32_t) * (size_t)(pow_fix_len + 1);
    int rc = grow(h, &h->d_aux, &h->d_aux_cap, bt + bv + bo + be + 64);
    if (rc) return rc;
    char* p = (char*)h->d_aux;
    double* d_t = (double*)p; p += bt;
    uint32_t* d_v = (uint32_t*)p; p += bv;
    int32_t* d_o = (int32_t*)p; p += bo;
    int32_t* d_e = (int32_t*)p; p += be;
    int32_t* d_out = (int32_t*)(((uintptr_t)p + 15) & ~(uintptr_t)15);
    HIPCHK(h, hipMemcpyAsync(d_t, totals, bt, hipMemcpyHostToDevice, h->cur));
    HIPCHK(h, hipMemcpyAsync(d_v, visits, bv, hipMemcpyHostToDevice, h->cur));
    HIPCHK(h, hipMemcpyAsync(d_o, pow_fix_offsets, bo, hipMemcpyHostToDevice, h->cur));
    if (pow_fix_len) HIPCHK(h, hipMemcpyAsync(d_e, pow_fix_entries, be - sizeof(int32_t), hipMemcpyHostToDevice, h->cur));
    hipLaunchKernelGGL(k_fastmcts_select, dim3(1), dim3(WAVE), 0, h->cur, d_v, d_t, n, root_visits,
                       2.0 * log_table[root_visits], exploration, PowFix{d_o, d_e, pow_fix_rows}, d_out);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemcpyAsync(out_best, d_out, sizeof(int32_t), hipMemcpyDeviceToHost, h->cur));
    HIPCHK(h, hipStreamSynchronize(h->cur));
    return BK_OK;
}

int bk_fastmcts(bk_handle h, int32_t n_games, const int32_t* legal_offset, const int32_t* iterations,
                const double* base, uint32_t* mt_state, const double* log_table, int32_t log_len,
                const int32_t* pow_fix_offsets, const int32_t* pow_fix_entries, int32_t pow_fix_rows,
                double exploration, bk_fastmcts_out* out, int32_t* visits_out, int mem) {
    if (!h || n_games < 0 || !legal_offset || !iterations || !base || !mt_state || !log_table || log_len <= 0 ||
        !pow_fix_offsets || pow_fix_rows < 0 || pow_fix_rows > log_len ||
        !out || (mem != BK_MEM_HOST && mem != BK_MEM_DEVICE))
        return set_err(h, BK_EINVAL, "bk_fastmcts: invalid arguments%s", "");
    const int32_t pow_fix_len = mem == BK_MEM_HOST ? pow_fix_offsets[pow_fix_rows] : 0;
    if (pow_fix_len > 0 && !pow_fix_entries)
        return set_err(h, BK_EINVAL, "bk_fastmcts: pow_fix_entries missing%s", "");
    if (n_games == 0) return BK_OK;
    HIPCHK(h, hipSetDevice(h->device));
    BK_IDLE(h, "bk_fastmcts");
    const size_t b_off = sizeof(int32_t) * (size_t)(n_games + 1), b_it = sizeof(int32_t) * (size_t)n_games,
                 b_base = sizeof(double) * (size_t)n_games, b_mt = sizeof(uint32_t) * 625 * (size_t)n_games,
                 b_log = sizeof(double) * (size_t)log_len, b_out = sizeof(bk_fastmcts_out) * (size_t)n_games,
                 b_fo = sizeof(int32_t) * (size_t)(pow_fix_rows + 1), b_fe = sizeof(int32_t) * (size_t)(pow_fix_len + 1);
    const int32_t* d_off = legal_offset;
    const int32_t* d_it = iterations;
    const double* d_base = base;
    uint32_t* d_mt = mt_state;
    const double* d_log = log_table;
    const int32_t* d_fo = pow_fix_offsets;
    const int32_t* d_fe = pow_fix_entries;
    bk_fastmcts_out* d_out = out;
    int32_t* d_vis = visits_out;
    int32_t n_legal_total = 0;
    if (mem == BK_MEM_HOST) {
        if (legal_offset[0] != 0) return set_err(h, BK_EINVAL, "bk_fastmcts: legal_offset[0] must be 0%s", "");
        for (int32_t i = 0; i < n_games; ++i)
            if (legal_offset[i + 1] < legal_offset[i] || iterations[i] < 0 || iterations[i] >= log_len)
                return set_err(h, BK_EINVAL, "bk_fastmcts: bad legal_offset/iterations%s", "");
        n_legal_total = legal_offset[n_games];
    }
    if (mem == BK_MEM_HOST) {
        // one staging buffer, 16-byte aligned sections
        auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
        const size_t tot = al(b_off) + al(b_it) + al(b_base) + al(b_mt) + al(b_log) + al(b_fo) + al(b_fe);
        int rc = grow(h, &h->d_in, &h->d_in_cap, tot);
        if (rc) return rc;
        rc = grow(h, &h->d_out, &h->d_out_cap, b_out);
        if (rc) return rc;
        char* p = (char*)h->d_in;
        HIPCHK(h, hipMemcpyAsync(p, legal_offset, b_off, hipMemcpyHostToDevice, h->cur)); d_off = (const int32_t*)p; p += al(b_off);
        HIPCHK(h, hipMemcpyAsync(p, iterations, b_it, hipMemcpyHostToDevice, h->cur)); d_it = (const int32_t*)p; p += al(b_it);
        HIPCHK(h, hipMemcpyAsync(p, base, b_base, hipMemcpyHostToDevice, h->cur)); d_base = (const double*)p; p += al(b_base);
        HIPCHK(h, hipMemcpyAsync(p, mt_state, b_mt, hipMemcpyHostToDevice, h->cur)); d_mt = (uint32_t*)p; p += al(b_mt);
        HIPCHK(h, hipMemcpyAsync(p, log_table, b_log, hipMemcpyHostToDevice, h->cur)); d_log = (const double*)p; p += al(b_log);
        HIPCHK(h, hipMemcpyAsync(p, pow_fix_offsets, b_fo, hipMemcpyHostToDevice, h->cur)); d_fo = (const int32_t*)p; p += al(b_fo);
        if (pow_fix_len)
            HIPCHK(h, hipMemcpyAsync(p, pow_fix_entries, b_fe - sizeof(int32_t), hipMemcpyHostToDevice, h->cur));
        d_fe = (const int32_t*)p;
        d_out = (bk_fastmcts_out*)h->d_out;
        if (visits_out) {
            rc = grow(h, &h->d_aux, &h->d_aux_cap, sizeof(int32_t) * (size_t)n_legal_total + 4);
            if (rc) return rc;
            d_vis = (int32_t*)h->d_aux;
        }
    }
    HIPCHK(h, hipMemsetAsync(h->d_counter, 0, 2 * sizeof(uint32_t), h->cur));  // [2] is sticky
    FastMctsArgs a{n_games, d_off, d_it, d_base, d_mt, d_log, log_len, PowFix{d_fo, d_fe, pow_fix_rows}, exploration,
                   d_out, d_vis,
                   h->d_counter + 1};
    HIPCHK(h, mark_start(h));
    h->last_kernel = "k_fastmcts";
    hipLaunchKernelGGL(k_fastmcts, dim3(n_games), dim3(WAVE), 0, h->cur, a);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, mark_end(h));
    if (mem == BK_MEM_HOST) {
        uint32_t ctr[4];
        HIPCHK(h, hipMemcpyAsync(out, d_out, b_out, hipMemcpyDeviceToHost, h->cur));
        HIPCHK(h, hipMemcpyAsync(mt_state, d_mt, b_mt, hipMemcpyDeviceToHost, h->cur));
        if (visits_out && n_legal_total > 0)
            HIPCHK(h, hipMemcpyAsync(visits_out, d_vis, sizeof(int32_t) * (size_t)n_legal_total,
                                     hipMemcpyDeviceToHost, h->cur));
        HIPCHK(h, hipMemcpyAsync(ctr, h->d_counter, sizeof ctr, hipMemcpyDeviceToHost, h->cur));
        HIPCHK(h, hipStreamSynchronize(h->cur));
        if (int rc = clear_own_sticky(h, ctr[2], BK_STICKY_FASTMCTS)) return rc;  // reported here
        if (ctr[1]) return set_err(h, BK_EINVAL, "bk_fastmcts: too many children or log table too short%s", "");
    }
    return BK_OK;
}

int bk_mcts(bk_handle h, const bk_state* roots, const bk_fset* root_sets, const uint8_t* players,
            const uint64_t* root_hash, int32_t n_games, const bk_mcts_cfg* cfg, const uint64_t* zobrist,
            int32_t n_zobrist, const int32_t* zobrist_index, uint32_t* mt_state, uint64_t* tt_keys,
            double* tt_vals, int32_t* tt_count, const double* log_table, int32_t log_len,
            bk_mcts_node* nodes, double* rewards, uint8_t* hit_flags, bk_mcts_out* out, int mem) {
    if (!h || !cfg || n_games < 0 || (mem != BK_MEM_HOST && mem != BK_MEM_DEVICE))
        return set_err(h, BK_EINVAL, "bk_mcts: invalid arguments%s", "");
    if (n_games == 0) return BK_OK;
    if (!roots || !root_sets || !players || !zobrist || n_zobrist < 1 || !zobrist_index ||
        !mt_state || !log_table || log_len < 1 || !out || (rewards == nullptr) != (hit_flags == nullptr))
        return set_err(h, BK_EINVAL, "bk_mcts: missing buffer%s", "");
    if (cfg->iterations < 0 || cfg->max_rollout_moves <= 0 || cfg->node_cap < 1 || cfg->time_limit_us < 0 ||
        cfg->iter_stop < 0 || (cfg->resume != 0 && cfg->resume != 1) ||
        (cfg->rollout_policy != BK_MCTS_ROLLOUT_RANDOM && cfg->rollout_policy != BK_MCTS_ROLLOUT_HEURISTIC))
        return set_err(h, BK_EINVAL, "bk_mcts: bad cfg (iterations/max_rollout_moves/node_cap/iter_stop/resume)%s", "");
    if (cfg->resume && !nodes)
        return set_err(h, BK_EINVAL, "bk_mcts: resume needs the caller's nodes buffer%s", "");
    if ((cfg->flags & BK_MCTS_STATE_ROWS) && mem != BK_MEM_DEVICE)
        return set_err(h, BK_EINVAL, "bk_mcts: BK_MCTS_STATE_ROWS needs BK_MEM_DEVICE buffers%s", "");
    if (cfg->use_tt && (!tt_keys || !tt_vals || !tt_count || cfg->tt_cap < 2 || (cfg->tt_cap & (cfg->tt_cap - 1))))
        return set_err(h, BK_EINVAL, "bk_mcts: use_tt needs tt buffers and a power-of-two tt_cap%s", "");
    if (mem == BK_MEM_HOST) {
        for (int32_t g = 0; g < n_games; ++g) {
            if (players[g] > 3 || zobrist_index[g] < 0 || zobrist_index[g] >= n_zobrist || mt_state[(size_t)g * 625 + 624] > 624)
                return set_err(h, BK_EINVAL, "bk_mcts: bad player / zobrist_index / mt pos%s", "");
            for (int q = 0; q < 4; ++q)
                if (root_sets[g].mask[q] + 1u > BK_FSET_SLOTS)
                    return set_err(h, BK_EINVAL, "bk_mcts: root frontier table too large%s", "");
            if (cfg->use_tt && (tt_count[g] < 0 || tt_count[g] >= cfg->tt_cap))
                return set_err(h, BK_EINVAL, "bk_mcts: bad tt_count%s", "");
        }
    }
    HIPCHK(h, hipSetDevice(h->device));
    BK_IDLE(h, "bk_mcts");
    const size_t n = (size_t)n_games, ttc = cfg->use_tt ? (size_t)cfg->tt_cap : 0;
    const size_t it = (size_t)cfg->iterations;
    struct Sec { const void* host; size_t bytes; int dir; void* dev; };  // dir: 1 in, 2 out, 3 in+out
    Sec sec[] = {
        {roots, sizeof(bk_state) * n, 1, nullptr},
        {root_sets, sizeof(bk_fset) * n, 1, nullptr},
        {players, n, 1, nullptr},
        {root_hash, sizeof(uint64_t) * n, 1, nullptr},
        {zobrist, sizeof(uint64_t) * MC_ZOB * (size_t)n_zobrist, 1, nullptr},
        {zobrist_index, sizeof(int32_t) * n, 1, nullptr},
        {mt_state, sizeof(uint32_t) * 625 * n, 3, nullptr},
        {tt_keys, sizeof(uint64_t) * ttc * n, 3, nullptr},
        {tt_vals, sizeof(double) * ttc * n, 3, nullptr},
        {tt_count, cfg->use_tt ? sizeof(int32_t) * n : 0, 3, nullptr},
        {log_table, sizeof(double) * (size_t)log_len, 1, nullptr},
        {nodes, sizeof(bk_mcts_node) * (size_t)cfg->node_cap * n, cfg->resume ? 3 : 2, nullptr},
        {rewards, sizeof(double) * it * n, cfg->resume ? 3 : 2, nullptr},
        {hit_flags, it * n, cfg->resume ? 3 : 2, nullptr},
        {out, sizeof(bk_mcts_out) * n, cfg->resume ? 3 : 2, nullptr},
    };
    const int NSEC = (int)(sizeof sec / sizeof sec[0]);
    const int NODES = 11;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t tot = 0;
    for (int i = 0; i < NSEC; ++i) {
        const bool staged = mem == BK_MEM_HOST || (i == NODES && nodes == nullptr);
        if (staged && sec[i].bytes && (sec[i].host || i == NODES)) tot += al(sec[i].bytes);
    }
    int rc = grow(h, &h->d_mc, &h->d_mc_cap, tot + 256);
    if (rc) return rc;
    char* p = (char*)h->d_mc;
    for (int i = 0; i < NSEC; ++i) {
        const bool staged = mem == BK_MEM_HOST || (i == NODES && nodes == nullptr);
        if (!staged) { sec[i].dev = const_cast<void*>(sec[i].host); continue; }
        if (!sec[i].bytes || (!sec[i].host && i != NODES)) { sec[i].dev = nullptr; continue; }
        sec[i].dev = p;
        if ((sec[i].dir & 1) && sec[i].host)
            HIPCHK(h, hipMemcpyAsync(p, sec[i].host, sec[i].bytes, hipMemcpyHostToDevice, h->cur));
        p += al(sec[i].bytes);
    }
    if (!root_hash) {  // ZobristHash.hash_board of every root, on the device
        rc = grow(h, &h->d_rh, &h->d_rh_cap, sizeof(uint64_t) * n);
        if (rc) return rc;
        hipLaunchKernelGGL(k_root_hash, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, h->cur,
                           (const bk_state*)sec[0].dev, (const uint64_t*)sec[4].dev, (const int32_t*)sec[5].dev,
                           (uint64_t*)h->d_rh, n_games);
        HIPCHK(h, hipGetLastError());
        sec[3].dev = h->d_rh;
    }
    // persistent grid: every resident slot pulls whole searches from the counter
    const bool heur = cfg->rollout_policy == BK_MCTS_ROLLOUT_HEURISTIC;
    // one wave per search (k_mcts_coop) when the batch cannot fill the chip with one
    // search per lane.  Measured crossovers (64 iterations, profiles/r03/coopsweep,
    // coopblocks): random rollouts ~44 searches per CU (k_mcts_pair 229 ms flat vs
    // k_mcts_coop 162 ms at 32 per CU with 4 blocks per CU); heuristic rollouts ~90 per CU
    // (k_mcts_h 1.88 s flat vs k_mcts_coop_h 1.33 s at 64 per CU, 2.61 s at 128) --
    // config 4 with 8,192 games on one GPU searches 8,192 at once: 164 -> 242 games/s
    bool coop = (int64_t)n_games <= (heur ? 80 : 40) * (int64_t)h->num_cu;
    coop = tune_or(h, BK_TUNE_MCTS_COOP, coop ? 1 : 0) != 0;
    const int blk = coop ? COOP_WAVES * WAVE : heur ? HBLOCK : BLOCK;
    // k_mcts_coop(_h) blocks (of COOP_WAVES searches) per CU: all the waves the registers
    // allow (k_mcts_coop 225 VGPRs: 2 per SIMD, twice the throughput of 1 --
    // profiles/r03/coopblocks; k_mcts_coop_h 404: 1)
    int coop_bpc = heur ? 2 : 4;
    if (tune_or(h, BK_TUNE_COOP_BLOCKS_PER_CU, 0) > 0) coop_bpc = (int)h->tune[BK_TUNE_COOP_BLOCKS_PER_CU];
    int blocks = h->num_cu * (coop ? coop_bpc : heur ? 3 : h->mcts_blocks_per_cu);
    // k_mcts is latency-bound at one wave per SIMD (config 5: 65,536 searches fill one
    // 256-lane block per CU): when the resident slots allow, every other lane takes a
    // search, so twice the waves hide each other's latency (11.14 vs 10.84 M sims/s,
    // profiles/r03/sweeps/mcts_spread.jsonl; 4 measured slower)
    int spread = (!heur && !coop && (int64_t)n_games * 2 <= (int64_t)blocks * blk) ? 2 : 1;
    spread = (int)tune_or(h, BK_TUNE_MCTS_SPREAD, spread);
    if (spread < 1 || spread > WAVE || (spread & (spread - 1)) || coop) spread = 1;
    const int per_block = coop ? COOP_WAVES : blk;  // searches a block holds at once
    const int need = (int)(((int64_t)n_games * spread + per_block - 1) / per_block);
    if (blocks > need) blocks = need;
    if (blocks < 1) blocks = 1;
    const uint32_t nslots = (uint32_t)blocks * per_block;
    rc = grow(h, &h->d_slab, &h->d_slab_cap, sizeof(uint32_t) * SLAB_WORDS * (size_t)nslots);
    if (rc) return rc;
    rc = grow(h, &h->d_mclane, &h->d_mclane_cap, sizeof(McLane) * (size_t)nslots);
    if (rc) return rc;
    int khz = 0;
    HIPCHK(h, hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device));
    if (khz <= 0) khz = 100000;
    HIPCHK(h, hipMemsetAsync(h->d_counter, 0, 2 * sizeof(uint32_t), h->cur));  // [2] is sticky
    const uint64_t per_lane = ((uint64_t)n_games * spread + nslots - 1) / nslots + 1;
    // a waiting lane waits at most one simulation of the others (2x)
    const uint64_t steps = 2 * per_lane * ((uint64_t)cfg->iterations + 1) * ((uint64_t)cfg->max_rollout_moves + 2) + 64;
    int32_t tree_batch = MC_TREE_BATCH;
    tree_batch = (int32_t)tune_or(h, BK_TUNE_TREE_BATCH, tree_batch);
    if (tree_batch < 1) tree_batch = 1;
    MctsArgs a{(const bk_state*)sec[0].dev, (const bk_fset*)sec[1].dev, (const uint8_t*)sec[2].dev,
               (const uint64_t*)sec[3].dev, n_games, *cfg, (const uint64_t*)sec[4].dev,
               (const int32_t*)sec[5].dev, (uint32_t*)sec[6].dev, (uint64_t*)sec[7].dev, (double*)sec[8].dev,
               (int32_t*)sec[9].dev, (const double*)sec[10].dev, log_len, (bk_mcts_node*)sec[11].dev,
               (double*)sec[12].dev, (uint8_t*)sec[13].dev, (bk_mcts_out*)sec[14].dev,
               (uint32_t*)h->d_slab, (McLane*)h->d_mclane, h->d_counter, steps,
               (uint64_t)cfg->time_limit_us * (uint64_t)khz / 1000u, tree_batch, spread, 1, 1};
    a.diag = h->d_diag;
    a.launch_seq = ++h->mcts_launches;
    a.state_rows = (cfg->flags & BK_MCTS_STATE_ROWS) ? 1 : 0;
    a.done = h->mcts_done;
    if (a.state_rows) {  // the searches work on copies of their agents' MT rows
        rc = grow(h, &h->d_mtwork, &h->d_mtwork_cap, sizeof(uint32_t) * (FM_N + 1) * n);
        if (rc) return rc;
        a.mt_rows = a.mt;
        a.mt = (uint32_t*)h->d_mtwork;
    }
    {
        const size_t sb = sizeof(uint32_t) * (((size_t)n_games + 31) / 32 + 1);
        rc = grow(h, &h->d_started, &h->d_started_cap, sb);
        if (rc) return rc;
        HIPCHK(h, hipMemsetAsync(h->d_started, 0, sb, h->cur));
        a.started = (uint32_t*)h->d_started;
    }
    a.coop_walk = (int)tune_or(h, BK_TUNE_COOP_WALK, a.coop_walk);
    a.coop_balanced = (int)tune_or(h, BK_TUNE_COOP_BAL, a.coop_balanced);
    // spread 2: the idle odd lane of each pair splits the even lane's stencil (k_mcts_pair)
    const bool pair = tune_or(h, BK_TUNE_MCTS_PAIR, 1) != 0;
    HIPCHK(h, mark_start(h));
    if (coop && heur) {
        h->last_kernel = "k_mcts_coop_h";
        a.kernel_id = BK_DIAG_K_COOP_H;
        hipLaunchKernelGGL(k_mcts_coop_h, dim3(blocks), dim3(blk), 0, h->cur, a);
    } else if (coop) {
        h->last_kernel = "k_mcts_coop";
        a.kernel_id = BK_DIAG_K_COOP;
        hipLaunchKernelGGL(k_mcts_coop, dim3(blocks), dim3(blk), 0, h->cur, a);
    } else if (heur) {
        h->last_kernel = "k_mcts_h";
        a.kernel_id = BK_DIAG_K_H;
        hipLaunchKernelGGL(k_mcts_h, dim3(blocks), dim3(HBLOCK), 0, h->cur, a);
    } else if (spread == 2 && pair) {
        h->last_kernel = "k_mcts_pair";
        a.kernel_id = BK_DIAG_K_PAIR;
        hipLaunchKernelGGL(k_mcts_pair, dim3(blocks), dim3(BLOCK), 0, h->cur, a);
    } else {
        h->last_kernel = "k_mcts";
        hipLaunchKernelGGL(k_mcts, dim3(blocks), dim3(BLOCK), 0, h->cur, a);
    }
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, mark_end(h));
    if (mem == BK_MEM_DEVICE && (cfg->flags & BK_MCTS_ASYNC)) {  // errors: bk_synchronize
        h->busy = true;  // the running search owns the scratch until then
        h->busy_stream = h->cur;
        return BK_OK;
    }
    uint32_t ctr[4];
    if (mem == BK_MEM_HOST) {
        for (int i = 0; i < NSEC; ++i)
            if ((sec[i].dir & 2) && sec[i].host && sec[i].bytes)
                HIPCHK(h, hipMemcpyAsync(const_cast<void*>(sec[i].host), sec[i].dev, sec[i].bytes,
                                         hipMemcpyDeviceToHost, h->cur));
    }
    HIPCHK(h, hipMemcpyAsync(ctr, h->d_counter, sizeof ctr, hipMemcpyDeviceToHost, h->cur));
    HIPCHK(h, hipStreamSynchronize(h->cur));
    if (int rc = clear_own_sticky(h, ctr[2], BK_STICKY_GUARD)) return rc;  // reported here
    if (ctr[1]) return set_err(h, BK_EOVERFLOW, "bk_mcts: step guard tripped%s", "");
    if (int rc = take_diag(h)) return rc;  // a search broke a tree invariant (mc_diag)
    return BK_OK;
}

}  // extern "C"
#endif  // BK_DEF(BK_U_HOST)
