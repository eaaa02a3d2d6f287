"""Philox4x32-10 in the oracle (the native BK_RNG_PHILOX stream the timed config-3 path
draws from), checked against the Random123 known-answer vectors.

Random123 (Salmon et al., SC'11) publishes kat_vectors for philox4x32 with 10 rounds;
the three below are its philox4x32_10 lines (counter, key -> output).  The native stream
is word 0 of philox4x32_10({draw counter, playout id, 0x5bd1e995, 0}, {seed lo, hi}).
"""
import numpy as np

from oracle import pyoracle as O

KAT = [  # (ctr[4], key[2], out[4])
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


def test_philox_known_answers():
    for ctr, key, out in KAT:
        assert O.philox4x32_10(ctr, key) == out


def test_native_stream_is_block_word0():
    for seed in (0, 1, 20260301 * 7919 + 1000, 2**64 - 1):
        for pid in (0, 5, 262143):
            for c in (0, 1, 77):
                blk = O.philox4x32_10([c, pid, 0x5BD1E995, 0], [seed & 0xFFFFFFFF, seed >> 32])
                assert O.philox_stream(seed, pid, c) == blk[0]


def _legal_replay(root_board, trace):
    """Replay a playout's moves on a copy of the root: every move must be in the legal
    list of its mover (-1 = pass, only when the mover has no legal move)."""
    b = O.copy_board(root_board)
    for mv in trace:
        p = b.cur
        legal = O.legal_moves(b, p, O.ORDER_NAIVE)
        if mv < 0:
            assert not legal
            b.cur = (b.cur + 1) & 3
        else:
            assert mv in legal
            O.place_move(b, p, mv)
    return b


def test_philox_playouts_legal_and_deterministic():
    """Arena playouts on the Philox stream: each ply a legal move (passes only when
    stuck), the game terminal, the draw count >= the placements, and the batch driver
    (threads, root_index) plays the same games as one call per playout."""
    from tests.helpers import POS, replay, pack_many
    roots = [replay(POS[i]) for i in (4, 9, 17)]
    seed = 20260301 * 7919 + 1000
    ridx = np.array([0, 1, 2, 2, 1, 0], np.int32)
    singles = []
    for pid, ri in enumerate(ridx.tolist()):
        b = O.copy_board(roots[ri])
        res, trace = O.playout_arena_philox(b, seed, pid)
        end = _legal_replay(roots[ri], trace)
        assert all(not O.legal_moves(end, p, O.ORDER_NAIVE) for p in range(4))
        assert res.plies == sum(1 for m in trace if m >= 0) and res.draws >= res.plies
        singles.append(bytes(res))
    st = (O.State * 3).from_buffer_copy(pack_many(roots).tobytes())
    batch = O.batch_playouts(st, len(ridx), seed, rng=O.RNG_PHILOX, root_index=ridx, threads=3,
                             order=O.ORDER_NAIVE)
    assert [bytes(r) for r in batch] == singles
    assert len(set(singles)) > 1


def test_philox_advance_budget():
    """max_plies: bk_advance stops after that many placements (the synthetic roots)."""
    b = O.new_board()
    res, trace = O.playout_arena_philox(b, 20260301, 3, max_plies=20)
    assert res.plies == 20 and len([m for m in trace if m >= 0]) == 20
    assert b.move_count == 20


def test_naive_via_frontier_plays_the_naive_games():
    """OR_ORDER_NAIVE_VIA_FRONTIER (bench.py's naive-order CPU baseline: frontier anchors,
    then a row-major sort) plays exactly the games of the full 400-anchor naive scan."""
    from tests.helpers import POS, replay, pack_many
    roots = [replay(POS[i]) for i in (0, 4, 9, 17, 30)]
    st = (O.State * len(roots)).from_buffer_copy(pack_many(roots).tobytes())
    seed = 20260301 * 7919 + 1007
    ridx = np.arange(40, dtype=np.int32) % len(roots)
    a = O.batch_playouts(st, 40, seed, rng=O.RNG_PHILOX, root_index=ridx, threads=4, order=O.ORDER_NAIVE)
    b = O.batch_playouts(st, 40, seed, rng=O.RNG_PHILOX, root_index=ridx, threads=4,
                         order=O.ORDER_NAIVE_VIA_FRONTIER)
    assert [bytes(r) for r in a] == [bytes(r) for r in b]
