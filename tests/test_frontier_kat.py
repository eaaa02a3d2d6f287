"""Frontier and bitboard known-answer cases on the host Board mirror (CPU only).

Mirrors the GPU-free cases of the reference's tests/test_frontier_basic.py:12-276
(start corners, single and two-cell placements, edge cells, incremental update vs full
recompute, the three frontier invariants) and tests/test_bitboard_basic.py:92-155
(bitboards agree with the grid after placements and after copy).  The frontier is the
reference's incremental set (engine/board.py:247-405), so stale entries may remain for
the player who did not move; the invariants are checked for the mover, as there.
"""
import numpy as np
import pytest

from reinforcementlearning_blokus_amd.engine.board import Board, Player, Position

DIAG = ((-1, -1), (-1, 1), (1, -1), (1, 1))
ORTH = ((-1, 0), (1, 0), (0, -1), (0, 1))


def check_invariants(board, player):
    v, g = player.value, board.grid
    corner = board.player_start_corners[player]
    for r, c in board.get_frontier(player):
        assert g[r, c] == 0, (r, c)
        if board.player_first_move[player] and (r, c) == (corner.row, corner.col):
            continue
        near = [(r + dr, c + dc) for dr, dc in DIAG if 0 <= r + dr < 20 and 0 <= c + dc < 20]
        assert any(g[x, y] == v for x, y in near), (r, c)
        side = [(r + dr, c + dc) for dr, dc in ORTH if 0 <= r + dr < 20 and 0 <= c + dc < 20]
        assert all(g[x, y] != v for x, y in side), (r, c)


def test_initial_frontiers_are_start_corners():
    b = Board()
    for p in Player:
        corner = b.player_start_corners[p]
        assert b.get_frontier(p) == {(corner.row, corner.col)}
        assert b.is_empty(corner)
    assert {(b.player_start_corners[p].row, b.player_start_corners[p].col) for p in Player} == \
        {(0, 0), (0, 19), (19, 19), (19, 0)}


def test_monomino_at_corner():
    b = Board()
    assert b.place_piece([Position(0, 0)], Player.RED, 1)
    f = b.get_frontier(Player.RED)
    assert f == {(1, 1)}
    assert b._verify_frontier_consistency(Player.RED)
    check_invariants(b, Player.RED)


def test_domino_at_corner():
    b = Board()
    assert b.place_piece([Position(0, 0), Position(0, 1)], Player.RED, 2)
    f = b.get_frontier(Player.RED)
    assert (1, 2) in f
    for cell in ((0, 0), (0, 1), (1, 1), (1, 0), (0, 2)):
        assert cell not in f
    assert b._verify_frontier_consistency(Player.RED)
    assert b.debug_rebuild_frontier(Player.RED)


def test_incremental_matches_rebuild_after_two_moves():
    b = Board()
    b.place_piece([Position(0, 0), Position(0, 1)], Player.RED, 2)
    assert b.debug_rebuild_frontier(Player.RED)
    # a legal continuation: (1,2) touches (0,1) corner-to-corner only
    b.current_player = Player.RED
    assert b.place_piece([Position(1, 2), Position(1, 3)], Player.RED, 3)
    assert b.debug_rebuild_frontier(Player.RED)
    assert b._verify_frontier_consistency(Player.RED)
    check_invariants(b, Player.RED)


def test_illegal_placement_rejected_and_board_unchanged():
    b = Board()
    before = b.grid.copy()
    # not covering RED's start corner on its first move
    assert not b.place_piece([Position(5, 5)], Player.RED, 1)
    # overlapping an occupied cell
    assert b.place_piece([Position(0, 0)], Player.RED, 1)
    assert not b.place_piece([Position(0, 0)], Player.BLUE, 1)
    assert np.count_nonzero(b.grid != before) == 1


@pytest.mark.parametrize("player, cell", [(Player.BLUE, (0, 19)), (Player.YELLOW, (19, 19)),
                                          (Player.GREEN, (19, 0))])
def test_frontier_stays_on_board_at_other_corners(player, cell):
    b = Board()
    b.current_player = player
    assert b.place_piece([Position(*cell)], player, 1)
    f = b.get_frontier(player)
    r, c = cell
    assert f == {(r + (1 if r == 0 else -1), c + (1 if c == 0 else -1))}
    assert all(0 <= x < 20 and 0 <= y < 20 for x, y in f)


def test_bitboards_follow_grid_and_copy():
    b = Board()
    b.place_piece([Position(0, 0), Position(1, 0), Position(1, 1)], Player.RED, 4)
    b.place_piece([Position(0, 19), Position(0, 18)], Player.BLUE, 2)
    for p in Player:
        bits = b.player_bits[p]
        cells = {(i // 20, i % 20) for i in range(400) if bits >> i & 1}
        assert cells == {(int(r), int(c)) for r, c in zip(*np.nonzero(b.grid == p.value))}
    assert b.occupied_bits == b.player_bits[Player.RED] | b.player_bits[Player.BLUE]
    b.assert_bitboard_consistent()
    c = b.copy()
    c.place_piece([Position(19, 19)], Player.YELLOW, 1, validate=False)
    assert b.player_bits[Player.YELLOW] == 0 and c.player_bits[Player.YELLOW] == 1 << 399
    assert b.get_frontier(Player.RED) == c.get_frontier(Player.RED)


def test_frontier_ranks_equal_fset_list_order():
    """frontier_ranks (vectorised, from the tables) ranks every player's frontier cells
    exactly as the iteration order fset_list gives (the batched arena's FastMCTS lists)."""
    from reinforcementlearning_blokus_amd import _native as N
    from reinforcementlearning_blokus_amd.engine.move_generator import _BIG, frontier_ranks
    from reinforcementlearning_blokus_amd.engine.pieces import ORIENT_CELLS, ORIENT_LIST
    rng = np.random.RandomState(5)
    boards = []
    for t in range(24):
        b = Board()
        for _ in range(rng.randint(0, 30)):  # unvalidated placements: arbitrary table histories
            g = rng.randint(len(ORIENT_CELLS))
            ar, ac = rng.randint(0, 16), rng.randint(0, 16)
            cells = [Position(ar + dr, ac + dc) for dr, dc in ORIENT_CELLS[g]]
            if all(b.is_empty(p) for p in cells):
                b.place_piece(cells, list(Player)[rng.randint(4)], ORIENT_LIST[g][0], validate=False)
        boards.append(b)
    sets = np.concatenate([b.frontier_tables for b in boards])
    for p in range(4):
        ranks = frontier_ranks(sets, [p] * len(boards))
        for i in range(len(boards)):
            want = np.full(400, _BIG, np.int64)
            for j, cell in enumerate(N.fset_list(sets[i:i + 1], p)):
                want[cell] = j
            assert np.array_equal(ranks[i], want), (i, p)
