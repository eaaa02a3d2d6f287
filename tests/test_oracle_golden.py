"""Pin the CPU oracle (oracle/blokus_oracle.c) against the reference's own outputs.

The golden vectors in tests/golden/ were produced by importing the reference
(tools/gen_fixtures.py).  If these pass, the oracle is a trustworthy checker for
the HIP path at sizes the reference itself cannot reach.
"""
import hashlib
import math

import pytest

from oracle import pyoracle as O
from tests.conftest import load_golden

POS = load_golden("positions.json")


def _sha(ints):
    return hashlib.sha256(",".join(str(i) for i in ints).encode()).hexdigest()


def replay(rec):
    """Rebuild the reference Board by replaying its place_piece log (cell order kept)."""
    b = O.new_board()
    for player_value, piece_id, cells in rec["log"]:
        # generate_random_valid_state places for board.current_player; passes advance it
        while b.cur != player_value - 1:
            b.cur = (b.cur + 1) & 3
        O.place_cells(b, player_value - 1, piece_id, [r * 20 + c for r, c in cells])
    b.cur = rec["state"]["current_player"] - 1
    return b


def test_orientation_table_matches_reference():
    ref = load_golden("pieces.json")
    mine = O.orient_table()
    assert len(mine) == len(ref) == 91
    for (pid, o, offs), r in zip(mine, ref):
        assert pid == r["piece_id"] and o == r["orientation"]
        assert [list(x) for x in offs] == r["offsets"]
    assert sum(len(x[2]) for x in mine) == 410


@pytest.mark.parametrize("idx", range(len(POS)))
def test_state_generator_and_frontier_layout(idx):
    rec = POS[idx]
    b, log = O.gen_state(rec["num_moves"], rec["seed"])
    st = rec["state"]
    assert len(log) == len(rec["log"])
    for p in range(4):
        bits = sum(1 << i for i in range(400) if b.grid[i] == p + 1)
        assert hex(bits) == st["player_bits"][p]
        assert sorted(i + 1 for i in range(21) if b.used[p] >> i & 1) == st["used"][p]
        assert bool(b.first[p]) == st["first"][p]
        # CPython set iteration order reproduced exactly
        assert O.frontier(b, p) == [r * 20 + c for r, c in st["frontier"][p]]
    assert b.cur + 1 == st["current_player"]
    assert b.move_count == st["move_count"]


@pytest.mark.parametrize("idx", range(len(POS)))
def test_legal_moves_sets_and_orders(idx):
    rec = POS[idx]
    b = replay(rec)
    for p in range(4):
        ref = rec["players"][p]
        fr = O.legal_moves(b, p, O.ORDER_FRONTIER)
        nv = O.legal_moves(b, p, O.ORDER_NAIVE)
        assert len(fr) == ref["count"]
        assert _sha(fr) == ref["sha_frontier"]
        assert _sha(nv) == ref["sha_naive"]
        assert sorted(fr) == sorted(nv)
        assert O.legal_moves(b, p, O.ORDER_NAIVE_VIA_FRONTIER) == nv  # the naive CPU baseline's list
        if "frontier_list" in ref:
            assert fr == ref["frontier_list"]
            assert nv == ref["naive_list"]
        assert bool(O.lib().or_has_moves(O.C.byref(b), p)) == ref["has_moves"]


def test_rng_streams():
    g = load_golden("rng.json")
    for rec in g["randint"]:
        m = O.MT()
        O.lib().or_mt_seed_numpy(O.C.byref(m), rec["seed"])
        assert [O.lib().or_np_randint(O.C.byref(m), n) for n in rec["n"]] == rec["draws"]
    for rec in g["uint64"]:
        m = O.MT()
        O.lib().or_mt_seed_numpy(O.C.byref(m), rec["seed"])
        assert [str(O.lib().or_np_uint64(O.C.byref(m))) for _ in rec["draws"]] == rec["draws"]
    for rec in g["py_random"]:
        m = _py_seeded(rec["seed"])
        assert [O.lib().or_py_random(O.C.byref(m)).hex() for _ in rec["draws"]] == rec["draws"]
    for rec in g["py_choice"]:
        m = _py_seeded(rec["seed"])
        assert [O.lib().or_py_randbelow(O.C.byref(m), n) for n in rec["n"]] == rec["draws"]


def _py_seeded(seed):
    key = []
    a = abs(seed)
    while a:
        key.append(a & 0xFFFFFFFF)
        a >>= 32
    key = key or [0]
    m = O.MT()
    O.lib().or_mt_seed_python(O.C.byref(m), (O.C.c_uint32 * len(key))(*key), len(key))
    return m


@pytest.mark.parametrize("order_name,order", [("frontier", O.ORDER_FRONTIER), ("naive", O.ORDER_NAIVE)])
def test_arena_playouts(order_name, order):
    for rec in load_golden(f"playouts_{order_name}.json"):
        b = replay(POS[rec["position"]])
        res, trace = O.playout_arena(b, rec["agent_seeds"], order)
        assert trace == rec["trace"]
        assert list(res.scores) == rec["scores"]
        assert [p + 1 for p in range(4) if res.winner_mask >> p & 1] == rec["winner_ids"]
        assert res.passes == rec["passes"] and res.turns == rec["turn_count"]
        assert b.move_count == rec["moves_made"]


@pytest.mark.parametrize("order_name,order", [("frontier", O.ORDER_FRONTIER), ("naive", O.ORDER_NAIVE)])
def test_mcts_rollouts_semantics_a(order_name, order):
    for rec in load_golden(f"rollouts_a_{order_name}.json"):
        b = replay(POS[rec["position"]])
        assert [O.board_score(b, p) for p in range(4)] == rec["start_scores"]
        reward, _ = O.rollout_a(b, rec["player"] - 1, rec["seed"], order)
        assert reward == rec["reward"]


def test_fastmcts_think():
    for rec in load_golden("fastmcts.json"):
        b = replay(POS[rec["position"]])
        mv, nodes, top = O.fastmcts(b, b.cur, rec["seed"], rec["iterations"])
        assert mv == rec["move"]
        assert nodes == rec["nodes"]
        assert [(t[0], t[1]) for t in top] == [(t[0], t[1]) for t in rec["top"]]
        for t, r in zip(top, rec["top"]):
            assert round(t[2], 4) == r[2]


def test_zobrist():
    for rec in load_golden("zobrist.json"):
        table = (O.C.c_uint64 * 2088)()
        O.lib().or_zobrist_table(rec["seed"], table)
        assert [str(x) for x in table[:10]] == rec["table_head"]
        assert [str(x) for x in table[2000:2004]] == rec["turn"]
        assert [str(x) for x in table[2004:2009]] == rec["piece_head"]
        for h, posrec in zip(rec["hashes"], POS[:12]):
            b = replay(posrec)
            assert str(O.lib().or_zobrist_hash(O.C.byref(b), table)) == h


def test_arena_full_games_match_run_single_game():
    """arena_runner.run_single_game (4 random agents, telemetry ON) from the empty board."""
    import hashlib as H
    for rec in load_golden("arena_small.json"):
        seats = rec["seat_assignment"]
        seeds = []
        for p in range(4):
            name = seats[str(p + 1)]
            payload = f"20260301|{rec['game_index']}|{name}|agent_seed".encode()
            seeds.append(int(H.sha256(payload).hexdigest()[:16], 16) % (2**31 - 1))
        b = O.new_board()
        res, _ = O.playout_arena(b, seeds, O.ORDER_FRONTIER)
        assert [res.scores[p] for p in range(4)] == [rec["final_scores"][str(p + 1)] for p in range(4)]
        assert [p + 1 for p in range(4) if res.winner_mask >> p & 1] == rec["winner_ids"]
        assert b.move_count == rec["moves_made"] and res.passes == rec["passes"]
        assert res.turns == rec["turn_count"]


MCTS = load_golden("mcts.json")


@pytest.mark.parametrize("case", range(len(MCTS)))
def test_mcts_search_matches_reference(case):
    """or_mcts vs MCTSAgent(rollout_agent=RandomAgent(seed)) searches: best move, every
    root child's (move, visits, total_reward), TT hits, rollout rewards in order, TT
    size and the rollout stream's final MT19937 state, over two consecutive calls."""
    c = MCTS[case]
    b = replay(POS[c["position"]])
    ztab = O.zobrist_table(c["zobrist_seed"])
    rng = O.numpy_mt(c["rollout_seed"])
    tt = O.TT() if c["use_tt"] else None
    hits, rewards = 0, []
    for call in c["calls"]:
        player = call["player"] - 1
        assert b.cur == player
        legal = O.legal_moves(b, player)
        assert len(legal) == call["n_legal"]
        if call["searched"]:
            res = O.mcts(b, player, c["iterations"], 1.414, c["max_rollout_moves"], ztab, rng, tt)
            assert res["move"] == call["move"]
            assert [list(x) for x in res["children"]] == call["root_children"]
            hits += res["hits"]
            rewards += [r for r, f in zip(res["rewards"].tolist(), res["hit_flags"].tolist()) if not f]
            assert hits == call["transposition_hits"]
            assert rewards == call["rollout_rewards"]
            assert (tt.count if tt else None) == call["tt_size"]
        else:
            assert call["move"] == (legal[0] if legal else None)
        assert rng.mti == call["rng_pos"]
        assert _sha(list(rng.mt)) == call["rng_sha"]
        if call["move"] is None:
            break
        O.place_move(b, player, call["move"])
        assert b.cur == (player + 1) % 4
