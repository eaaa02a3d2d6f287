"""The oracle's HeuristicAgent restatement (oracle/pyoracle.py heuristic_*) against the
reference's own outputs (tests/golden/heuristic.json): per-move scores bit for bit,
softmax probabilities, 12-ply heuristic self-play traces and two full 4-heuristic games.
CPU only; this pins the checker the GPU heuristic tests use."""
import hashlib

import numpy as np
import pytest

from oracle import pyoracle as O
from tests.conftest import load_golden
from tests.helpers import POS, replay

H = load_golden("heuristic.json")


def _sha(items):
    return hashlib.sha256(",".join(str(i) for i in items).encode()).hexdigest()


@pytest.mark.parametrize("case", range(len(H["cases"])))
def test_scores_and_probabilities(case):
    c = H["cases"][case]
    b = replay(POS[c["position"]])
    p = c["player"] - 1
    moves = O.legal_moves(b, p, O.ORDER_FRONTIER)
    assert len(moves) == c["n_legal"]
    assert _sha(moves) == c["moves_sha"]
    scores = [O.heuristic_score(b, p, m) for m in moves]
    assert _sha(float(x).hex() for x in scores) == c["scores_sha"]
    if "scores" in c:
        assert [float(x).hex() for x in scores] == c["scores"]


@pytest.mark.parametrize("case", range(len(H["cases"])))
def test_selfplay_traces(case):
    """12 turns of heuristic self-play, one HeuristicAgent(seed * 10 + player) per seat."""
    c = H["cases"][case]
    b = replay(POS[c["position"]])
    rngs = [np.random.RandomState(c["seed"] * 10 + p + 1) for p in range(4)]
    trace = []
    for _ in range(12):
        if all(not O.legal_moves(b, q, O.ORDER_FRONTIER) for q in range(4)):
            break
        p = b.cur
        mv = O.heuristic_choice(b, p, rngs[p])
        if mv is None:
            trace.append(-1)
            b.cur = (b.cur + 1) & 3
            continue
        trace.append(mv)
        O.place_move(b, p, mv)
    assert trace == c["selfplay_trace"]
    for p in range(4):
        st = rngs[p].get_state()
        assert [int(st[2]), _sha(int(x) for x in st[1])] == c["selfplay_rng"][str(p + 1)]


@pytest.mark.parametrize("game", range(len(H["games"])))
def test_full_games(game):
    g = H["games"][game]
    b = O.new_board()
    scores, wm, moves, passes, turns, trace = O.mixed_playout_arena(
        b, [g["seed"] + p + 1 for p in range(4)], 0xF)
    assert trace == g["trace"]
    assert list(scores) == g["scores"] and (passes, turns) == (g["passes"], g["turns"])
    assert [p + 1 for p in range(4) if wm >> p & 1] == g["winner_ids"]


def test_c_heuristic_score_equals_pinned_restatement():
    """or_heuristic_score (the C _evaluate_move behind the config-4 CPU baseline) equals
    pyoracle.heuristic_score, which tests/golden/heuristic.json pins to the reference."""
    from tests.helpers import POS, replay
    n = 0
    for rec in POS[:24]:
        b = replay(rec)
        for p in range(4):
            for mv in O.legal_moves(b, p, O.ORDER_FRONTIER)[::3]:
                assert O.lib().or_heuristic_score(O.C.byref(b), p, mv) == O.heuristic_score(b, p, mv)
                n += 1
    assert n > 1000


def test_c_arena4_game_runs_and_is_deterministic():
    """or_arena4_game (config-4 CPU baseline): a full mixed-seat game, reproducible."""
    a = O.arena4_game([0, 1, 2, 3], [5, 6, 7, 8], 8, 50)
    b = O.arena4_game([0, 1, 2, 3], [5, 6, 7, 8], 8, 50)
    assert a == b and a[0] > 40 and sum(a[1]) > 150
