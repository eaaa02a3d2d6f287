"""summary.json statistics (reference: analytics/tournament/arena_stats.py:22-350).

Same keys and formulas as the reference's compute_summary, so downstream tooling that
reads ``summary.json`` works on GPU-produced runs.
"""
from __future__ import annotations

import itertools
import json
import math
from pathlib import Path
from statistics import median
from typing import Any, Dict, Iterable, List, Mapping, Optional, Sequence, Union

import numpy as np


def load_games_jsonl(path: Union[str, Path]) -> List[Dict[str, Any]]:
    with Path(path).open("r", encoding="utf-8") as fh:
        return [json.loads(line) for line in fh if line.strip()]


def _mean(v: Sequence[float]) -> Optional[float]:
    return float(sum(v) / len(v)) if v else None


def _std(v: Sequence[float]) -> Optional[float]:
    if not v:
        return None
    m = _mean(v)
    return float(math.sqrt(sum((x - m) ** 2 for x in v) / len(v)))


def _percentile(v: Sequence[float], q: float) -> Optional[float]:
    """Linear interpolation between closest ranks (arena_stats.py:49-65)."""
    if not v:
        return None
    if q <= 0:
        return float(min(v))
    if q >= 1:
        return float(max(v))
    s = sorted(v)
    idx = (len(s) - 1) * q
    lo, hi = math.floor(idx), math.ceil(idx)
    if lo == hi:
        return float(s[lo])
    return float(s[lo] + (s[hi] - s[lo]) * (idx - lo))


def _safe_div(a: float, b: float) -> Optional[float]:
    return None if b == 0 else float(a / b)


def _to_float(x: Any) -> Optional[float]:
    try:
        return None if x is None else float(x)
    except (TypeError, ValueError):
        return None


def _score_summary(v: Sequence[float]) -> Dict[str, Optional[float]]:
    if not v:
        return {"count": 0, "mean": None, "median": None, "std": None, "p25": None, "p75": None,
                "min": None, "max": None}
    return {"count": len(v), "mean": _mean(v), "median": float(median(v)), "std": _std(v),
            "p25": _percentile(v, 0.25), "p75": _percentile(v, 0.75), "min": float(min(v)), "max": float(max(v))}


def _pairwise(games: Iterable[Mapping[str, Any]], names: Sequence[str]) -> Dict[str, Dict[str, Any]]:
    pw = {f"{a}__vs__{b}": {"agent_a": a, "agent_b": b, "a_beats_b": 0, "b_beats_a": 0, "tie": 0, "total": 0}
          for a, b in itertools.combinations(sorted(names), 2)}
    for g in games:
        if g.get("error"):
            continue
        sc = g.get("agent_scores") or {}
        for a, b in itertools.combinations(sorted(names), 2):
            if a not in sc or b not in sc:
                continue
            e = pw[f"{a}__vs__{b}"]
            e["total"] += 1
            sa, sb = int(sc[a]), int(sc[b])
            e["a_beats_b" if sa > sb else "b_beats_a" if sb > sa else "tie"] += 1
    return pw


def _efficiency(games, names, thinking, win_stats, score_stats):
    acc = {n: {"moves": 0.0, "total_time_ms": 0.0, "total_simulations": 0.0, "moves_with_simulations": 0.0,
               "all_move_times": []} for n in names}
    for g in games:
        if g.get("error"):
            continue
        for n, st in (g.get("agent_move_stats") or {}).items():
            if n not in acc:
                continue
            a = acc[n]
            a["moves"] += float(st.get("moves", 0))
            a["total_time_ms"] += _to_float(st.get("total_time_ms")) or 0.0
            a["all_move_times"].extend(st.get("move_times_ms", []))
            sims = _to_float(st.get("total_simulations"))
            if sims is not None:
                a["total_simulations"] += sims
                a["moves_with_simulations"] += float(st.get("moves_with_simulations", 0))
    out = {}
    for n in names:
        a = acc[n]
        moves, tot_ms, sims, sim_moves = a["moves"], a["total_time_ms"], a["total_simulations"], a["moves_with_simulations"]
        avg_ms = _safe_div(tot_ms, moves)
        tt = thinking.get(n)
        win_rate = float(win_stats.get(n, {}).get("win_rate", 0.0))
        mean_score = _to_float(score_stats.get(n, {}).get("mean")) or 0.0
        avg_s = (avg_ms or 0.0) / 1000.0
        times = a["all_move_times"]
        out[n] = {
            "moves": moves, "total_time_ms": tot_ms, "avg_time_ms_per_move": avg_ms,
            "move_time_ms_p50": float(np.percentile(times, 50)) if times else None,
            "move_time_ms_p95": float(np.percentile(times, 95)) if times else None,
            "move_time_ms_max": float(np.max(times)) if times else None,
            "configured_thinking_time_ms": float(tt) if tt is not None else None,
            "avg_budget_utilization": _safe_div(avg_ms or 0.0, float(tt)) if tt else None,
            "total_simulations": sims if sim_moves > 0 else None,
            "avg_simulations_per_move": _safe_div(sims, sim_moves) if sim_moves > 0 else None,
            "simulations_per_second": _safe_div(sims, tot_ms / 1000.0) if sim_moves > 0 else None,
            "win_rate_per_second": _safe_div(win_rate, avg_s) if avg_s > 0 else None,
            "score_per_second": _safe_div(mean_score, avg_s) if avg_s > 0 else None,
        }
    return out


def compute_summary(games: Sequence[Mapping[str, Any]], *, run_id: str, run_seed: int, seat_policy: str,
                    agent_names: Sequence[str], thinking_time_ms_by_agent: Mapping[str, Optional[int]],
                    run_config: Mapping[str, Any]) -> Dict[str, Any]:
    """arena_stats.py:247-350: win points (ties share a win), seat breakdown, score
    distributions, pairwise head-to-head counts, time/simulation efficiency."""
    win_stats = {n: {"games_played": 0.0, "outright_wins": 0.0, "shared_wins": 0.0, "win_points": 0.0,
                     "win_rate": 0.0} for n in agent_names}
    wins_by_seat = {n: {str(s): 0.0 for s in range(4)} for n in agent_names}
    games_by_seat = {n: {str(s): 0 for s in range(4)} for n in agent_names}
    completed = errors = 0
    for g in games:
        if g.get("error"):
            errors += 1
            continue
        completed += 1
        winners = list(g.get("winner_agents") or [])
        share = 1.0 / len(winners) if winners else 0.0
        for pid, name in (g.get("seat_assignment") or {}).items():
            name, seat = str(name), int(pid) - 1
            if name not in win_stats:
                continue
            win_stats[name]["games_played"] += 1
            games_by_seat[name][str(seat)] += 1
            if name in winners:
                win_stats[name]["outright_wins" if len(winners) == 1 else "shared_wins"] += 1
                win_stats[name]["win_points"] += share
                wins_by_seat[name][str(seat)] += share
    for n in agent_names:
        gp = win_stats[n]["games_played"]
        win_stats[n]["win_rate"] = float(win_stats[n]["win_points"] / gp) if gp else 0.0
    seat_breakdown = {n: {str(s): {"games": games_by_seat[n][str(s)], "win_points": wins_by_seat[n][str(s)],
                                   "win_rate": float(wins_by_seat[n][str(s)] / games_by_seat[n][str(s)])
                                   if games_by_seat[n][str(s)] else 0.0} for s in range(4)} for n in agent_names}
    scores: Dict[str, List[float]] = {n: [] for n in agent_names}
    for g in games:
        if g.get("error"):
            continue
        for n, sc in (g.get("agent_scores") or {}).items():
            if n in scores:
                scores[n].append(float(sc))
    score_stats = {n: _score_summary(v) for n, v in scores.items()}
    pw = _pairwise(games, agent_names)
    return {
        "run_id": run_id, "seed": run_seed, "seat_policy": seat_policy, "num_games": len(games),
        "completed_games": completed, "error_games": errors, "run_config": dict(run_config),
        "win_stats": win_stats, "wins_by_seat": seat_breakdown, "score_stats": score_stats,
        "pairwise_matchups": pw, "pairwise_total_comparisons": sum(e["total"] for e in pw.values()),
        "time_sim_efficiency": _efficiency(games, agent_names, thinking_time_ms_by_agent, win_stats, score_stats),
        "game_duration_sec": _score_summary([_to_float(g.get("duration_sec")) or 0.0 for g in games
                                             if not g.get("error")]),
    }
