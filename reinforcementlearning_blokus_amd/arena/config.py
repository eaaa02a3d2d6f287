"""Run configuration and seeding (analytics/tournament/arena_runner.py:40-292)."""
from __future__ import annotations

import hashlib
import json
import random
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Sequence

DEFAULT_OUTPUT_ROOT = "arena_runs"
DEFAULT_MAX_TURNS = 2500
SUPPORTED_SEAT_POLICIES = {"randomized", "round_robin"}
DEFAULT_SNAPSHOT_PLYS = [8, 16, 24, 32, 40, 48, 56, 64]


@dataclass(frozen=True)
class AgentConfig:
    name: str
    type: str
    thinking_time_ms: Optional[int] = None
    params: Dict[str, Any] = field(default_factory=dict)

    @classmethod
    def from_dict(cls, item: Mapping[str, Any]) -> "AgentConfig":
        if "name" not in item:
            raise ValueError("Agent entries must include 'name'")
        if "type" not in item:
            raise ValueError(f"Agent '{item['name']}' is missing required field 'type'")
        params = dict(item.get("params") or {})
        params.update({k: v for k, v in item.items() if k not in {"name", "type", "thinking_time_ms", "params"}})
        tt = item.get("thinking_time_ms")
        return cls(name=str(item["name"]), type=str(item["type"]),
                   thinking_time_ms=int(tt) if tt is not None else None, params=params)

    def to_dict(self) -> Dict[str, Any]:
        return {"name": self.name, "type": self.type, "thinking_time_ms": self.thinking_time_ms,
                "params": dict(self.params)}


@dataclass(frozen=True)
class SnapshotConfig:
    """Snapshot datasets (ML features) are outside the hot path: only ``enabled=False``
    is supported; the field is kept so reference configs load unchanged."""
    enabled: bool = False
    strategy: str = "fixed_ply"
    checkpoints: List[int] = field(default_factory=lambda: list(DEFAULT_SNAPSHOT_PLYS))

    @classmethod
    def from_dict(cls, item: Mapping[str, Any]) -> "SnapshotConfig":
        cps = item.get("checkpoints", list(DEFAULT_SNAPSHOT_PLYS))
        if not isinstance(cps, list):
            raise ValueError("snapshots.checkpoints must be a list of integers")
        return cls(enabled=bool(item.get("enabled", False)), strategy=str(item.get("strategy", "fixed_ply")),
                   checkpoints=sorted({int(v) for v in cps if int(v) >= 0}))

    def validate(self) -> None:
        if self.strategy != "fixed_ply":
            raise ValueError(f"Unsupported snapshot strategy '{self.strategy}'. Supported values: ['fixed_ply'].")
        if self.enabled:
            raise ValueError("snapshot datasets are not supported by the GPU arena (out of scope)")

    def to_dict(self) -> Dict[str, Any]:
        return {"enabled": self.enabled, "strategy": self.strategy, "checkpoints": list(self.checkpoints)}


@dataclass(frozen=True)
class RunConfig:
    agents: List[AgentConfig]
    num_games: int
    seed: int
    seat_policy: str = "randomized"
    output_root: str = DEFAULT_OUTPUT_ROOT
    max_turns: int = DEFAULT_MAX_TURNS
    notes: str = ""
    snapshots: SnapshotConfig = field(default_factory=SnapshotConfig)

    @classmethod
    def from_dict(cls, config: Mapping[str, Any]) -> "RunConfig":
        agents_raw = config.get("agents")
        if agents_raw is None:
            agents_raw = _legacy_agents_to_list(config)
        if not isinstance(agents_raw, list):
            raise ValueError("RunConfig 'agents' must be a list.")
        snaps = config.get("snapshots") or {}
        if not isinstance(snaps, Mapping):
            raise ValueError("RunConfig 'snapshots' must be an object when provided.")
        rc = cls(agents=[AgentConfig.from_dict(a) for a in agents_raw], num_games=int(config.get("num_games", 100)),
                 seed=int(config.get("seed", 0)), seat_policy=str(config.get("seat_policy", "randomized")),
                 output_root=str(config.get("output_root", DEFAULT_OUTPUT_ROOT)),
                 max_turns=int(config.get("max_turns", DEFAULT_MAX_TURNS)), notes=str(config.get("notes", "")),
                 snapshots=SnapshotConfig.from_dict(snaps))
        rc.validate()
        return rc

    def validate(self) -> None:
        if self.num_games <= 0:
            raise ValueError("num_games must be > 0.")
        if len(self.agents) != 4:
            raise ValueError(f"Arena expects exactly 4 agents; received {len(self.agents)}.")
        if len({a.name for a in self.agents}) != len(self.agents):
            raise ValueError("Agent names must be unique.")
        if self.seat_policy not in SUPPORTED_SEAT_POLICIES:
            raise ValueError(f"Unsupported seat_policy '{self.seat_policy}'. "
                             f"Expected one of {sorted(SUPPORTED_SEAT_POLICIES)}.")
        if self.max_turns <= 0:
            raise ValueError("max_turns must be > 0.")
        self.snapshots.validate()

    def to_dict(self) -> Dict[str, Any]:
        return {"agents": [a.to_dict() for a in self.agents], "num_games": self.num_games, "seed": self.seed,
                "seat_policy": self.seat_policy, "output_root": self.output_root, "max_turns": self.max_turns,
                "notes": self.notes, "snapshots": self.snapshots.to_dict()}

    @property
    def agent_names(self) -> List[str]:
        return [a.name for a in self.agents]


def _legacy_agents_to_list(config: Mapping[str, Any]) -> List[Dict[str, Any]]:
    """scripts/arena_config.json shape: {name: {type, time_limit | thinking_time_ms, ...}}."""
    out: List[Dict[str, Any]] = []
    for name, item in config.items():
        if not isinstance(item, Mapping) or "type" not in item:
            continue
        tt = item.get("thinking_time_ms")
        if tt is None and item.get("time_limit") is not None:
            tt = int(float(item["time_limit"]) * 1000)
        out.append({"name": str(name), "type": str(item["type"]), "thinking_time_ms": tt,
                    "params": {k: v for k, v in item.items() if k not in {"type", "thinking_time_ms"}}})
    if not out:
        raise ValueError("Invalid run config: missing 'agents' list and no legacy agent entries were found.")
    return out


def load_run_config(config_path: str) -> RunConfig:
    with Path(config_path).open("r", encoding="utf-8") as fh:
        payload = json.load(fh)
    if not isinstance(payload, Mapping):
        raise ValueError("Run config must be a JSON object.")
    return RunConfig.from_dict(payload)


def stable_hash_int(*parts: Any, mod: int = 2**31 - 1) -> int:
    """sha256 of the '|'-joined parts, first 16 hex digits, mod 2^31-1 (:241-245)."""
    return int(hashlib.sha256("|".join(str(p) for p in parts).encode("utf-8")).hexdigest()[:16], 16) % mod


def game_seed_from_run_seed(run_seed: int, game_index: int) -> int:
    return stable_hash_int(run_seed, game_index, "game_seed")


def agent_seed(run_seed: int, game_index: int, agent_name: str) -> int:
    return stable_hash_int(run_seed, game_index, agent_name, "agent_seed")


def seat_assignment_for_game(agent_names: Sequence[str], game_index: int, game_seed: int,
                             seat_policy: str) -> Dict[str, str]:
    """Seat -> agent name (:279-292): round_robin rotates, randomized shuffles with
    random.Random(stable_hash_int(game_seed, 'seat_assignment'))."""
    order = list(agent_names)
    if seat_policy == "round_robin":
        shift = game_index % len(order)
        order = order[shift:] + order[:shift]
    else:
        random.Random(stable_hash_int(game_seed, "seat_assignment")).shuffle(order)
    return {str(pv): order[i] for i, pv in enumerate((1, 2, 3, 4))}
