"""MI355X-native rebuild of the Blokus legal-move generator and random-rollout loop.

Host-side mirror of the reference API (engine/, agents/, mcts/) over hand-written
HIP kernels for gfx950 reached through a ctypes C-ABI (include/blokus_hip.h).
"""
__version__ = "0.1.0"
