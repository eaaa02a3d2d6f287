"""MCTS over the GPU engine (reference: mcts/)."""
