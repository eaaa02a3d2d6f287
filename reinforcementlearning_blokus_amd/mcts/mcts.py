"""Name-compatibility stub: the reference's mcts/mcts.py:1-3 is a docstring only; the
search lives in mcts_agent.py."""
