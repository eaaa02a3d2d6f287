"""Name-compatibility stub: the reference's agents/base_agent.py:1-3 is a docstring only.
The agent contract is duck-typed: select_action(board, player, legal_moves) -> Move | None."""
