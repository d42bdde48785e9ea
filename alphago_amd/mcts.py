"""Reference module path ``AlphaGo.mcts`` (AlphaGo/mcts.py:4-175).

``TreeNode`` / ``MCTS`` keep the reference API (with the SURVEY Q3/Q4 fixes);
``ParallelMCTS`` -- an empty stub in the reference (mcts.py:174-175) -- is the
batched multi-tree search on the native forest (``alphago_amd.search.mcts``)."""
from .search.mcts import MCTS, BatchedMCTS, ParallelMCTS, TreeNode

__all__ = ["TreeNode", "MCTS", "ParallelMCTS", "BatchedMCTS"]
