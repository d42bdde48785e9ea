"""Reference module path ``AlphaGo.ai`` (AlphaGo/ai.py:6-68): policy players.

Implementations live in ``alphago_amd.search.players`` (sensible-move masks from
the native featurizer, batched ``get_moves`` on the HIP inference engine)."""
from .search.players import GreedyPolicyPlayer, MCTSPlayer, ProbabilisticPolicyPlayer, sensible_moves

__all__ = ["GreedyPolicyPlayer", "ProbabilisticPolicyPlayer", "MCTSPlayer", "sensible_moves"]
