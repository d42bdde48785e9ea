"""Reference package path ``AlphaGo.training`` (SL, RL and value trainers)."""
