"""Serving: dynamic batching of network evaluations and an HTTP/JSON position service."""
from .batcher import BatcherPool, BatchingEvaluator, engine_eval_fn, latency_summary, state_eval_fn  # noqa: F401
from .server import GoService, make_server, position_from_moves, post_json, random_positions, serve_cli  # noqa: F401
