"""Command-line entry point: ``python -m alphago_amd <command> ...``

Commands
  convert        SGF -> HDF5 training data          (reference game_converter CLI)
  init-model     write a new policy/value model JSON (+ random weights)
  train-sl       supervised policy training          (reference supervised_policy_trainer CLI)
  train-rl       RL policy training by self-play     (reference reinforcement_policy_trainer CLI)
  value-generate self-play positions for the value net
  selfplay-mcts  batched MCTS self-play games (SGF + states / pi / outcomes HDF5)
  selfplay-to-sl MCTS self-play records -> SL training data (most-visited or played move targets)
  train-value    value-network regression
  gtp            run a GTP v2 engine on stdin/stdout (reference interface/gtp_wrapper)
  match          play games between two players (policy / mcts / random / external GTP)
  bench          the headline SL throughput benchmark (bench.py)
  serve          HTTP/JSON policy/value/genmove service with dynamic batching

Player specs (gtp/match): ``random``, ``policy:MODEL.json[:greedy|:T]``,
``mcts:POLICY.json[,VALUE.json]:PLAYOUTS``, ``gtp:COMMAND LINE``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import List, Optional


def make_player(spec: str, device=None):
    from .gtp.client import GTPClientPlayer
    from .models.policy import CNNPolicy, CNNValue
    from .search.arena import RandomPlayer
    from .search.players import GreedyPolicyPlayer, MCTSPlayer, ProbabilisticPolicyPlayer

    if spec == "random":
        return RandomPlayer()
    kind, _, rest = spec.partition(":")
    if kind == "gtp":
        return GTPClientPlayer(rest)
    if kind == "policy":
        path, _, opt = rest.partition(":")
        pol = CNNPolicy.load_model(path, device=device)
        if opt == "greedy":
            return GreedyPolicyPlayer(pol)
        return ProbabilisticPolicyPlayer(pol, temperature=float(opt) if opt else 1.0)
    if kind == "mcts":
        nets, _, n = rest.rpartition(":")
        if not nets:
            nets, n = n, "1600"
        paths = nets.split(",")
        pol = CNNPolicy.load_model(paths[0], device=device)
        val = CNNValue.load_model(paths[1], device=device) if len(paths) > 1 else None
        return MCTSPlayer(pol, val, n_playout=int(n))
    raise ValueError("unknown player spec %r" % spec)


def _init_model(argv):
    from .features import DEFAULT_FEATURES, VALUE_FEATURES
    from .models.policy import CNNPolicy, CNNValue

    p = argparse.ArgumentParser(prog="alphago_amd init-model")
    p.add_argument("kind", choices=["policy", "value"])
    p.add_argument("json_out")
    p.add_argument("--weights", default=None, help="also write random-init weights (Keras HDF5)")
    p.add_argument("--features", default=None, help="comma-separated feature list")
    p.add_argument("--board", type=int, default=19)
    p.add_argument("--filters", type=int, default=None)
    p.add_argument("--layers", type=int, default=12)
    p.add_argument("--seed", type=int, default=0)
    a = p.parse_args(argv)
    import torch

    torch.manual_seed(a.seed)
    if a.kind == "policy":
        feats = a.features.split(",") if a.features else DEFAULT_FEATURES
        m = CNNPolicy(feats, board=a.board, filters_per_layer=a.filters or 128, layers=a.layers, device="cpu")
    else:
        feats = a.features.split(",") if a.features else VALUE_FEATURES
        m = CNNValue(feats, board=a.board, filters_per_layer=a.filters or 152, layers=a.layers, device="cpu")
    m.save_model(a.json_out, a.weights)
    print(a.json_out)


def _gtp(argv):
    p = argparse.ArgumentParser(prog="alphago_amd gtp")
    p.add_argument("--player", default="random")
    p.add_argument("--size", type=int, default=19)
    a = p.parse_args(argv)
    from .gtp.engine import run_gtp

    run_gtp(make_player(a.player), size=a.size)


def _match(argv):
    p = argparse.ArgumentParser(prog="alphago_amd match")
    p.add_argument("player1")
    p.add_argument("player2")
    p.add_argument("--games", type=int, default=10)
    p.add_argument("--size", type=int, default=19)
    p.add_argument("--komi", type=float, default=7.5)
    p.add_argument("--sgf-dir", default=None)
    a = p.parse_args(argv)
    from .search.arena import play_match

    res = play_match(make_player(a.player1), make_player(a.player2), a.games, a.size, a.komi, sgf_dir=a.sgf_dir)
    print(json.dumps(res))
    return res


from .parallel.launch import ExitCode as _Exit  # noqa: E402  (explicit process exit codes)


def main(argv: Optional[List[str]] = None) -> int:
    """Dispatch a command; returns a process exit code."""
    r = _dispatch(list(sys.argv[1:] if argv is None else argv))
    return int(r) if isinstance(r, _Exit) else 0


def _dispatch(argv: List[str]):
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return _Exit(0)
    cmd, rest = argv[0], argv[1:]
    if cmd == "convert":
        from .data.convert import run_game_converter
        return run_game_converter(rest)
    if cmd == "init-model":
        return _init_model(rest)
    if cmd == "serve":
        from .serve.server import serve_cli
        return _Exit(serve_cli(rest))
    if cmd == "train-sl":
        from .train.sl import run_training
        return run_training(rest)
    if cmd == "train-rl":
        from .train.rl import run
        return run(rest)
    if cmd == "value-generate":
        from .train.value import generate_cli
        return generate_cli(rest)
    if cmd == "selfplay-mcts":
        from .search.selfplay_mcts import selfplay_cli
        return selfplay_cli(rest)
    if cmd == "selfplay-to-sl":
        from .data.selfplay_to_sl import selfplay_to_sl_cli
        return selfplay_to_sl_cli(rest)
    if cmd == "train-value":
        from .train.value import train_cli
        return train_cli(rest)
    if cmd == "gtp":
        return _gtp(rest)
    if cmd == "match":
        return _match(rest)
    if cmd == "bench":
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import bench
        sys.argv = ["bench.py"] + rest
        return _Exit(bench.main() or 0)
    print("unknown command %r\n%s" % (cmd, __doc__))
    return _Exit(2)


if __name__ == "__main__":
    sys.exit(main() or 0)
