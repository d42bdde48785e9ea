"""CLI, match harness, and driving an external GTP engine over a pipe."""
import json
import os
import subprocess
import sys

import pytest

from alphago_amd import go
from alphago_amd.cli import main as cli_main
from alphago_amd.gtp.client import GTPClientPlayer
from alphago_amd.search.arena import RandomPlayer, play_match

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_match_random_vs_random():
    res = play_match(RandomPlayer(1), RandomPlayer(2), n_games=2, size=7, max_moves=120)
    assert res["player1_wins"] + res["player2_wins"] + res["draws"] == 2


def test_external_gtp_engine(tmp_path):
    """Our own GTP front-end, launched as a subprocess, used as an external opponent."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "alphago_amd", "gtp", "--player", "random", "--size", "9"]
    eng = GTPClientPlayer(cmd)
    try:
        assert eng.name == "alphago_amd"
        gs = go.GameState(9)
        for _ in range(6):
            mv = eng.get_move(gs)
            assert gs.is_legal(mv)
            gs.do_move(mv)
        res = play_match(eng, RandomPlayer(3), n_games=2, size=9, max_moves=80,
                         sgf_dir=str(tmp_path / "sgf"))
        assert res["player1_wins"] + res["player2_wins"] + res["draws"] == 2
        assert len(os.listdir(str(tmp_path / "sgf"))) == 2
    finally:
        eng.close()


def test_cli_init_model_and_match(tmp_path, capsys):
    j = str(tmp_path / "p.json")
    w = str(tmp_path / "p.hdf5")
    cli_main(["init-model", "policy", j, "--weights", w, "--board", "9", "--filters", "8", "--layers", "2",
              "--features", "board,ones,turns_since"])
    spec = json.load(open(j))
    assert spec["weights_file"] == w
    capsys.readouterr()
    assert cli_main(["match", "policy:%s:greedy" % j, "random", "--games", "2", "--size", "9"]) == 0
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert res["player1_wins"] + res["player2_wins"] + res["draws"] == 2
