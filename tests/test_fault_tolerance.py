"""Failure detection and recovery: native checkpoints resume
bit-identically, injected faults are recovered by resume / torchrun restarts,
and the watchdog turns a hang into a clean non-zero exit."""
import os
import socket
import subprocess
import sys

import pytest
import torch

from alphago_amd.train import checkpoint as ckpt
from alphago_amd.train.sl import run_training
from alphago_amd.utils import faults

from test_sl_training import _data

from alphago_amd.models.policy import CNNPolicy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model(tmp_path, device):
    """Model JSON + fixed initial weights (so separate runs start identically)."""
    torch.manual_seed(0)
    pol = CNNPolicy(["board", "ones", "turns_since"], filters_per_layer=16, layers=4, device=device)
    j = str(tmp_path / "model.json")
    pol.save_model(j, str(tmp_path / "init.hdf5"))
    return j


def _args(model, data, out, *extra):
    return [model, data, out, "--epochs", "2", "-l", "96", "-B", "16", "--backend", "torch",
            "--checkpoint-every", "2", "--resume", *extra]


def test_faults_parse():
    f = faults.parse("exit@12:rank1:once=/tmp/x")
    assert f == {"kind": "exit", "step": 12, "rank": 1, "once": "/tmp/x"}
    assert faults.parse(None) is None
    with pytest.raises(ValueError):
        faults.parse("boom@1")


def test_resume_after_injected_fault_is_bit_identical(tmp_path, monkeypatch):
    data = _data(tmp_path)
    model = _model(tmp_path, "cpu")
    ref_out = str(tmp_path / "ref")
    ref_meta = run_training(_args(model, data, ref_out))
    ref = ckpt.load(os.path.join(ref_out, "checkpoint.pt"))

    out = str(tmp_path / "faulty")
    marker = str(tmp_path / "fired")
    monkeypatch.setenv("ALPHAGO_AMD_FAULT", "raise@9:once=%s" % marker)  # epoch 1, step 3
    faults.reload_from_env()
    try:
        with pytest.raises(faults.InjectedFault):
            run_training(_args(model, data, out))
        assert os.path.exists(marker)
        mid = ckpt.load(os.path.join(out, "checkpoint.pt"))
        assert (mid["epoch"], mid["step"]) == (1, 2)  # last checkpoint before the fault
        meta = run_training(_args(model, data, out))  # marker present -> runs through
    finally:
        monkeypatch.delenv("ALPHAGO_AMD_FAULT")
        faults.reload_from_env()
    got = ckpt.load(os.path.join(out, "checkpoint.pt"))
    assert torch.equal(got["trainer"]["flat"], ref["trainer"]["flat"])
    assert got["trainer"]["iterations"] == ref["trainer"]["iterations"] == 12
    assert [e["loss"] for e in meta["epochs"]] == [e["loss"] for e in ref_meta["epochs"]]


def test_watchdog_exits_on_hang(tmp_path):
    code = ("import sys, time; sys.path.insert(0, %r)\n"
            "from alphago_amd.utils.watchdog import Watchdog\n"
            "w = Watchdog(%r, rank=3, timeout=1.0, interval=0.2).start()\n"
            "w.beat(7)\n"
            "time.sleep(30)\n") % (ROOT, str(tmp_path))
    r = subprocess.run([sys.executable, "-c", code], timeout=60, capture_output=True, text=True)
    assert r.returncode == 75, r.stderr
    txt = open(tmp_path / "hang.rank3.txt").read()
    assert "after step 7" in txt and "<module>" in txt  # message + the hung thread's stack
    assert os.path.exists(tmp_path / "heartbeat.rank3.json")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(args, env_extra, timeout=300):
    env = dict(os.environ)
    env.pop("ALPHAGO_AMD_FAULT", None)
    env.update(env_extra)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), "--max-restarts=1",
           "-m", "alphago_amd", "train-sl"] + args
    return subprocess.run(cmd, env=env, timeout=timeout, capture_output=True, text=True)


def test_torchrun_restart_recovers_crashed_rank(tmp_path):
    """A rank dies mid-epoch (os._exit); torchrun restarts the group, which
    resumes from the last checkpoint and ends with the same weights as an
    uninterrupted 2-rank run."""
    data = _data(tmp_path)
    model = _model(tmp_path, "cpu")
    r = _torchrun(_args(model, data, str(tmp_path / "ref")), {})
    assert r.returncode == 0, r.stderr[-3000:]
    marker = str(tmp_path / "fired")
    r = _torchrun(_args(model, data, str(tmp_path / "run")), {"ALPHAGO_AMD_FAULT": "exit@4:rank1:once=%s" % marker})
    assert r.returncode == 0, r.stderr[-3000:]
    assert os.path.exists(marker)
    a = ckpt.load(str(tmp_path / "ref" / "checkpoint.pt"))
    b = ckpt.load(str(tmp_path / "run" / "checkpoint.pt"))
    assert torch.equal(a["trainer"]["flat"], b["trainer"]["flat"])
    # the epoch metrics survive the restart too: every rank's partial epoch
    # sums are checkpointed and restored per rank (not rank 0's for all)
    import json
    ma = json.load(open(str(tmp_path / "ref" / "metadata.json")))
    mb = json.load(open(str(tmp_path / "run" / "metadata.json")))
    assert [e["loss"] for e in ma["epochs"]] == [e["loss"] for e in mb["epochs"]]
    assert [e["acc"] for e in ma["epochs"]] == [e["acc"] for e in mb["epochs"]]
    # each rank holds only its shard of the data
    n_rows = ma["data"]["rows_per_rank"]
    assert len(n_rows) == 2 and abs(n_rows[0] - n_rows[1]) <= 1
