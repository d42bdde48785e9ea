"""End-to-end SL training smoke (spec: reference tests/test_supervised_policy_trainer.py)."""
import json
import os

import numpy as np
import pytest
import torch

from alphago_amd.data.convert import GameConverter
from alphago_amd.models.policy import CNNPolicy
from alphago_amd.train.sl import run_training

REF = "/root/reference/tests/test_data"
FIXTURE = os.path.join(REF, "hdf5", "alphago-vs-lee-sedol-features.hdf5")


def _data(tmp_path):
    if os.path.exists(FIXTURE):
        return FIXTURE
    # no reference checkout: synthesise a small file in the same schema
    from alphago_amd.io.h5lite import H5Writer
    p = str(tmp_path / "synth.h5")
    rng = np.random.default_rng(0)
    with H5Writer(p) as f:
        f["states"] = rng.integers(0, 2, (200, 12, 19, 19), dtype=np.uint8)
        f["actions"] = rng.integers(0, 19, (200, 2), dtype=np.uint8)
    return p


def _model(tmp_path, device):
    pol = CNNPolicy(["board", "ones", "turns_since"], filters_per_layer=16, layers=5, device=device)
    j = str(tmp_path / "model.json")
    pol.save_model(j)
    return j


def test_train_one_epoch_cpu(tmp_path):
    out = str(tmp_path / "out")
    data = _data(tmp_path)
    meta = run_training([_model(tmp_path, "cpu"), data, out, "--epochs", "1", "-l", "64", "-B", "16",
                         "--backend", "torch"])
    for f in ("metadata.json", "shuffle.npz", "weights.00000.hdf5", "checkpoint.pt"):
        assert os.path.exists(os.path.join(out, f)), f
    assert len(meta["epochs"]) == 1 and "val_loss" in meta["epochs"][0]
    # resume continues numbering (reference overwrote weights.00000)
    meta = run_training([_model(tmp_path, "cpu"), data, out, "--epochs", "1", "-l", "64", "-B", "16",
                         "--backend", "torch", "--weights", "weights.00000.hdf5"])
    assert len(meta["epochs"]) == 2
    assert os.path.exists(os.path.join(out, "weights.00001.hdf5"))
    with open(os.path.join(out, "metadata.json")) as f:
        assert json.load(f)["training_data"] == data


@pytest.mark.gpu
def test_train_one_epoch_hip(tmp_path, cuda_device):
    out = str(tmp_path / "out")
    meta = run_training([_model(tmp_path, "cuda"), _data(tmp_path), out, "--epochs", "2", "-B", "32",
                         "--backend", "hip", "-r", "0.05"])
    assert len(meta["epochs"]) == 2
    assert os.path.exists(os.path.join(out, "weights.00001.hdf5"))
    assert meta["epochs"][1]["loss"] < meta["epochs"][0]["loss"] + 0.5


def _step_records(path):
    with open(path) as f:
        recs = [json.loads(line) for line in f]
    return [r for r in recs if "step" in r], [r for r in recs if "step" not in r]


def test_step_metrics_jsonl_cpu(tmp_path):
    """--metrics/--log-every: one per-step record every N steps (SURVEY.md §5 metrics row)
    next to the per-epoch record."""
    out = str(tmp_path / "out")
    mpath = str(tmp_path / "m.jsonl")
    run_training([_model(tmp_path, "cpu"), _data(tmp_path), out, "--epochs", "1", "-l", "64", "-B", "8",
                  "--backend", "torch", "--metrics", mpath, "--log-every", "2"])
    steps, epochs = _step_records(mpath)
    assert [r["step"] for r in steps] == [2, 4, 6, 8]
    assert len(epochs) == 1
    for r in steps:
        assert r["world"] == 1 and r["positions_per_s"] > 0 and r["tflops"] > 0
        assert 0.0 <= r["acc"] <= 1.0 and np.isfinite(r["loss"])
        assert "allreduce_exposed_ms_per_step" not in r  # torch backend, one rank


@pytest.mark.gpu
def test_step_metrics_jsonl_hip(tmp_path, cuda_device):
    out = str(tmp_path / "out")
    mpath = str(tmp_path / "m.jsonl")
    run_training([_model(tmp_path, "cuda"), _data(tmp_path), out, "--epochs", "1", "-l", "128", "-B", "16",
                  "--backend", "hip", "--metrics", mpath, "--log-every", "4"])
    steps, _ = _step_records(mpath)
    assert [r["step"] for r in steps] == [4, 8]
    assert all(r["hbm_gb"] > 0 and r["positions_per_s"] > 0 for r in steps)


@pytest.mark.gpu
def test_train_sl_fp8_forward_hip(tmp_path, cuda_device):
    """train-sl --precision fp8: e4m3 block-scaled forward, bf16 backward, through the CLI."""
    out = str(tmp_path / "out")
    meta = run_training([_model(tmp_path, "cuda"), _data(tmp_path), out, "--epochs", "2", "-B", "32",
                         "--backend", "hip", "--precision", "fp8", "-r", "0.05"])
    assert len(meta["epochs"]) == 2 and np.isfinite(meta["epochs"][1]["loss"])


def test_chunk_cache_threaded_gather_matches_reads(tmp_path):
    """the prefetch worker and validation share one _ChunkCache; concurrent gathers
    from two threads must return exactly the rows a direct read returns."""
    import threading
    from alphago_amd.data.dataset import _ChunkCache
    from alphago_amd.io.h5lite import H5File, H5Writer
    p = str(tmp_path / "chunked.h5")
    rng = np.random.default_rng(1)
    states = rng.integers(0, 255, (900, 3, 5, 5), dtype=np.uint8)
    with H5Writer(p) as f:
        f.create_chunked("states", states, chunk_rows=16, compression="lzf")
    ds = H5File(p)["states"]
    assert ds.chunked
    cache = _ChunkCache(ds, capacity=4, threads=2)  # small: constant eviction
    errors = []

    def worker(seed):
        r = np.random.default_rng(seed)
        out = np.empty((32, 3, 5, 5), np.uint8)
        for _ in range(150):
            rows = r.integers(0, 900, 32)
            cache.gather(rows, out)
            if not np.array_equal(out, states[rows]):
                errors.append(seed)
                return

    ts = [threading.Thread(target=worker, args=(s,)) for s in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors


def test_streamed_chunked_data_with_validation_cpu(tmp_path):
    """--resident no on an LZF-chunked file with a validation split: the prefetch worker decodes
    ahead while the epoch-end validation reads the same chunk cache."""
    if not os.path.exists(FIXTURE):
        pytest.skip("reference fixture not present")
    out = str(tmp_path / "out")
    meta = run_training([_model(tmp_path, "cpu"), FIXTURE, out, "--epochs", "2", "-l", "256", "-B", "16",
                         "--backend", "torch", "--resident", "no"])
    assert meta["data"]["resident"] is False and meta["data"]["chunked"] is True
    assert len(meta["epochs"]) == 2
    assert all(np.isfinite(e["val_loss"]) for e in meta["epochs"])
