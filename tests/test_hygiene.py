"""Source-level checks of the production HIP library (CPU: no build or GPU needed)."""
import glob
import os

from alphago_amd import _build


def test_production_sources_have_no_process_global_switches():
    """Kernel choices are explicit op arguments (docs/ARCHITECTURE.md): no environment lookups in the
    production library's sources or the headers they include (round 5 left AGK_WGRAD_XCD behind)."""
    kd = os.path.join(_build.CSRC, "kernels")
    files = _build._hip_sources("prod") + sorted(glob.glob(os.path.join(kd, "*.h")))
    assert files
    bad = [f for f in files if "getenv" in open(f).read()]
    assert not bad, bad


def test_checkpoint_refuses_other_optimizer_or_hyperparameters(tmp_path):
    """A resume must keep the optimizer and its hyperparameters: an Adam checkpoint in an SGD trainer
    (moments dropped) or a different momentum / beta is refused instead of silently accepted."""
    import pytest
    import torch

    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.train import checkpoint as ckpt
    from alphago_amd.train.engine import make_policy_trainer

    def trainer(**kw):
        torch.manual_seed(0)
        return make_policy_trainer(PolicyNet(4, board=9, filters_per_layer=8, layers=2), 2, 0.01, backend="torch",
                                   device="cpu", **kw)

    path = str(tmp_path / "c.pt")
    ckpt.save(path, trainer(optimizer="adam"))
    st = ckpt.load(path)["trainer"]
    ckpt.load_trainer_state(trainer(optimizer="adam"), st)  # same optimizer: fine
    with pytest.raises(ValueError, match="optimizer"):
        ckpt.load_trainer_state(trainer(), st)  # SGD keeps no moments
    ckpt.save(path, trainer(optimizer="momentum", momentum=0.9))
    st = ckpt.load(path)["trainer"]
    with pytest.raises(ValueError, match="hyperparameters"):
        ckpt.load_trainer_state(trainer(optimizer="momentum", momentum=0.5), st)
    ckpt.load_trainer_state(trainer(optimizer="momentum", momentum=0.9), st)


def test_value_trainer_defaults_match_the_cli():
    """models/value.py value_trainer.train uses train-value's defaults (Adam 3e-4, decay 0), not the
    paper's SGD(0.003) that round 4/5 measured at the constant predictor on this init."""
    import numpy as np

    from alphago_amd.models.value import value_trainer
    from alphago_amd.train.value import DEFAULT_LR, DEFAULT_OPTIMIZER

    rng = np.random.default_rng(0)
    vt = value_trainer(rng.integers(0, 2, (16, 49, 9, 9), dtype=np.uint8), rng.choice([-1, 1], 16), minibatch=4,
                       device="cpu", board=9, filters_per_layer=8, layers=2, dense=8)
    vt.train(steps=2, backend="torch")
    sched = vt._trainer.sched
    assert sched.optimizer == DEFAULT_OPTIMIZER == "adam"
    assert sched.lr == DEFAULT_LR["adam"] == 3e-4 and sched.decay == 0.0
