"""Value-network training throughput (BASELINE config 5: "Value-net training
from self-play positions, DP=8, fp8 MFMA conv path").

Paper/reference value net (AlphaGo/models/value.py:12-31): 49 planes, 5x5 +
11x 3x3 convs of 152 filters (160-wide tiles), 1x1 conv, Dense(256),
Dense(1, tanh); MSE.  Data (--data material, default): random-game positions
labelled tanh of their stone / atari balance (data/synthetic.py
value_material_pool); --data teacher: labelled by a fixed random-init value
teacher of the same architecture; with a held-out MSE after the timed steps
and --quality-steps more; --data random: random planes and +-1 outcomes
(speed only).  Random-init student, train-value's optimizer defaults (Adam).
Runs under torchrun for DP (RCCL all-reduce).

    python benchmarks/value_training_benchmark.py --precision fp8 --steps 20
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/value_training_benchmark.py
Prints one JSON line (rank 0): positions/s for the whole job, ms/step, MSE.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alphago_amd.models.nets import ValueNet  # noqa: E402
from alphago_amd.parallel import dist as agdist  # noqa: E402
from alphago_amd.train.engine import make_value_trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024, help="per-GPU minibatch")
    ap.add_argument("--filters", type=int, default=152)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--precision", default="fp8", choices=["bf16", "fp8"])
    ap.add_argument("--pool", type=int, default=65536)
    ap.add_argument("--heldout", type=int, default=2048)
    ap.add_argument("--data", default="material", choices=["material", "teacher", "random"],
                    help="material (default): tanh of the stone / atari balance, learnable in a few hundred steps; "
                         "teacher: a random-init value teacher's outputs; random: +-1 outcomes (speed only)")
    ap.add_argument("--quality-steps", type=int, default=1600,
                    help="after the clock: this many more steps before the held-out MSE (0: none)")
    ap.add_argument("--optimizer", default=None, choices=["sgd", "momentum", "adam"],
                    help="default: train-value's (train/value.py DEFAULT_OPTIMIZER)")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--conv-tile", type=int, default=0, choices=[0, 64, 128, 256, 384, 385, 386, 387],
                    help="forward/dgrad conv tiling (0 = automatic)")
    ap.add_argument("--overlap", action="store_true", help="wgrad on a second stream beside the dgrad")
    ap.add_argument("--fp8-dgrad", action="store_true", help="(default with the fp8 wgrad) fp8 precision: e5m2 x e4m3 dgrad")
    ap.add_argument("--no-fp8-dgrad", action="store_true", help="fp8 precision: keep the bf16 dgrad")
    ap.add_argument("--fp8-wgrad", action="store_true", help="(default) fp8 precision: e5m2 x e4m3 wgrad (160-wide layers)")
    ap.add_argument("--no-fp8-wgrad", action="store_true", help="fp8 precision: keep the bf16 wgrad")
    a = ap.parse_args()
    env = agdist.init_from_env()
    dev = env.device
    torch.manual_seed(7 + env.rank)
    net = ValueNet(49, filters_per_layer=a.filters, layers=a.layers)
    kw = ({"precision": a.precision, "conv_tile": a.conv_tile, "overlap": True if a.overlap else None,
           "fp8_dgrad": False if a.no_fp8_dgrad else (True if a.fp8_dgrad else None),
           "fp8_wgrad": not a.no_fp8_wgrad} if dev.type == "cuda" else {})
    from alphago_amd.train.value import DECAY, DEFAULT_LR, DEFAULT_OPTIMIZER
    opt = a.optimizer or DEFAULT_OPTIMIZER
    lr = a.lr if a.lr is not None else DEFAULT_LR[opt]
    kw.update(optimizer=opt, momentum=0.9 if opt == "momentum" else 0.0)
    tr = make_value_trainer(net, a.batch, lr=lr, decay=0.0 if opt == "adam" else DECAY, device=dev, **kw)
    g = torch.Generator(device=dev).manual_seed(11 + env.rank)
    t_data = time.perf_counter()
    if a.data == "material":
        from alphago_amd.data.synthetic import value_material_pool
        planes, tz = value_material_pool(a.pool + a.heldout, seed=1 + env.rank)
        allp, allz = torch.from_numpy(planes).to(dev), torch.from_numpy(tz).to(dev)
        pool, pz = allp[:a.pool], allz[:a.pool]
        hp, hz = allp[a.pool:], allz[a.pool:]
    elif a.data == "teacher":
        import numpy as np

        from alphago_amd.data.synthetic import random_game_states, value_teacher, value_teacher_pool
        from alphago_amd.features import VALUE_FEATURES, Preprocess
        probe = Preprocess(VALUE_FEATURES).states_to_uint8(random_game_states(1024, np.random.default_rng(0)))
        teacher = value_teacher(49, a.filters, a.layers, device=dev, probe=probe)
        planes, tz = value_teacher_pool(a.pool + a.heldout, teacher, seed=1 + env.rank)
        del teacher
        allp, allz = torch.from_numpy(planes).to(dev), torch.from_numpy(tz).to(dev)
        pool, pz = allp[:a.pool], allz[:a.pool]
        hp, hz = allp[a.pool:], allz[a.pool:]
    else:
        pool = torch.randint(0, 2, (a.pool, 49, 19, 19), dtype=torch.uint8, device=dev, generator=g)
        pz = (torch.randint(0, 2, (a.pool,), device=dev, generator=g) * 2 - 1).float()
        hp = hz = None
    t_data = time.perf_counter() - t_data

    def batch():
        """One random minibatch of the resident pool: the pool and the drawn rows (the HIP input-pack
        kernel gathers the boards itself; the torch backend index_selects)."""
        idx = torch.randint(0, a.pool, (a.batch,), device=dev, generator=g)
        sym = torch.randint(0, 8, (a.batch,), device=dev, dtype=torch.int32, generator=g)
        return pool, pz.index_select(0, idx), sym, None, idx

    ls = torch.zeros((), device=dev, dtype=torch.float64)
    for _ in range(a.warmup):  # the exact timed body: every kernel is loaded before the clock starts
        l, _ = tr.step(*batch())
        ls += l.double()
    ls.zero_()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    agdist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        l, _ = tr.step(*batch())
        ls += l.double()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    agdist.barrier()
    dt = agdist.all_reduce_max(time.perf_counter() - t0)
    agdist.all_reduce_sum_(ls)
    n = env.world_size
    pos = a.batch * n * a.steps
    heldout = None
    if hp is not None:  # after the clock: more training, then the held-out MSE (whole batches)
        for _ in range(a.quality_steps):
            tr.step(*batch())
        se = torch.zeros((), device=dev, dtype=torch.float64)
        cnt = 0
        for i in range(0, hp.shape[0] - a.batch + 1, a.batch):
            se += tr.evaluate(hp[i:i + a.batch], hz[i:i + a.batch])[0].double()
            cnt += a.batch
        heldout = {"heldout_mse": round(float(se) / max(cnt, 1), 5), "heldout_var": round(float(hz.var()), 5),
                   "heldout_n": cnt, "trained_steps": a.warmup + a.steps + a.quality_steps, "optimizer": opt,
                   "lr": lr}
    if env.is_main:
        print(json.dumps({"metric": "value-net training positions/s (whole job)", "value": round(pos / dt, 1),
                          "unit": "positions/s", "n_gpus": n, "ms_per_step": round(dt / a.steps * 1e3, 3),
                          "precision": a.precision if dev.type == "cuda" else "fp32", "mse": round(float(ls) / pos, 4),
                          "config": {"model": "value net %d-layer %d filters 49 planes" % (a.layers, a.filters),
                                     "global_batch": a.batch * n, "parallelism": "dp%d" % n},
                          **(heldout or {}), "data_s": round(t_data, 1),
                          "data": {"material": "random-game positions labelled tanh(stone + atari balance) "
                                               "(synthetic), random-init student",
                                   "teacher": "value-teacher-labelled random-game positions (synthetic), "
                                              "random-init student",
                                   "random": "synthetic positions/outcomes, random-init weights"}[a.data]}),
              flush=True)
    agdist.shutdown()


if __name__ == "__main__":
    main()
