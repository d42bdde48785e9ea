"""Value-network pipeline: self-play data generation + regression training.

The reference only declares the value network (AlphaGo/models/value.py:12-43;
``get_samples``/``train`` are TODO) and its trainer module is an empty file
(AlphaGo/training/reinforcement_value_trainer.py).  This implements the
paper's procedure:

generate: for each game draw U ~ Uniform{1..max_u}; the SL policy plays moves
  1..U-1, move U is uniformly random among sensible moves, then the RL policy
  plays to the end.  The position after move U is recorded together with the
  outcome z in {-1, 0, +1} from the perspective of the player to move there.
  One position per game (avoids correlated samples).  Thousands of games run
  in lock-step, two batched GPU forwards per ply.  Output: HDF5 with
  ``states`` (N, 49, S, S) uint8 (chunks of 64 rows, LZF) and ``outcomes``
  (N,) int8.  Under torchrun every rank plays its own games into a per-rank
  file and rank 0 merges them into ONE dataset (``merge_value_files``).
train: MSE regression with SGD (paper lr 0.003, value.py:8-9), DP across
  ranks (each rank loads only its shard of the permutation), HIP MFMA trunk +
  small fused head, random D4 augmentation; native checkpoint / ``--resume``
  (bit-identical) and ``--watchdog-timeout`` as in the SL trainer.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import List, Optional

import numpy as np
import torch

from .. import go
from ..data.dataset import PositionDataset, shard_rows
from ..features import VALUE_FEATURES, Preprocess
from ..io.h5lite import H5File, H5Writer
from ..models.policy import CNNPolicy, CNNValue
from ..parallel import dist as agdist
from ..parallel.launch import add_gpus_arg, cli_ranks, exit_status
from ..search.selfplay import BatchedSampler
from ..utils import faults
from ..utils.metrics import MetricsLogger, StepMetrics
from ..utils.watchdog import Watchdog, enable_collective_timeouts
from . import checkpoint as ckpt
from .engine import make_value_trainer

LEARNING_RATE = .003
DECAY = 8.664339379294006e-08
# Defaults of train-value (round 5): the reference's SGD(0.003) on its uniform(+-0.05) init does not learn
# a 12-layer value trunk (profiles/r4/raw/value_parity_keras_init_4ep.json: every arm at the constant
# predictor; profiles/r5/README.md: the material task).  Keras 1.0 Adam at 3e-4 learns it in fp32 and on
# the HIP path; --optimizer sgd --learning-rate 0.003 --init keras restores the reference configuration.
DEFAULT_OPTIMIZER = "adam"
DEFAULT_LR = {"sgd": LEARNING_RATE, "momentum": LEARNING_RATE, "adam": 3e-4}
DEFAULT_INIT = "keras"


def generate_positions(sl_policy: CNNPolicy, rl_policy: CNNPolicy, n_games: int, size: int = 19,
                       max_u: int = 450, max_moves: int = 600, temperature: float = 1.0, seed: int = 0,
                       features: Optional[List[str]] = None, native: Optional[bool] = None):
    """Returns (planes uint8 (N, F, S, S), outcomes int8 (N,)) with N <= n_games.  With GPU engines the
    games run on the pipelined native driver (search/lockstep.py); ``native=False`` keeps this loop."""
    rng = np.random.default_rng(seed)
    feats = Preprocess(features or VALUE_FEATURES)
    sl = BatchedSampler(sl_policy, temperature, seed=seed)
    rl = BatchedSampler(rl_policy, temperature, seed=seed + 1)
    U = rng.integers(1, max_u + 1, size=n_games)
    from ..search.lockstep import generate_value_positions_lockstep, lockstep_ok
    if native is None:
        native = lockstep_ok(sl, rl)
    if native:
        return generate_value_positions_lockstep(sl, rl, n_games, size, U, max_moves, feats.feature_list, seed)
    states = [go.GameState(size) for _ in range(n_games)]
    recorded = [None] * n_games
    rec_player = [0] * n_games
    for ply in range(max_moves):
        active = [i for i in range(n_games) if not states[i].is_end_of_game]
        if not active:
            break
        g_sl = [i for i in active if ply < U[i] - 1]
        g_rand = [i for i in active if ply == U[i] - 1]
        g_rl = [i for i in active if ply > U[i] - 1]
        for group, sampler in ((g_sl, sl), (g_rl, rl)):
            if group:
                moves, _, _ = sampler.select([states[i] for i in group], need_planes=False)
                for k, i in enumerate(group):
                    states[i].do_move(moves[k])
        for i in g_rand:
            mask = states[i].legal_mask(False)
            cand = np.flatnonzero(mask)
            mv = go.PASS_MOVE if len(cand) == 0 else divmod(int(rng.choice(cand)), size)
            states[i].do_move(mv)
            recorded[i] = feats.state_to_uint8(states[i])
            rec_player[i] = states[i].current_player
    keep = [i for i in range(n_games) if recorded[i] is not None]
    if not keep:
        return np.zeros((0, feats.output_dim, size, size), np.uint8), np.zeros(0, np.int8)
    planes = np.stack([recorded[i] for i in keep])
    z = np.array([states[i].get_winner() * rec_player[i] for i in keep], dtype=np.int8)
    return planes, z


def generate_cli(argv=None):
    p = argparse.ArgumentParser(description="Generate value-network training positions by self-play")
    p.add_argument("sl_json")
    p.add_argument("rl_json")
    p.add_argument("outfile")
    p.add_argument("--games", type=int, default=1024, help="games per rank")
    p.add_argument("--batch-games", type=int, default=512)
    p.add_argument("--max-u", type=int, default=450)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--keep-shards", action="store_true", help="keep the per-rank files after merging")
    add_gpus_arg(p)
    argv = list(sys.argv[1:] if argv is None else argv)
    a = p.parse_args(argv)
    code = cli_ranks("value-generate", a, argv)
    if code is not None:
        return code
    env = agdist.init_from_env()
    sl = CNNPolicy.load_model(a.sl_json, device=env.device)
    rl = CNNPolicy.load_model(a.rl_json, device=env.device)
    out = a.outfile if env.world_size == 1 else "%s.rank%d" % (a.outfile, env.rank)
    tmp = out + ".tmp"
    n = 0
    C = Preprocess(VALUE_FEATURES).output_dim
    S = sl.model.board
    with H5Writer(tmp) as f:
        f.attrs["features"] = np.array([x.encode() for x in VALUE_FEATURES])
        st = f.stream_dataset("states", (C, S, S), np.uint8, chunk_rows=STATE_CHUNK_ROWS, compression="lzf")
        zs = []
        done = 0
        while done < a.games:
            g = min(a.batch_games, a.games - done)
            planes, z = generate_positions(sl, rl, g, size=S, max_u=a.max_u,
                                           seed=a.seed * 100003 + env.rank * 1009 + done)
            st.append(planes)
            zs.append(z)
            done += g
            n += len(z)
        st.finish()
        f.create_dataset("outcomes", data=np.concatenate(zs) if zs else np.zeros(0, np.int8))
    os.replace(tmp, out)
    if env.world_size > 1:
        # one trainable dataset: rank 0 concatenates the per-rank files (chunk-sliced
        # streaming copy, constant memory) into ``outfile``
        agdist.barrier()
        if env.is_main:
            shards = ["%s.rank%d" % (a.outfile, r) for r in range(env.world_size)]
            merge_value_files(shards, a.outfile)
            if not a.keep_shards:
                for sh in shards:
                    os.remove(sh)
        agdist.barrier()
        tot = torch.tensor([float(n)], dtype=torch.float64,
                           device=env.device if env.backend == "nccl" else "cpu")
        agdist.all_reduce_sum_(tot)
        n = int(tot.item())
    return n


STATE_CHUNK_ROWS = 64


def merge_value_files(paths: List[str], outfile: str, block_rows: int = 4096) -> int:
    """Concatenate value-position files (states + outcomes) into one file with
    the same layout; rows are streamed a block at a time."""
    tmp = outfile + ".tmp"
    total = 0
    with H5Writer(tmp) as w:
        first = H5File(paths[0])
        shape = first["states"].shape[1:]
        if "features" in first.attrs:
            w.attrs["features"] = first.attrs["features"]
        first.close()
        st = w.stream_dataset("states", shape, np.uint8, chunk_rows=STATE_CHUNK_ROWS, compression="lzf")
        zs = []
        for pth in paths:
            with H5File(pth) as f:
                ds = f["states"]
                if ds.shape[1:] != shape:
                    raise ValueError("%s: row shape %s != %s" % (pth, ds.shape[1:], shape))
                for r0 in range(0, ds.shape[0], block_rows):
                    st.append(ds.read_rows(r0, r0 + block_rows))
                zs.append(np.asarray(f["outcomes"].read()).astype(np.int8))
                total += ds.shape[0]
        st.finish()
        w.create_dataset("outcomes", data=np.concatenate(zs) if zs else np.zeros(0, np.int8))
    os.replace(tmp, outfile)
    return total


class ValueDataset(PositionDataset):
    """Value positions (``states`` + ``outcomes``) of one rank's shard; same
    residency modes as the policy data (data/dataset.py)."""

    def __init__(self, path: str, device, rows: Optional[np.ndarray] = None, resident: str = "auto"):
        super().__init__(path, device, resident=resident, rows=rows, targets="outcomes")

    @property
    def z(self):
        return self.targets


def train_cli(argv=None):
    p = argparse.ArgumentParser(description="Train the value network on self-play positions")
    p.add_argument("model", help="value-network JSON (CNNValue.save_model)")
    p.add_argument("train_data")
    p.add_argument("out_directory")
    p.add_argument("--minibatch", "-B", type=int, default=32, help="per-GPU minibatch")
    p.add_argument("--epochs", "-E", type=int, default=10)
    p.add_argument("--learning-rate", "-r", type=float, default=None,
                   help="default: %s" % ", ".join("%s %g" % kv for kv in DEFAULT_LR.items()))
    p.add_argument("--decay", "-d", type=float, default=None,
                   help="Keras lr decay; default: the paper's %g for SGD, 0 for Adam (Keras 1.0 Adam has none)" % DECAY)
    p.add_argument("--optimizer", default=DEFAULT_OPTIMIZER, choices=["sgd", "momentum", "adam"],
                   help="Keras 1.0 SGD(lr, decay) / SGD(lr, momentum, decay, nesterov) / Adam(lr) (default %(default)s)")
    p.add_argument("--momentum", type=float, default=0.9, help="with --optimizer momentum")
    p.add_argument("--nesterov", action="store_true")
    p.add_argument("--init", default=DEFAULT_INIT, choices=["keras", "he"],
                   help="weights of a model JSON without a weights file: keras = uniform(+-0.05) (value.py:17,21), "
                        "he = fan-in scaled uniform (models/nets.py he_uniform_)")
    p.add_argument("--fp8-bf16-layers", default="",
                   help="--precision fp8: trunk layers kept in bf16, e.g. 0,11 (per-layer precision; default: all fp8, at parity with fp32 under Adam, profiles/r5)")
    p.add_argument("--train-val-test", nargs=3, type=float, default=[0.93, .05, .02])
    p.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp8"])
    p.add_argument("--fp8-scale-guard", type=int, default=0,
                   help="fp8: activation scale exponents fall at most this many binades per step (0: unguarded, "
                        "the default; a 1-binade guard collapsed more SL runs, profiles/r6/README.md)")
    p.add_argument("--resident", default="auto", choices=["auto", "yes", "no"])
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--metrics", default=None, help="JSONL metrics file (per-epoch and per-step records)")
    p.add_argument("--log-every", type=int, default=100,
                   help="with --metrics: one per-step record every N steps (0 = epoch records only)")
    p.add_argument("--verbose", "-v", action="store_true")
    p.add_argument("--checkpoint-every", type=int, default=0,
                   help="also write the native checkpoint every N steps (0: end of epoch only)")
    p.add_argument("--resume", action="store_true",
                   help="continue from out_directory/checkpoint.pt if it exists (exact step, RNG, cursor)")
    p.add_argument("--watchdog-timeout", type=float, default=0.0,
                   help="exit a rank that makes no progress for this many seconds (0: off)")
    add_gpus_arg(p)
    argv = list(sys.argv[1:] if argv is None else argv)
    a = p.parse_args(argv)
    code = cli_ranks("train-value", a, argv)
    if code is not None:
        return code
    env = agdist.init_from_env()
    dev = env.device
    world, rank = env.world_size, env.rank
    val = CNNValue.load_model(a.model, device=dev)
    with open(a.model) as f:
        has_weights = bool(json.load(f).get("weights_file"))
    if a.init == "he" and not has_weights:
        from ..models.nets import he_uniform_
        g = torch.Generator(device="cpu").manual_seed(a.seed)
        net_cpu = val.model.to("cpu")
        he_uniform_(net_cpu, generator=g)
        val.model = net_cpu.to(dev)
    lr = a.learning_rate if a.learning_rate is not None else DEFAULT_LR[a.optimizer]
    decay = a.decay if a.decay is not None else (0.0 if a.optimizer == "adam" else DECAY)
    with H5File(a.train_data) as f:
        n = f["states"].shape[0]
    perm = np.random.default_rng(a.seed).permutation(n)
    n_train = int(a.train_val_test[0] * n)
    n_val = int(a.train_val_test[1] * n)
    tr_idx, va_idx = perm[:n_train], perm[n_train:n_train + n_val]
    my_tr, my_va = shard_rows(tr_idx, rank, world), shard_rows(va_idx, rank, world)
    data = ValueDataset(a.train_data, dev, rows=np.concatenate([my_tr, my_va]), resident=a.resident)
    n_my_tr = len(my_tr)
    B = a.minibatch
    kw = {"optimizer": a.optimizer, "momentum": a.momentum if a.optimizer == "momentum" else 0.0,
          "nesterov": a.nesterov}
    if a.precision != "bf16":
        kw["precision"] = a.precision
        kw["fp8_bf16_layers"] = [int(x) for x in a.fp8_bf16_layers.split(",") if x.strip() != ""]
        kw["fp8_scale_guard"] = a.fp8_scale_guard
    backend = a.backend if a.backend != "auto" else ("hip" if dev.type == "cuda" else "torch")
    if backend == "torch":
        kw.pop("precision", None)
        kw.pop("fp8_bf16_layers", None)
        kw.pop("fp8_scale_guard", None)
    trainer = make_value_trainer(val.model, B, lr, decay, backend=backend, device=dev, **kw)
    gen = torch.Generator(device=dev)
    gen.manual_seed(a.seed + rank)
    if env.is_main:
        os.makedirs(a.out_directory, exist_ok=True)
    agdist.barrier()
    meta = {"epochs": [], "best_epoch": 0, "training_data": a.train_data, "model_file": a.model,
            "data": {"rows_per_rank": agdist.all_gather_object(len(data)) if env.distributed else [len(data)]}}
    if kw.get("fp8_bf16_layers"):
        # the weights file carries no per-layer precision: fp8 inference (HipTrunkInference precision="fp8")
        # runs every layer in fp8, so a net trained with bf16 layers should be evaluated in bf16
        meta["fp8_bf16_layers"] = sorted(kw["fp8_bf16_layers"])
        if env.is_main:
            import warnings
            warnings.warn("--fp8-bf16-layers %s: fp8 inference ignores per-layer precision (it runs every layer in "
                          "fp8); evaluate this net with precision bf16 to match its training" % meta["fp8_bf16_layers"])
    log = MetricsLogger(a.metrics if env.is_main else None)
    # per-step records: "acc" is the sign agreement of v and z (the trainer's metric sum)
    step_log = StepMetrics(log, a.log_every if a.metrics else 0, B * world, val.model.flops_per_position(), dev,
                           trainer)
    steps = max(1, n_train // (B * world))
    ck_path = os.path.join(a.out_directory, "checkpoint.pt")
    cursor, start_epoch, start_step = 0, 0, 0
    ls = torch.zeros((), device=dev, dtype=torch.float64)
    state = ckpt.load(ck_path) if a.resume else None
    if state is not None and "legacy" not in state:
        ckpt.load_trainer_state(trainer, state["trainer"])
        cursor, start_epoch, start_step = int(state["cursor"]), int(state["epoch"]), int(state["step"])
        gen.set_state(state["rng"][rank])
        ls.copy_(state["sums"][rank].to(dev))
        meta = state["metadata"]
        if a.verbose and env.is_main:
            print("resumed at epoch %d step %d" % (start_epoch, start_step), flush=True)

    def save_native(epoch, step):
        rng = agdist.all_gather_object(gen.get_state()) if env.distributed else [gen.get_state()]
        part = ls.detach().to("cpu", copy=True)
        part = agdist.all_gather_object(part) if env.distributed else [part]
        if env.is_main:
            ckpt.save(ck_path, trainer, cursor=cursor, epoch=epoch, step=step, rng=rng, sums=part, metadata=meta,
                      config=vars(a))

    enable_collective_timeouts()
    wd = Watchdog(a.out_directory if a.watchdog_timeout > 0 else None, rank, a.watchdog_timeout)
    if a.watchdog_timeout > 0:
        wd.start()
    for ep in range(start_epoch, a.epochs):
        t0 = time.perf_counter()
        for step in range(start_step, steps):
            gstep = ep * steps + step
            faults.maybe_inject(gstep, rank)
            x, z = data.batch(np.arange(cursor * B, (cursor + 1) * B) % max(1, n_my_tr))
            cursor += 1
            sym = torch.randint(0, 8, (B,), device=dev, dtype=torch.int32, generator=gen)
            l, c = trainer.step(x, z, sym)
            ls += l.double()
            step_log.on_step(gstep, ep, l, c)
            wd.beat(gstep)
            if a.checkpoint_every and (gstep + 1) % a.checkpoint_every == 0 and step + 1 < steps:
                save_native(ep, step + 1)
        start_step = 0
        tot = ls.clone()
        ls.zero_()
        agdist.all_reduce_sum_(tot)
        logs = {"loss": float(tot) / (steps * B * world)}
        if n_val:
            vl, vn = torch.zeros((), device=dev, dtype=torch.float64), 0
            mine = np.arange(n_my_tr, len(data))
            for i in range(0, len(mine) - B + 1, B):
                x, z = data.batch(mine[i:i + B])
                l, _ = trainer.evaluate(x, z)
                vl += l.double()
                vn += B
            st = torch.stack([vl, torch.tensor(float(vn), device=dev, dtype=torch.float64)])
            agdist.all_reduce_sum_(st)
            if float(st[1]) > 0:
                logs["val_loss"] = float(st[0]) / float(st[1])
        meta["epochs"].append(logs)
        key = "val_loss" if "val_loss" in logs else "loss"
        if logs[key] < meta["epochs"][meta["best_epoch"]][key]:
            meta["best_epoch"] = len(meta["epochs"]) - 1
        if env.is_main:
            val.save_weights(os.path.join(a.out_directory, "weights.%05d.hdf5" % ep))
            with open(os.path.join(a.out_directory, "metadata.json"), "w") as f:
                json.dump(meta, f)
            log.log(epoch=ep, positions_per_s=steps * B * world / (time.perf_counter() - t0), **logs)
            if a.verbose:
                print("epoch %d %s" % (ep, logs), flush=True)
        save_native(ep + 1, 0)
        agdist.barrier()
    wd.stop()
    data.close()
    return meta


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "generate":
        sys.exit(exit_status(generate_cli(sys.argv[2:])))
    sys.exit(exit_status(train_cli(sys.argv[2:] if len(sys.argv) > 1 and sys.argv[1] == "train" else sys.argv[1:])))
