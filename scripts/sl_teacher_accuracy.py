"""Top-1 accuracy of the SL pipeline on a learnable synthetic task (no expert
games are available offline): positions from random games, labelled with the
greedy move of a fixed random-init "teacher" policy network (12 x 192, 48
planes; alphago_amd/data/synthetic.py), written to the training-HDF5 schema,
then learned by a fresh student network through the real SL trainer CLI
(``train/sl.py run_training``).  The student's held-out top-1 agreement with
the teacher is the accuracy figure (reference metric:
supervised_policy_trainer.py:199-200).

H6 parity: ``--arms hip-bf16,hip-fp8fwd,torch-fp32`` trains the
same student initialisation on the same data and seeds with the HIP bf16
engine, the HIP fp8-forward engine and the fp32 PyTorch trainer.
``--real-epochs E`` adds a real-move check: each arm also trains on four of the
reference's Lee Sedol games (tests/test_data/sgf) and is scored on the fifth.

Usage: python scripts/sl_teacher_accuracy.py OUT_DIR [--positions N] [--epochs E] [--lr R] [--batch B]
       [--arms A,B,..] [--real-epochs E]
Prints one JSON line with the per-arm, per-epoch acc / val_acc."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alphago_amd.features import DEFAULT_FEATURES  # noqa: E402
from alphago_amd.io.h5lite import H5Writer  # noqa: E402
from alphago_amd.models.policy import CNNPolicy  # noqa: E402
from alphago_amd.train.sl import run_training  # noqa: E402


def _real_games(out, features):
    """The reference's five Lee Sedol games (tests/test_data/sgf) as 48-plane HDF5: the first four
    for training, the fifth held out (all of its positions: a game-level split)."""
    from alphago_amd.data.convert import GameConverter
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
    pre = (os.path.join(here, "lee_sedol_train.h5"), os.path.join(here, "lee_sedol_heldout.h5"))
    if all(os.path.exists(p) for p in pre):  # converted in-tree (the reference checkout is not on the GPU box)
        return pre[0], pre[1], "Lee-Sedol-vs-AlphaGo-20160315.sgf"
    sgf_dir = "/root/reference/tests/test_data/sgf"
    games = sorted(os.path.join(sgf_dir, f) for f in os.listdir(sgf_dir) if "Lee" in f) if os.path.isdir(sgf_dir) \
        else []
    if len(games) < 2:
        return None
    conv = GameConverter(features)
    tr, ho = os.path.join(out, "real_train.h5"), os.path.join(out, "real_heldout.h5")
    conv.sgfs_to_hdf5(games[:-1], tr, 19)
    conv.sgfs_to_hdf5(games[-1:], ho, 19)
    return tr, ho, os.path.basename(games[-1])


def _heldout_top1(model_json, weights, h5, dev):
    """Top-1 agreement of the trained student with the held-out file's moves (legal-masked argmax)."""
    from alphago_amd.io.h5lite import H5File
    f = H5File(h5)
    planes = np.asarray(f["states"].read())
    acts = np.asarray(f["actions"].read()).astype(np.int64)
    tgt = acts[:, 0] * 19 + acts[:, 1]
    pol = CNNPolicy.load_model(model_json, device=dev, weights_file=weights)
    probs = np.concatenate([pol.engine.evaluate(planes[i:i + 512]).float().cpu().numpy().copy()
                            for i in range(0, len(planes), 512)])
    return float((probs.argmax(1) == tgt).mean()), int(len(tgt))


def _uniform_baseline(h5):
    """Expected top-1 of a uniform pick over the sensible moves (the 'sensibleness' plane of
    DEFAULT_FEATURES: legal and not filling an own eye) -- the floor a trained net must beat."""
    from alphago_amd.io.h5lite import H5File
    planes = np.asarray(H5File(h5)["states"].read())
    sens = planes[:, 46].reshape(len(planes), -1)  # 48 planes: ..., sensibleness (46), zeros (47)
    n = sens.sum(1).clip(min=1)
    return float((1.0 / n).mean())


ARMS = {"hip-bf16": ["--backend", "hip"], "hip-fp8fwd": ["--backend", "hip", "--precision", "fp8"],
        "hip-fp8fwd-guard1": ["--backend", "hip", "--precision", "fp8", "--fp8-scale-guard", "1"],
        "torch-fp32": ["--backend", "torch"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--positions", type=int, default=131072)
    ap.add_argument("--epochs", type=int, default=8)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--arms", default="hip-bf16",
                    help="comma list of %s: the same data, student init and seeds per arm" % ",".join(ARMS))
    ap.add_argument("--real-seeds", type=int, default=1,
                    help="student initialisations / data orders averaged in the real-move check")
    ap.add_argument("--real-batch", type=int, default=32)
    ap.add_argument("--real-lr", type=float, default=0.0, help="real-move lr (0: --lr)")
    ap.add_argument("--real-only", action="store_true", help="skip the teacher task (real-move check only)")
    ap.add_argument("--real-epochs", type=int, default=0,
                    help=">0: also train each arm on 4 reference Lee Sedol games and report held-out top-1 on the "
                         "fifth (real moves)")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    small = dev.type == "cpu"
    F, L = (16, 3) if small else (192, 12)
    rng = np.random.default_rng(a.seed)
    t0 = time.perf_counter()
    h5 = os.path.join(a.out, "teacher.h5")
    acts = np.zeros((0, 2))
    if not a.real_only:
        torch.manual_seed(1000 + a.seed)
        teacher = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=F, layers=L, device=dev)
        with H5Writer(h5) as f:
            f.attrs["features"] = np.array([x.encode() for x in DEFAULT_FEATURES])
            f.attrs["board_size"] = np.int64(19)
            states_ds = f.stream_dataset("states", (teacher.preprocessor.output_dim, 19, 19), np.uint8)
            from alphago_amd.data.synthetic import teacher_pool
            planes, idx = teacher_pool(a.positions, teacher, seed=a.seed, symmetrize=False)
            states_ds.append(planes)
            states_ds.finish()
            acts = np.stack([idx // 19, idx % 19], axis=1).astype(np.uint8)
            f.create_dataset("actions", data=acts)
            f.create_group("file_offsets")["synthetic"] = np.array([0, len(acts)], dtype=np.int64)
        del teacher
    t_data = time.perf_counter() - t0
    real = _real_games(a.out, DEFAULT_FEATURES) if a.real_epochs > 0 else None
    results = {}
    for arm in [x for x in a.arms.split(",") if x]:
        torch.manual_seed(2000 + a.seed)  # the same student initialisation in every arm
        student = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=F, layers=L, device=dev)
        model_json = os.path.join(a.out, "student_%s.json" % arm)
        student.save_model(model_json)
        run_dir = os.path.join(a.out, "run_" + arm)
        t1 = time.perf_counter()
        res = {}
        if not a.real_only:
            run_training([model_json, h5, run_dir, "--minibatch", str(a.batch), "--epochs", str(a.epochs),
                          "--learning-rate", str(a.lr), "--decay", "0", "--no-symmetries", "--seed", str(a.seed)]
                         + ARMS[arm])
            ep = json.load(open(os.path.join(run_dir, "metadata.json")))["epochs"]
            res = {"acc": [round(e.get("acc", 0), 4) for e in ep],
                   "val_acc": [round(e.get("val_acc", 0), 4) for e in ep],
                   "train_s": round(time.perf_counter() - t1, 1)}
        if real is not None:
            tops = []
            for rs in range(a.real_seeds):
                torch.manual_seed(3000 + a.seed + rs)  # the same initialisation per seed in every arm
                stu = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=F, layers=L, device=dev)
                rj = os.path.join(a.out, "real_student_%s_%d.json" % (arm, rs))
                stu.save_model(rj)
                rdir = os.path.join(a.out, "real_%s_%d" % (arm, rs))
                run_training([rj, real[0], rdir, "--minibatch", str(a.real_batch), "--epochs", str(a.real_epochs),
                              "--learning-rate", str(a.real_lr or a.lr), "--decay", "0", "--seed",
                              str(a.seed + rs), "--train-val-test", "1.0", "0.0", "0.0"] + ARMS[arm])
                w = os.path.join(rdir, "weights.%05d.hdf5" % (a.real_epochs - 1))
                top1, n = _heldout_top1(rj, w, real[1], dev)
                tops.append(round(top1, 4))
            res["real_heldout_top1"] = round(float(np.mean(tops)), 4)
            res["real_heldout_top1_per_seed"] = tops
            res["real_heldout_positions"] = n
            res["real_heldout_game"] = real[2]
            res["real_uniform_sensible_baseline"] = round(_uniform_baseline(real[1]), 4)
        results[arm] = res
    print(json.dumps({"metric": "SL top-1 agreement with a random-init teacher policy (held-out)",
                      "positions": int(len(acts)), "epochs": a.epochs, "minibatch": a.batch, "lr": a.lr,
                      "chance": round(1.0 / 300, 4), "data_s": round(t_data, 1), "net": "%dx%d" % (L, F),
                      "device": str(dev), "arms": results}))


if __name__ == "__main__":
    main()
