"""Top-1 accuracy of the SL pipeline on a learnable synthetic task (no expert
games are available offline): positions from random games, labelled with the
greedy move of a fixed random-init "teacher" policy network (12 x 192, 48
planes), written to the training-HDF5 schema, then learned by a fresh student
network through the real SL trainer CLI (``train/sl.py run_training``).  The
student's held-out top-1 agreement with the teacher is the accuracy figure.

Usage: python scripts/sl_teacher_accuracy.py OUT_DIR [--positions N] [--epochs E] [--lr R] [--batch B]
Prints one JSON line with the per-epoch acc / val_acc from metadata.json."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alphago_amd import go  # noqa: E402
from alphago_amd._native import engine  # noqa: E402
from alphago_amd.features import DEFAULT_FEATURES  # noqa: E402
from alphago_amd.io.h5lite import H5Writer  # noqa: E402
from alphago_amd.models.policy import CNNPolicy  # noqa: E402
from alphago_amd.train.sl import run_training  # noqa: E402


def random_game_states(n_positions, rng):
    """Positions from random games (uniform over non-eye legal moves, 1 % passes)."""
    out = []
    while len(out) < n_positions:
        gs = go.GameState()
        for _ in range(int(rng.integers(20, 300))):
            moves = gs.get_legal_moves(include_eyes=False)
            if not moves or rng.random() < 0.01:
                gs.do_move(go.PASS_MOVE)
            else:
                gs.do_move(moves[int(rng.integers(len(moves)))])
            if gs.is_end_of_game:
                break
            out.append(gs.copy())
    return out[:n_positions]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--positions", type=int, default=131072)
    ap.add_argument("--epochs", type=int, default=8)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    small = dev.type == "cpu"
    F, L = (16, 3) if small else (192, 12)
    rng = np.random.default_rng(a.seed)
    t0 = time.perf_counter()
    torch.manual_seed(1000 + a.seed)
    teacher = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=F, layers=L, device=dev)
    h5 = os.path.join(a.out, "teacher.h5")
    n_done = 0
    with H5Writer(h5) as f:
        f.attrs["features"] = np.array([x.encode() for x in DEFAULT_FEATURES])
        f.attrs["board_size"] = np.int64(19)
        states_ds = f.stream_dataset("states", (teacher.preprocessor.output_dim, 19, 19), np.uint8)
        actions = []
        chunk = 8192
        while n_done < a.positions:
            sts = random_game_states(min(chunk, a.positions - n_done), rng)
            planes = teacher.preprocessor.states_to_uint8(sts)
            masks = engine().featurize_batch(sts, ["sensibleness"], 16).reshape(len(sts), -1)
            probs = []
            for i in range(0, len(sts), 1024):
                p = teacher.engine.evaluate(planes[i:i + 1024], masks[i:i + 1024]).float().cpu().numpy()
                probs.append(p.copy())
            probs = np.concatenate(probs) * (masks > 0)
            has = masks.sum(1) > 0
            idx = np.argmax(probs, axis=1)
            keep = np.nonzero(has)[0]  # positions with no sensible move (teacher would pass) are dropped
            states_ds.append(planes[keep])
            actions.append(np.stack([idx[keep] // 19, idx[keep] % 19], axis=1).astype(np.uint8))
            n_done += len(sts)
        states_ds.finish()
        acts = np.concatenate(actions)
        f.create_dataset("actions", data=acts)
        f.create_group("file_offsets")["synthetic"] = np.array([0, len(acts)], dtype=np.int64)
    t_data = time.perf_counter() - t0
    torch.manual_seed(2000 + a.seed)
    student = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=F, layers=L, device=dev)
    model_json = os.path.join(a.out, "student.json")
    student.save_model(model_json)
    run_dir = os.path.join(a.out, "run")
    t1 = time.perf_counter()
    run_training([model_json, h5, run_dir, "--minibatch", str(a.batch), "--epochs", str(a.epochs),
                  "--learning-rate", str(a.lr), "--decay", "0", "--no-symmetries", "--seed", str(a.seed)])
    t_train = time.perf_counter() - t1
    meta = json.load(open(os.path.join(run_dir, "metadata.json")))
    ep = meta["epochs"]
    print(json.dumps({"metric": "SL top-1 agreement with a random-init teacher policy (held-out)",
                      "positions": int(len(acts)), "epochs": len(ep), "minibatch": a.batch, "lr": a.lr,
                      "acc": [round(e.get("acc", 0), 4) for e in ep],
                      "val_acc": [round(e.get("val_acc", 0), 4) for e in ep],
                      "chance": round(1.0 / 300, 4), "data_s": round(t_data, 1), "train_s": round(t_train, 1),
                      "net": "%dx%d" % (L, F), "device": str(dev)}))


if __name__ == "__main__":
    main()
