"""Round-6 playing-strength and value-learning evidence on one MI355X.

Stages (each reads what the earlier ones wrote under OUT/nets, which is small enough to travel
back through gpurun_out/ between GPU calls):

  sl      teacher-labelled pool (random-game positions labelled by a fixed random-init 12x192
          teacher, data/synthetic.py) -> SL student 12x192 through the real SL CLI (train/sl.py)
          -> OUT/nets/sl.{json,hdf5}
  rl      train-rl (train/rl.py, REINFORCE, opponent pool) from the SL net; per-iteration win_rate
          JSONL -> OUT/rl_winrate.jsonl, final learner -> OUT/nets/rl.{json,hdf5}
  match   RL vs SL, both sampling their policy at T = 1 (ProbabilisticPolicyPlayer semantics),
          colours alternated, batched (search/arena.py batched_match) -> OUT/match_rl_vs_sl.json
  value   value-generate procedure (train/value.py generate_positions: SL to move U-1, a random
          move at U, RL to the end; one position per game) -> train-value CLI defaults in three arms
          (torch fp32, HIP bf16, HIP fp8) x seeds; held-out MSE vs var(z) -> OUT/value_selfplay.json,
          best HIP-bf16 net -> OUT/nets/value.{json,hdf5}
  search  batched MCTS (SL policy + value net, 1600 playouts, 32 leaves per tree) vs the greedy raw
          SL policy, colours alternated; per-move search times; single-tree genmove latency
          -> OUT/search_vs_policy.json

Reference: RL loop /root/reference/AlphaGo/training/reinforcement_policy_trainer.py:106-125 and its
opponent pool :164-175; value net /root/reference/AlphaGo/models/value.py:7-39; search
/root/reference/AlphaGo/mcts.py:142-161.

Usage: python scripts/r6/evidence.py STAGE OUT [options]
"""
import argparse
import json
import math
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def wilson(k, n, z=1.96):
    if n == 0:
        return (0.0, 0.0)
    p = k / n
    d = 1 + z * z / n
    c = (p + z * z / (2 * n)) / d
    h = z * math.sqrt(p * (1 - p) / n + z * z / (4 * n * n)) / d
    return (round(c - h, 4), round(c + h, 4))


def log(*a):
    print("[%s]" % time.strftime("%H:%M:%S"), *a, flush=True)


DEV = torch.device("cuda" if torch.cuda.is_available() else "cpu")
HIP = "hip" if DEV.type == "cuda" else "torch"
PNET = (192, 12)   # policy filters, layers (--small: a CPU rehearsal)
VNET = (152, 12)


def relativize(json_path, weights_name):
    """Point a saved model JSON at its weights file by a name relative to the JSON (the nets travel
    between GPU boxes through gpurun_out/)."""
    with open(json_path) as f:
        spec = json.load(f)
    spec["weights_file"] = weights_name
    with open(json_path, "w") as f:
        json.dump(spec, f)


def dump(path, obj):
    with open(path, "w") as f:
        json.dump(obj, f, indent=1)
    log("wrote", path)


def stage_sl(a):
    from alphago_amd.data.synthetic import teacher_pool
    from alphago_amd.features import DEFAULT_FEATURES
    from alphago_amd.io.h5lite import H5Writer
    from alphago_amd.models.policy import CNNPolicy
    from alphago_amd.train.sl import run_training
    dev = DEV
    work = a.work
    os.makedirs(work, exist_ok=True)
    h5 = os.path.join(work, "teacher.h5")
    t0 = time.perf_counter()
    torch.manual_seed(1000)
    teacher = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=PNET[0], layers=PNET[1], device=dev)
    planes, idx = teacher_pool(a.positions, teacher, seed=11, symmetrize=False)
    del teacher
    with H5Writer(h5) as f:
        f.attrs["features"] = np.array([x.encode() for x in DEFAULT_FEATURES])
        f.attrs["board_size"] = np.int64(19)
        ds = f.stream_dataset("states", (planes.shape[1], 19, 19), np.uint8)
        ds.append(planes)
        ds.finish()
        f.create_dataset("actions", data=np.stack([idx // 19, idx % 19], axis=1).astype(np.uint8))
        f.create_group("file_offsets")["synthetic"] = np.array([0, len(idx)], dtype=np.int64)
    log("teacher pool", len(idx), "positions in %.1f s" % (time.perf_counter() - t0))
    torch.manual_seed(2000)
    student = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=PNET[0], layers=PNET[1], device=dev)
    mj = os.path.join(work, "student.json")
    student.save_model(mj)
    run_dir = os.path.join(work, "sl_run")
    t1 = time.perf_counter()
    run_training([mj, h5, run_dir, "--minibatch", str(a.batch), "--epochs", str(a.epochs), "--learning-rate",
                  str(a.lr), "--decay", "0", "--no-symmetries", "--seed", "0", "--backend", HIP, "--verbose"])
    meta = json.load(open(os.path.join(run_dir, "metadata.json")))
    ep = meta["epochs"]
    last = sorted(f for f in os.listdir(run_dir) if f.startswith("weights.") and f.endswith(".hdf5"))[-1]
    nets = a.nets
    os.makedirs(nets, exist_ok=True)
    pol = CNNPolicy.load_model(mj, device=dev, weights_file=os.path.join(run_dir, last))
    pol.save_model(os.path.join(nets, "sl.json"), os.path.join(nets, "sl.hdf5"))
    relativize(os.path.join(nets, "sl.json"), "sl.hdf5")
    dump(os.path.join(a.out, "sl_teacher.json"),
         {"positions": len(idx), "epochs": a.epochs, "batch": a.batch, "lr": a.lr, "net": "12x192, 48 planes",
          "acc": [round(e.get("acc", 0), 4) for e in ep], "val_acc": [round(e.get("val_acc", 0), 4) for e in ep],
          "train_s": round(time.perf_counter() - t1, 1), "weights": last})


def _load_policy(a, name, dev):
    from alphago_amd.models.policy import CNNPolicy
    nets = a.nets
    return CNNPolicy.load_model(os.path.join(nets, name + ".json"), device=dev,
                                weights_file=os.path.join(nets, name + ".hdf5"))


def stage_rl(a):
    from alphago_amd.train.rl import run
    nets = a.nets
    folder = os.path.join(a.work, "rl_pool")
    shutil.rmtree(folder, ignore_errors=True)
    metrics = os.path.join(a.out, "rl_winrate%s.jsonl" % a.tag)
    if os.path.exists(metrics):
        os.remove(metrics)
    t0 = time.perf_counter()
    res = run([os.path.join(nets, "sl.hdf5"), os.path.join(nets, "sl.json"), "--model_folder", folder,
               "--learning_rate", str(a.lr), "--save_every", str(a.save_every), "--game_batch_size", str(a.games),
               "--iterations", str(a.iterations), "--minibatch", str(a.batch), "--backend", HIP,
               "--metrics", metrics, "--checkpoint-dir", os.path.join(a.work, "rl_ck"), "--checkpoint-every",
               str(a.iterations), "--seed", str(a.seed), "--verbose", "--baseline", a.baseline,
               "--clip-grad-norm", str(a.clip), "--weight-decay", str(a.wd), "--eval-every", str(a.eval_every),
               "--eval-games", "200"])
    last = res["best"]["path"] if a.eval_every > 0 and res["best"]["path"] else res["pool"][-1]
    assert last is not None
    shutil.copy(last, os.path.join(nets, "rl%s.hdf5" % a.tag))
    shutil.copy(os.path.join(nets, "sl.json"), os.path.join(nets, "rl%s.json" % a.tag))
    relativize(os.path.join(nets, "rl%s.json" % a.tag), "rl%s.hdf5" % a.tag)
    h = res["history"]
    dump(os.path.join(a.out, "rl_summary%s.json" % a.tag),
         {"iterations": a.iterations, "games_per_iteration": a.games, "lr": a.lr, "save_every": a.save_every,
          "baseline": a.baseline, "clip_grad_norm": a.clip, "weight_decay": a.wd, "eval_every": a.eval_every,
          "selected": ("best eval snapshot (iteration %d, eval win rate %.3f over 200 games vs SL)" %
                       (res["best"]["iteration"], res["best"]["eval_win_rate"])) if a.eval_every > 0 else "last",
          "eval_curve": [(r["iteration"] + 1, round(r["eval_win_rate"], 3)) for r in h if "eval_win_rate" in r],
          "skipped_updates": int(sum(1 for r in res["history"] if r.get("skipped"))),
          "opponent_pool": "the SL net only" if a.save_every >= a.iterations else
          "the SL net + a snapshot every %d iterations, one drawn uniformly per iteration" % a.save_every,
          "seconds": round(time.perf_counter() - t0, 1), "final_weights": os.path.basename(last),
          "win_rate_first10": round(float(np.mean([r["win_rate"] for r in h[:10]])), 4),
          "win_rate_last10": round(float(np.mean([r["win_rate"] for r in h[-10:]])), 4),
          "games_per_s_mean": round(float(np.mean([r["games_per_s"] for r in h])), 1)})


def stage_match(a):
    from alphago_amd.search.arena import batched_match
    from alphago_amd.search.selfplay import BatchedSampler
    dev = DEV
    sl, rl = _load_policy(a, "sl", dev), _load_policy(a, "rl" + a.tag, dev)
    out = {"rl_run": "rl_summary%s.json" % a.tag}
    for label, t in (("T1", 1.0),):
        t0 = time.perf_counter()
        res = batched_match(BatchedSampler(rl, t, seed=a.seed * 2 + 1), BatchedSampler(sl, t, seed=a.seed * 2 + 2),
                            a.games, seed=a.seed)
        k, n = res["player1_wins"], a.games
        res.update({"rl_win_rate": round(k / n, 4), "ci95": wilson(k, n), "seconds": round(time.perf_counter() - t0, 1),
                    "temperature": t})
        out[label] = res
        log(label, res)
    with open(os.path.join(a.out, "rl_summary%s.json" % a.tag)) as f:
        out["rl_opponent_pool"] = json.load(f).get("opponent_pool")
    out["note"] = ("RL = train-rl from the SL net (REINFORCE); both players sample their policy (p^(1/T)) over "
                   "sensible moves; colours alternate by game")
    dump(os.path.join(a.out, "match_rl%s_vs_sl.json" % a.tag), out)


def stage_value(a):
    from alphago_amd.features import VALUE_FEATURES
    from alphago_amd.io.h5lite import H5File, H5Writer
    from alphago_amd.models.policy import CNNValue
    from alphago_amd.train.value import STATE_CHUNK_ROWS, generate_positions, train_cli
    dev = DEV
    os.makedirs(a.work, exist_ok=True)
    data = os.path.join(a.work, "value_selfplay.h5")
    sl, rl = _load_policy(a, "sl", dev), _load_policy(a, "rl" + a.tag, dev)
    t0 = time.perf_counter()
    n = 0
    zs = []
    with H5Writer(data + ".tmp") as f:
        f.attrs["features"] = np.array([x.encode() for x in VALUE_FEATURES])
        st = None
        done = 0
        while done < a.positions:
            g = min(a.batch_games, a.positions - done)
            planes, z = generate_positions(sl, rl, g, size=19, max_u=450, seed=a.seed * 100003 + done)
            if st is None:
                st = f.stream_dataset("states", planes.shape[1:], np.uint8, chunk_rows=STATE_CHUNK_ROWS,
                                      compression="lzf")
            st.append(planes)
            zs.append(z)
            done += g
            n += len(z)
            log("value-generate: %d games -> %d positions, %.0f positions/s" % (done, n, n / (time.perf_counter() - t0)))
        st.finish()
        f.create_dataset("outcomes", data=np.concatenate(zs))
    os.replace(data + ".tmp", data)
    gen_s = time.perf_counter() - t0
    z = np.concatenate(zs).astype(np.float64)
    import hashlib
    with H5File(data) as f:  # identifies the dataset across GPU calls (generation is seeded)
        h = hashlib.sha1(np.asarray(f["outcomes"].read()).tobytes())
        st_ds = f["states"]
        for r0 in range(0, st_ds.shape[0], 8192):
            h.update(np.ascontiguousarray(st_ds.read_rows(r0, r0 + 8192)).tobytes())
    digest = h.hexdigest()[:16]
    log("dataset sha1", digest)
    torch.manual_seed(3)
    val = CNNValue(VALUE_FEATURES, filters_per_layer=VNET[0], layers=VNET[1], device="cpu")
    vj = os.path.join(a.work, "value_init.json")
    val.save_model(vj)
    arms = {"torch-fp32": ["--backend", "torch"], "hip-bf16": ["--backend", HIP],
            "hip-fp8": ["--backend", HIP, "--precision", "fp8"]}
    only = [x for x in a.arms.split(",") if x]
    results = {}
    for arm in only:
        for seed in range(a.seeds):
            od = os.path.join(a.work, "v_%s_%d" % (arm, seed))
            shutil.rmtree(od, ignore_errors=True)
            t1 = time.perf_counter()
            meta = train_cli([vj, data, od, "-B", str(a.batch), "-E", str(a.epochs), "--seed", str(seed),
                              "--train-val-test", "0.9", "0.1", "0.0", "--verbose"] + arms[arm])
            # the held-out rows of this seed's split: var(z) and the constant (train-mean) predictor
            perm = np.random.default_rng(seed).permutation(len(z))
            ntr = int(0.9 * len(z))
            ztr, zva = z[perm[:ntr]], z[perm[ntr:ntr + int(0.1 * len(z))]]
            var = float(zva.var())
            const = float(((zva - ztr.mean()) ** 2).mean())
            vl = [round(e["val_loss"], 4) for e in meta["epochs"]]
            tl = [round(e["loss"], 4) for e in meta["epochs"]]
            best = int(np.argmin(vl))
            results.setdefault(arm, []).append({"seed": seed, "val_mse": vl, "train_mse": tl, "best_epoch": best,
                                                "best_val_mse": vl[best], "var_z_heldout": round(var, 4),
                                                "const_mse_heldout": round(const, 4),
                                                "best_ratio_to_var": round(vl[best] / var, 4),
                                                "train_s": round(time.perf_counter() - t1, 1)})
            log(arm, seed, results[arm][-1])
            if arm == "hip-bf16" and seed == 0:
                nets = a.nets
                v = CNNValue.load_model(vj, device=dev, weights_file=os.path.join(od, "weights.%05d.hdf5" % best))
                v.save_model(os.path.join(nets, "value.json"), os.path.join(nets, "value.hdf5"))
                relativize(os.path.join(nets, "value.json"), "value.hdf5")
    summ = {arm: {"best_val_mse_mean": round(float(np.mean([r["best_val_mse"] for r in rs])), 4),
                  "ratio_to_var_mean": round(float(np.mean([r["best_ratio_to_var"] for r in rs])), 4)}
            for arm, rs in results.items()}
    if "torch-fp32" in summ:
        for arm in summ:
            summ[arm]["vs_fp32"] = round(summ[arm]["best_val_mse_mean"] / summ["torch-fp32"]["best_val_mse_mean"] - 1, 4)
    dump(os.path.join(a.out, "value_selfplay_%s.json" % "_".join(only)),
         {"positions": int(len(z)), "dataset_sha1_16": digest, "rl_net": "rl%s" % a.tag,
          "generate_s": round(gen_s, 1), "z_mean": round(float(z.mean()), 4),
          "z_var": round(float(z.var()), 4), "batch": a.batch, "epochs": a.epochs,
          "config": "train-value defaults (Adam 3e-4, Keras uniform init, decay 0), 12x152 value net, 49 planes; "
                    "90/10 split by position; self-play positions from value-generate (SL to U-1, random move at U, "
                    "RL to the end, one position per game)",
          "summary": summ, "arms": results})


def stage_search(a):
    from alphago_amd import go
    from alphago_amd.models.policy import CNNValue
    from alphago_amd.search.mcts import BatchedMCTS
    from alphago_amd.search.players import MCTSPlayer
    from alphago_amd.search.selfplay import BatchedSampler
    dev = DEV
    sl = _load_policy(a, "sl", dev)
    nets = a.nets
    val = CNNValue.load_model(os.path.join(nets, "value.json"), device=dev,
                              weights_file=os.path.join(nets, "value.hdf5"))
    # single-tree genmove latency on positions from greedy SL self-play
    player = MCTSPlayer(sl, val, n_playout=a.playouts, leaves_per_batch=a.leaves)
    greedy = BatchedSampler(sl, 0.0, greedy=True)
    st = go.GameState(19)
    lat = []
    for k in range(a.latency_moves):
        t0 = time.perf_counter()
        player.get_move(st)
        if DEV.type == "cuda":
            torch.cuda.synchronize()
        lat.append((time.perf_counter() - t0) * 1e3)
        mv = greedy.get_moves([st])[0] if k % 2 else player.get_move(st)
        st.do_move(mv)
        if st.is_end_of_game:
            st = go.GameState(19)
    lat = lat[2:]  # first calls build graphs
    search = BatchedMCTS(sl, val, n_trees=a.games, lmbda=0.0, seed=a.seed)
    states = [go.GameState(19) for _ in range(a.games)]
    m_black = [g % 2 == 0 for g in range(a.games)]
    # both players are deterministic (argmax of visits, argmax of the policy): every game pair (2p, 2p+1)
    # starts from its own random opening of --opening sensible moves, played identically in both games
    # of the pair (colours swapped between them)
    for g in range(0, a.games, 2):
        rng = np.random.default_rng(1000 + g)
        for _ in range(a.opening):
            legal = states[g].get_legal_moves(include_eyes=False)
            if not legal:
                break
            mv = legal[int(rng.integers(len(legal)))]
            for h in (g, g + 1):
                if h < a.games:
                    states[h].do_move(mv)
    rounds = []
    t0 = time.perf_counter()
    while True:
        live = [i for i in range(a.games) if not states[i].is_end_of_game and len(states[i].history) < 722]
        if not live:
            break
        # every round: one search over all games where MCTS is to move, then the greedy replies of every
        # game where the policy is to move -- after the first round all games search together
        mine = [i for i in live if (states[i].current_player == go.BLACK) == m_black[i]]
        if mine:
            t1 = time.perf_counter()
            mvs = search.search(states, a.playouts, a.leaves, temperature=0.0, active=mine)
            rounds.append({"trees": len(mine), "s": time.perf_counter() - t1})
            for i in mine:
                try:
                    states[i].do_move(mvs[i])
                except go.IllegalMove:
                    states[i].do_move(go.PASS_MOVE)
        theirs = [i for i in range(a.games) if not states[i].is_end_of_game and len(states[i].history) < 722
                  and (states[i].current_player == go.BLACK) != m_black[i]]
        if theirs:
            mvs2 = greedy.get_moves([states[i] for i in theirs])
            for k, i in enumerate(theirs):
                try:
                    states[i].do_move(mvs2[k])
                except go.IllegalMove:
                    states[i].do_move(go.PASS_MOVE)
        if len(rounds) % 10 == 0:
            log("search round %d: %d live, %.1f s" % (len(rounds), len(live), time.perf_counter() - t0))
    wins = draws = 0
    for g, s in enumerate(states):
        w = s.get_winner()
        draws += w == 0
        wins += w != 0 and (w == go.BLACK) == m_black[g]
    dump(os.path.join(a.out, "search_vs_policy.json"),
         {"games": a.games, "mcts_wins": int(wins), "policy_wins": int(a.games - wins - draws), "draws": int(draws),
          "mcts_win_rate": round(wins / a.games, 4), "ci95": wilson(wins, a.games),
          "playouts": a.playouts, "leaves_per_tree": a.leaves, "opponent": "greedy raw SL policy (argmax over sensible moves)",
          "opening": "%d random sensible moves per game pair, the same in both games of a pair (colours swapped)" % a.opening,
          "mean_length": float(np.mean([len(s.history) for s in states])), "seconds": round(time.perf_counter() - t0, 1),
          "batched_round_s_p50": round(float(np.median([r["s"] for r in rounds])), 3),
          "search_rounds": len(rounds), "leaf_evals_per_s": round(search.forest.total_evals /
                                                                   max(1e-9, sum(r["s"] for r in rounds)), 1),
          "genmove_single_tree_ms_p50": round(float(np.percentile(lat, 50)), 2),
          "genmove_single_tree_ms_p95": round(float(np.percentile(lat, 95)), 2), "genmove_samples": len(lat),
          "note": "MCTS = SL policy priors + value net (lambda 0, c_puct 5), argmax of visits; batched: one tree per "
                  "game, all MCTS-to-move games searched together each round"})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stage", choices=["sl", "rl", "match", "value", "search"])
    ap.add_argument("out")
    ap.add_argument("--work", default="/tmp/r6_work")
    ap.add_argument("--positions", type=int, default=262144)
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--games", type=int, default=512)
    ap.add_argument("--iterations", type=int, default=100)
    ap.add_argument("--save-every", type=int, default=10)
    ap.add_argument("--batch-games", type=int, default=4096)
    ap.add_argument("--arms", default="hip-bf16,hip-fp8,torch-fp32")
    ap.add_argument("--seeds", type=int, default=3)
    ap.add_argument("--playouts", type=int, default=1600)
    ap.add_argument("--leaves", type=int, default=32)
    ap.add_argument("--latency-moves", type=int, default=40)
    ap.add_argument("--opening", type=int, default=8, help="search: random opening moves per game pair")
    ap.add_argument("--baseline", default="mean", choices=["mean", "none"], help="rl: REINFORCE baseline")
    ap.add_argument("--clip", type=float, default=0.0, help="rl: gradient-norm clip (0: off)")
    ap.add_argument("--wd", type=float, default=0.0, help="rl: weight decay")
    ap.add_argument("--eval-every", type=int, default=0, help="rl: evaluate vs SL every N iterations, keep the best")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--small", action="store_true", help="tiny nets (CPU rehearsal of the pipeline)")
    ap.add_argument("--nets", default=None, help="where the nets are read / written (default OUT/nets)")
    ap.add_argument("--tag", default="", help="rl / match: suffix of the RL run's files (lr sweeps)")
    a = ap.parse_args()
    if a.small:
        global PNET, VNET
        PNET, VNET = (16, 2), (16, 2)
    os.makedirs(a.out, exist_ok=True)
    a.nets = a.nets or os.path.join(a.out, "nets")
    os.makedirs(a.nets, exist_ok=True)
    {"sl": stage_sl, "rl": stage_rl, "match": stage_match, "value": stage_value, "search": stage_search}[a.stage](a)


if __name__ == "__main__":
    main()
