"""Training throughput with the data path in the loop: device-resident shard vs
host-streamed shard (pinned ring + prefetch thread + copy stream), from a
contiguous and from an LZF-chunked HDF5 file (the reference's layout,
game_converter.py:71-86).

Writes two synthetic files of --rows positions (feature-plane-like sparse
uint8 planes) to --dir, then times --steps SL steps of the 12x192 policy net at
--batch boards per step in each mode.  One JSON line per mode.

    python benchmarks/data_streaming_benchmark.py --rows 32768 --batch 2176
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from alphago_amd.data.dataset import PositionDataset, block_shuffle  # noqa: E402
from alphago_amd.io.h5lite import H5Writer  # noqa: E402
from alphago_amd.models.nets import PolicyNet  # noqa: E402
from alphago_amd.train.engine import make_policy_trainer  # noqa: E402


def synth_planes(rng, n, planes=48, size=19):
    """Feature-plane-like rows: a random board (3 one-hot planes), a ones plane,
    sparse one-hot families, zeros elsewhere (compresses like real data)."""
    b = rng.integers(0, 3, (n, size, size))
    x = np.zeros((n, planes, size, size), np.uint8)
    for c in range(3):
        x[:, c] = b == c
    x[:, 3] = 1
    for fam in range(4, planes - 1, 8):
        k = rng.integers(0, 8, (n, size, size))
        occ = rng.random((n, size, size)) < 0.3
        for j in range(min(8, planes - 1 - fam)):
            x[:, fam + j] = occ & (k == j)
    return x


def write(path, x, t, chunked):
    with H5Writer(path) as f:
        acts = np.stack([t // 19, t % 19], 1).astype(np.uint8)
        if chunked:
            s = f.stream_dataset("states", x.shape[1:], np.uint8, chunk_rows=64, compression="lzf")
            for i in range(0, len(x), 4096):
                s.append(x[i:i + 4096])
            s.finish()
            f.create_chunked("actions", acts, 1024, "lzf")
        else:
            f["states"] = x
            f["actions"] = acts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32768)
    ap.add_argument("--batch", type=int, default=2176)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dir", default="/tmp/agdata")
    ap.add_argument("--modes", default="resident,stream-contiguous,stream-lzf")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    os.makedirs(args.dir, exist_ok=True)
    rng = np.random.default_rng(0)
    x = synth_planes(rng, args.rows)
    t = rng.integers(0, 361, args.rows)
    pc, pz = os.path.join(args.dir, "contig.h5"), os.path.join(args.dir, "lzf.h5")
    t0 = time.perf_counter()
    write(pc, x, t, False)
    write(pz, x, t, True)
    print(json.dumps({"write_s": round(time.perf_counter() - t0, 2), "raw_bytes": int(x.nbytes),
                      "lzf_bytes": os.path.getsize(pz)}), flush=True)
    del x
    torch.manual_seed(0)
    net = PolicyNet(48, filters_per_layer=192, layers=12)
    trainer = make_policy_trainer(net, args.batch, 0.003, 0.0, backend="hip", device=dev)
    B = args.batch
    total = args.warmup + args.steps
    for mode in args.modes.split(","):
        path = pz if mode == "stream-lzf" else pc
        rows = rng.permutation(args.rows)
        resident = "yes" if mode == "resident" else "no"
        if mode == "stream-lzf":
            rows = block_shuffle(rows, 64, seed=1)
        t_open = time.perf_counter()
        ds = PositionDataset(path, dev, resident=resident, rows=rows)
        open_s = time.perf_counter() - t_open
        batches = (np.arange(k * B, (k + 1) * B) % len(rows) for k in range(total))
        it = ds.prefetch(batches, B) if resident == "no" else (ds.batch(b) for b in batches)
        g = torch.Generator(device=dev)
        g.manual_seed(5)
        for k in range(total):
            if k == args.warmup:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            planes, tgt = next(it)
            sym = torch.randint(0, 8, (B,), device=dev, dtype=torch.int32, generator=g)
            trainer.step(planes, tgt, sym)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if resident == "no":
            it.close()
        ds.close()
        print(json.dumps({"mode": mode, "positions_per_s": round(args.steps * B / dt, 1),
                          "ms_per_step": round(dt / args.steps * 1e3, 3), "open_s": round(open_s, 2),
                          "batch": B, "rows": args.rows}), flush=True)


if __name__ == "__main__":
    main()
