#!/usr/bin/env python
"""Headline benchmark: SL policy-network training throughput.

Metric (BASELINE.json): SL-policy positions/sec for the whole node (+ top-1
move accuracy) on the 19x19, 12-layer, 192-filter, 48-plane policy network
(reference CNNPolicy architecture, policy.py:93-156; paper size), bf16 compute
with fp32 master weights, SGD with Keras decay, per-board random D4
augmentation, on synthetic positions and random-init weights (no datasets or
checkpoints are reachable offline).

Single GPU:   python bench.py --steps 20 --warmup 5
N GPUs:       python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
                  --master-addr 127.0.0.1 --master-port P bench.py --gpus N
          or    python bench.py --gpus N   (starts the N ranks itself, parallel/launch.py)
Weak scaling: the per-GPU batch is fixed; the global batch is N x per-GPU batch.
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

PAPER_SL_POS_PER_S = 3000.0  # paper SL throughput, 50 GPUs aggregate (derived)


def teacher_pool_on_device(args, dev, rank):
    import torch
    """Teacher-labelled pool (alphago_amd/data/synthetic.py): the same fixed teacher on every rank,
    a different position stream per rank; the teacher is freed before the student trains."""
    from alphago_amd.data.synthetic import teacher_pool
    from alphago_amd.features import DEFAULT_FEATURES
    from alphago_amd.models.policy import CNNPolicy
    cpu_rng = torch.get_rng_state()
    torch.manual_seed(4242)  # one teacher for all ranks
    teacher = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=args.filters, layers=args.layers, device=dev)
    torch.set_rng_state(cpu_rng)
    planes, tgt = teacher_pool(args.pool, teacher, seed=7000 + rank)
    del teacher
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    return torch.from_numpy(planes).to(dev), torch.from_numpy(tgt).to(dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=25)
    # Warmup runs at least --warmup steps AND at least this many seconds of sustained load (chunks
    # of 10 steps, the decision all-reduced so every rank runs the same number of steps).
    ap.add_argument("--min-warmup-s", type=float, default=3.0)
    # 2176 boards x 361 points = 2046 forward tiles of 384 pixels: eight full rounds over the 256 CUs.
    # Alternating A/B on one box (3 rounds each, profiles/r1_batch_sweep_v8.md): 1088 -> 110.5-111.4k,
    # 2176 -> 117.2-117.9k (+6 %: the per-step serial tail, head, wgrad reduce and SGD amortise over
    # twice the boards), 3264 -> 119.9-120.1k, 4352 -> 120.0k (flat).
    ap.add_argument("--batch", type=int, default=2176, help="per-GPU minibatch (boards)")
    ap.add_argument("--filters", type=int, default=192)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--planes", type=int, default=48)
    ap.add_argument("--lr", type=float, default=0.03, help="reference SL default (-r 0.03, supervised_policy_trainer.py)")
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--pool", type=int, default=65536, help="synthetic positions resident on device")
    ap.add_argument("--data", default="teacher", choices=["teacher", "random"],
                    help="teacher: random-game positions labelled by a fixed random-init teacher of the same "
                         "architecture (learnable: top1_acc measures learning); random: random planes/labels")
    ap.add_argument("--overlap", action="store_true",
                    help="run the wgrad on a second stream beside the dgrad at any batch (default: automatic, on for "
                         "B = 8 .. 256 where it wins, serial outside -- slower at the bench batch)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp8"],
                    help="conv forward precision (fp8 = e4m3 block-scaled MFMA forward, bf16 backward)")
    ap.add_argument("--graph", action="store_true", help="run each training step as a HIP-graph replay")
    ap.add_argument("--conv-tile", type=int, default=0, choices=[0, 36, 37, 64, 65, 128, 130, 256, 384, 385, 386, 387],
                    help="forward/dgrad conv tiling (0 = automatic)")
    ap.add_argument("--wgrad-wgs", type=int, default=0,
                    help="target workgroups per wgrad launch (sets the split-K factor; 0 = one resident round)")
    ap.add_argument("--reduce-stream", type=int, default=None, choices=[0, 1],
                    help="1: split-K wgrad reduce on a side stream beside the dgrad (default: engine default)")
    ap.add_argument("--wgrad-direct", type=int, default=None, choices=[0, 1],
                    help="1: split-free wgrad (no split-K slab / reduce) on every layer; 0: never (default: engine "
                         "default, automatic at small batches)")
    ap.add_argument("--wgrad-ksub", type=int, default=4, choices=[1, 2, 4, 8],
                    help="split-free wgrad: 32-pixel sub-steps per pipeline stage")
    ap.add_argument("--merged-reduce", type=int, default=None, choices=[0, 1],
                    help="1: one split-K reduce launch for all layers after the backward (one process); 0: one "
                         "per layer (default: engine default)")
    ap.add_argument("--profile", default=None,
                    help="after the timed run, profile 6 more steps (torch.profiler + roctx ranges) into DIR")
    args = ap.parse_args()

    # `python bench.py --gpus N` without torchrun: this process only supervises N ranks started by
    # torch.distributed.run (it never touches the GPU); a torchrun world that differs from --gpus, or
    # fewer visible GPUs than --gpus, is refused (alphago_amd/parallel/launch.py).
    from alphago_amd.parallel.launch import ensure_ranks
    code = ensure_ranks(args.gpus, [os.path.abspath(__file__)], sys.argv[1:], require_gpu=args.backend == "hip")
    if code is not None:
        return code

    import torch
    from alphago_amd.models.nets import PolicyNet
    from alphago_amd.parallel import dist as agdist
    from alphago_amd.train.engine import make_policy_trainer

    env = agdist.init_from_env()
    if env.world_size != args.gpus:  # belt and braces: the JSON line must describe the world that ran
        raise SystemExit("bench.py: --gpus %d but the process group has %d ranks" % (args.gpus, env.world_size))
    dev = env.device
    torch.manual_seed(1234 + env.rank)
    net = PolicyNet(args.planes, board=19, filters_per_layer=args.filters, layers=args.layers)
    kw = {} if args.backend == "torch" else {"overlap": True if args.overlap else None, "precision": args.precision,
                                             "wgrad_target_wgs": args.wgrad_wgs, "conv_tile": args.conv_tile,
                                             "reduce_stream": None if args.reduce_stream is None
                                             else bool(args.reduce_stream),
                                             "wgrad_direct": None if args.wgrad_direct is None
                                             else bool(args.wgrad_direct), "wgrad_ksub": args.wgrad_ksub,
                                             "merged_reduce": None if args.merged_reduce is None
                                             else bool(args.merged_reduce)}
    trainer = make_policy_trainer(net, args.batch, args.lr, 0.0, backend=args.backend, device=dev, **kw)
    if args.graph:
        trainer.enable_graphs()

    # synthetic dataset, resident in HBM (uint8 one-hot planes + move targets), built before the clock
    g = torch.Generator(device=dev)
    g.manual_seed(99 + env.rank)
    t_pool = time.perf_counter()
    if args.data == "teacher" and args.planes == 48:
        pool, pool_tgt = teacher_pool_on_device(args, dev, env.rank)
        data_desc = ("synthetic: %d random-game positions per rank (48 native-featurized planes) labelled by a "
                     "fixed random-init %dx%d teacher (D4-averaged argmax); random-init student" %
                     (args.pool, args.layers, args.filters))
    else:
        pool = torch.randint(0, 2, (args.pool, args.planes, 19, 19), device=dev, dtype=torch.uint8, generator=g)
        pool_tgt = torch.randint(0, 361, (args.pool,), device=dev, dtype=torch.int32, generator=g)
        data_desc = "synthetic (random uint8 planes/targets, random-init weights)"
    pool_s = time.perf_counter() - t_pool

    def batch():
        """(step args, step kwargs) of one random minibatch of the resident pool.  Eager steps pass the
        pool and the drawn rows: the input-pack kernel gathers the boards itself (no index_select
        pass over the planes).  Graph replays take the gathered minibatch (static input buffers)."""
        idx = torch.randint(0, args.pool, (args.batch,), device=dev, generator=g)
        sym = torch.randint(0, 8, (args.batch,), device=dev, dtype=torch.int32, generator=g)
        if args.graph:
            return (pool.index_select(0, idx), pool_tgt.index_select(0, idx), sym), {}
        return (pool, pool_tgt.index_select(0, idx), sym), {"rows": idx}

    loss_sum = torch.zeros((), device=dev)
    corr_sum = torch.zeros((), device=dev)

    def run(n):
        # The warmup runs this exact loop body too: every kernel of the timed region (including the
        # metric accumulation) is loaded before the clock starts.  On a fresh box the first launch of
        # a not-yet-used kernel from libtorch's code objects cost ~52 ms of host time (cold page
        # cache), which landed inside the timed region of the round-1 driver run: 20 x 18.4 ms of
        # GPU work measured as 21.1 ms/step (profiles/r2_fresh_box_diagnosis.md).
        for _ in range(n):
            bargs, bkw = batch()
            l, c = trainer.step(*bargs, **bkw)
            loss_sum.add_(l)
            corr_sum.add_(c)

    t_warm = time.perf_counter()
    warm_steps = 0
    run(args.warmup)
    warm_steps += args.warmup
    while True:
        if dev.type == "cuda":
            torch.cuda.synchronize()
        warm_s = agdist.all_reduce_max(time.perf_counter() - t_warm)  # the slowest rank's warmup time
        if warm_s >= args.min_warmup_s:
            break
        run(10)
        warm_steps += 10
    loss_sum.zero_()
    corr_sum.zero_()
    if hasattr(trainer, "comm_events") and (env.distributed or getattr(trainer, "_proxy", None) is not None):
        trainer.comm_events = []  # (start, end) events around the backward's all-reduce wait, per step
    if dev.type == "cuda":
        torch.cuda.synchronize()
    agdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    t_host = time.perf_counter() - t0  # host enqueue time: ~dt means the host, not the GPU, sets the pace
    if dev.type == "cuda":
        torch.cuda.synchronize()
    agdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt_rank = time.perf_counter() - t0
    rank_ms = [round(float(v) / args.steps * 1e3, 3) for v in agdist.all_gather_object(dt_rank)]
    dt = agdist.all_reduce_max(dt_rank)
    comm = None
    ev = getattr(trainer, "comm_events", None)
    if ev:  # exposed all-reduce per step, max over ranks
        comm = agdist.all_reduce_max(sum(a.elapsed_time(b) for a, b in ev) / len(ev))
    # per-rank device memory (the PyTorch caching allocator's peak reservation: weights, optimizer state,
    # activations, teacher pool, graph pools; RCCL's own buffers are outside it), max over ranks
    hbm_gib = agdist.all_reduce_max(torch.cuda.max_memory_reserved(dev) / 2 ** 30) if dev.type == "cuda" else 0.0
    n = env.world_size
    stats = torch.stack([loss_sum, corr_sum]).double()
    agdist.all_reduce_sum_(stats)
    positions = args.batch * n * args.steps
    value = positions / dt
    if env.is_main:
        out = {
            "metric": "SL-policy positions/sec (whole node) + top-1 move acc, 19x19 12-layer net",
            "value": round(value, 1),
            "unit": "positions/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": warm_steps,
            "warmup_s": round(warm_s, 2),
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "host_ms_per_step": round(t_host / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / PAPER_SL_POS_PER_S, 2),
            "dtype": (args.precision if args.precision == "bf16" else "fp8-fwd/bf16-bwd") if args.backend == "hip"
            else "fp32",
            "data": data_desc,
            "top1_acc": round(float(stats[1]) / positions, 4),
            "mean_loss": round(float(stats[0]) / positions, 4),
            "tflops": round(net.flops_per_position() * 3 * value / 1e12, 1),
            "dist_backend": agdist.live_backend(),
            "world_size": agdist.live_world_size(),
            "rank_ms_per_step": rank_ms,
            "allreduce_exposed_ms_per_step": None if comm is None else round(comm, 3),
            "pool_build_s": round(pool_s, 1),
            "hbm_peak_gib_per_rank": round(hbm_gib, 2),
            "config": {
                "model": "SL policy net (%d-layer, %d filters, %d planes)" % (args.layers, args.filters, args.planes),
                "global_batch": args.batch * n,
                "per_gpu_batch": args.batch,
                "seq_len": 361,
                "parallelism": "dp%d" % n,
                "backend": args.backend,
                "graph": bool(args.graph),
                "wgrad_direct": None if args.backend != "hip" else any(getattr(trainer, "wgrad_direct", [])),
                "merged_reduce": None if args.backend != "hip" else bool(getattr(trainer, "merged_reduce", False)),
                "baseline": "paper SL throughput ~3.0k pos/s (50 GPUs), BASELINE.md (A)",
            },
        }
        print(json.dumps(out), flush=True)
    if args.profile:  # outside the timed region
        from alphago_amd.utils.profiling import Profiler
        with Profiler(os.path.join(args.profile, "rank%d" % env.rank), wait=1, warmup=2, active=3) as prof:
            for _ in range(6):
                bargs, bkw = batch()
                trainer.step(*bargs, **bkw)
                prof.step()
        if dev.type == "cuda":
            torch.cuda.synchronize()
    agdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
