"""Serving throughput and latency: many concurrent clients, one GPU, dynamic batching.

Each client thread sends single-position policy requests back to back (closed
loop).  Two paths are measured:

* ``engine``: pre-featurised planes through ``BatchingEvaluator`` over the
  HIP-graph policy engine.  This is the batching and engine cost alone.
* ``service``: ``GoService.policy_moves``, the HTTP handler's work minus the
  socket.  Each client plays through a game and sends the whole move list at
  every turn.  The service finds the position (prefix cache), encodes each
  round in one native call, runs the GPU featurizer and trunk in the engine's
  HIP graph, and renormalises over the legal moves.

Each path runs with ``max_batch=1`` (one evaluation per request, i.e. no
batching) and with the dynamic batch.

    python benchmarks/serving_benchmark.py --clients 64 --requests 4000
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from alphago_amd.serve import (BatchingEvaluator, GoService, engine_eval_fn, latency_summary,  # noqa: E402
                               position_from_moves, random_positions)


def closed_loop(n_clients, n_requests, fn):
    lat = [[] for _ in range(n_clients)]
    per = n_requests // n_clients

    def client(k):
        for i in range(per):
            t = time.perf_counter()
            fn(k, i)
            lat[k].append(time.perf_counter() - t)

    ts = [threading.Thread(target=client, args=(k,)) for k in range(n_clients)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    flat = [x for l in lat for x in l]
    p50, p99, mx = latency_summary(flat)
    return {"requests_per_s": round(len(flat) / dt, 1), "p50_ms": round(p50, 3), "p99_ms": round(p99, 3),
            "max_ms": round(mx, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--requests", type=int, default=4096)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-wait-ms", type=float, default=1.0)
    ap.add_argument("--filters", type=int, default=192)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--positions", type=int, default=512)
    a = ap.parse_args()

    from alphago_amd.features import DEFAULT_FEATURES
    from alphago_amd.models.policy import CNNPolicy

    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    torch.manual_seed(0)
    pol = CNNPolicy(DEFAULT_FEATURES, board=19, filters_per_layer=a.filters, layers=a.layers, device=dev)
    positions = random_positions(19, a.positions, max_moves=200, seed=0)
    planes = pol.preprocessor.states_to_uint8([position_from_moves(19, m) for m in positions])
    out = {"device": torch.cuda.get_device_name(0) if dev != "cpu" else "cpu",
           "model": "policy %d x %d, %d planes" % (a.layers, a.filters, planes.shape[1]),
           "clients": a.clients, "requests": a.requests, "max_wait_ms": a.max_wait_ms, "runs": {}}
    for mb in (1, a.max_batch):
        b = BatchingEvaluator(engine_eval_fn(pol.engine), max_batch=mb, max_wait_ms=a.max_wait_ms)
        for i in range(8):  # warm every graph bucket the run can hit
            b.evaluate(planes[:min(len(planes), 1 << i)])
        b0 = b.stats()
        r = closed_loop(a.clients, a.requests, lambda k, i: b.evaluate(planes[(k * 7919 + i) % len(planes)]))
        s = b.stats()
        r["mean_batch"] = round((s["boards"] - b0["boards"]) / max(1, s["rounds"] - b0["rounds"]), 1)
        b.close()
        out["runs"]["engine_max_batch_%d" % mb] = r
        # service: each client plays through its own game and asks for the policy at every
        # turn, sending the whole move list each time (a stateless HTTP client)
        svc = GoService(pol, None, max_batch=mb, max_wait_ms=a.max_wait_ms)
        svc.policy_moves(positions[0])
        games = [positions[(k * 7919) % len(positions)] for k in range(a.clients)]
        r = closed_loop(a.clients, a.requests // 2,
                        lambda k, i: svc.policy_moves(games[k][:i % (len(games[k]) + 1)], top_k=5))
        s = svc.stats()["policy"]
        r["mean_batch"] = round(s["mean_batch"], 1)
        r["cache_hits"] = svc.cache_hits
        svc.close()
        out["runs"]["service_max_batch_%d" % mb] = r
        print(json.dumps({"max_batch": mb, **out["runs"]["engine_max_batch_%d" % mb]}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
