"""Why alternate genmoves differ in time: per genmove, the number of leaf evaluations, the boards whose
GPU featurisation overflowed (host fallback), and host time split.  Usage: python scripts/r4/genmove_diag.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd.features import DEFAULT_FEATURES, VALUE_FEATURES  # noqa: E402
from alphago_amd.gtp.engine import GTPEngine  # noqa: E402
from alphago_amd.models.policy import CNNPolicy, CNNValue  # noqa: E402
from alphago_amd.search import mcts as M  # noqa: E402
from alphago_amd.search.players import MCTSPlayer  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    pol = CNNPolicy(DEFAULT_FEATURES, filters_per_layer=192, layers=12, device=dev)
    val = CNNValue(VALUE_FEATURES, filters_per_layer=152, layers=12, device=dev)
    st = {"evals": 0, "leaves": 0, "bad": 0, "t_submit": 0.0, "t_finish": 0.0, "t_gather": 0.0}
    o_sub, o_fin = M.BatchedMCTS._submit, M.BatchedMCTS._finish

    def sub(self, f, slot, pe, ve):
        t = time.perf_counter()
        st["evals"] += 1
        st["leaves"] += f.n_pending
        r = o_sub(self, f, slot, pe, ve)
        st["t_submit"] += time.perf_counter() - t
        return r

    def fin(self, f, handles, pe, ve):
        t = time.perf_counter()
        hp, hv = handles
        _, _, bad = pe.collect(hp)
        st["bad"] += len(bad)
        r = o_fin(self, f, handles, pe, ve)
        st["t_finish"] += time.perf_counter() - t
        return r

    M.BatchedMCTS._submit, M.BatchedMCTS._finish = sub, fin
    st["t_engine"] = 0.0
    for eng_obj in (pol.engine, val.engine):
        o = eng_obj.submit_encoded

        def timed(*args, _o=o, **kw):
            t = time.perf_counter()
            r = _o(*args, **kw)
            st["t_engine"] += time.perf_counter() - t
            return r
        eng_obj.submit_encoded = timed
    player = MCTSPlayer(pol, val, n_playout=1600, leaves_per_batch=32)
    eng = GTPEngine(player)
    for c in ("boardsize 19", "clear_board", "genmove b", "clear_board"):
        eng.send(c)
    color = "b"
    for _ in range(int(os.environ.get("DIAG_MOVES", "6"))):
        for k in st:
            st[k] = 0 if isinstance(st[k], int) else 0.0
        t0 = time.perf_counter()
        reply = eng.send("genmove " + color)
        torch.cuda.synchronize()
        ms = 1000 * (time.perf_counter() - t0)
        print(json.dumps({"color": color, "reply": reply.strip(), "ms": round(ms, 1), "evals": st["evals"],
                          "leaves": st["leaves"], "overflow_boards": st["bad"],
                          "submit_ms": round(1000 * st["t_submit"], 1),
                          "engine_submit_ms": round(1000 * st["t_engine"], 1), "finish_ms": round(1000 * st["t_finish"], 1)}),
              flush=True)
        color = "w" if color == "b" else "b"


if __name__ == "__main__":
    main()
