"""SL training on the reference fixture dataset (the reference's version of this
benchmark was broken: benchmarks/supervised_policy_training_benchmark.py passed 6
positional args to run_training).  Runs a few epochs of the real CLI on the
1033-position fixture with the reference minimodel architecture and reports
positions/s from the metrics log.  Prints JSON."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alphago_amd.models.policy import CNNPolicy  # noqa: E402
from alphago_amd.train.sl import run_training  # noqa: E402

FIXTURE = "/root/reference/tests/test_data/hdf5/alphago-vs-lee-sedol-features.hdf5"


def main():
    backend = sys.argv[1] if len(sys.argv) > 1 else ("hip" if torch.cuda.is_available() else "torch")
    with tempfile.TemporaryDirectory() as d:
        data = FIXTURE
        if not os.path.exists(data):  # no reference checkout: same schema, synthetic content
            import numpy as np
            from alphago_amd.io.h5lite import H5Writer
            data = os.path.join(d, "synthetic.h5")
            rng = np.random.default_rng(0)
            with H5Writer(data) as f:
                f["states"] = rng.integers(0, 2, (1033, 12, 19, 19), dtype=np.uint8)
                f["actions"] = rng.integers(0, 19, (1033, 2), dtype=np.uint8)
        pol = CNNPolicy(["board", "ones", "turns_since"], filters_per_layer=192, layers=12, device="cpu")
        j = os.path.join(d, "model.json")
        pol.save_model(j)
        metrics = os.path.join(d, "m.jsonl")
        meta = run_training([j, data, os.path.join(d, "out"), "-E", "3", "-B", "64", "-r", "0.003",
                             "--backend", backend, "--metrics", metrics])
        rows = [json.loads(l) for l in open(metrics)]
        print(json.dumps({"backend": backend, "epochs": meta["epochs"],
                          "positions_per_s_last_epoch": rows[-1]["positions_per_s"]}))


if __name__ == "__main__":
    main()
