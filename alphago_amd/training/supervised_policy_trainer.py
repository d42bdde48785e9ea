"""Reference module path ``AlphaGo.training.supervised_policy_trainer``.

``run_training`` (same CLI: model, train_data, out_directory, -B/-E/-l/-r/-d/
--weights/--train-val-test) is ``alphago_amd.train.sl.run_training``; it trains
on the HIP engine from a device-resident dataset with per-board D4
augmentation on the GPU.  The numpy helpers below keep the reference's
host-side generator API for code that feeds its own model:

* ``one_hot_action`` -- the true one-hot target (the reference fancy-indexes two
  whole rows);
* ``BOARD_TRANSFORMATIONS`` -- the 8 board symmetries in the reference's order
  (identity, rot90 x1..3, fliplr, flipud, transpose, fliplr(rot90));
* ``shuffled_hdf5_batch_generator`` -- yields FRESH arrays per batch (the
  reference reuses and mutates one buffer after ``yield``, a race with Keras'
  prefetch queue, Q17).
"""
import numpy as np

from ..train.sl import MetadataWriter, run_training

MetadataWriterCallback = MetadataWriter


def _symmetry(k: int):
    rot = k % 4 if k < 4 else 0

    def f(plane):
        if k < 4:
            return np.rot90(plane, rot)
        if k == 4:
            return plane[:, ::-1]
        if k == 5:
            return plane[::-1, :]
        if k == 6:
            return plane.T
        return np.rot90(plane, 1)[:, ::-1]

    return f


BOARD_TRANSFORMATIONS = [_symmetry(k) for k in range(8)]


def one_hot_action(action, size=19):
    """(x, y) -> size x size float array with a single 1 at [x][y]."""
    out = np.zeros((size, size))
    x, y = int(action[0]), int(action[1])
    out[x, y] = 1.0
    return out


def shuffled_hdf5_batch_generator(state_dataset, action_dataset, indices, batch_size, transforms=()):
    """Endless (X, Y) batches visiting ``indices`` in order, one random symmetry per sample."""
    transforms = list(transforms) or [BOARD_TRANSFORMATIONS[0]]
    size = state_dataset.shape[-1]
    rng = np.random.default_rng()
    X, Y, n = [], [], 0
    while True:
        for i in indices:
            f = transforms[rng.integers(len(transforms))]
            X.append(np.stack([f(p) for p in np.asarray(state_dataset[i])]))
            Y.append(f(one_hot_action(action_dataset[i], size)).reshape(-1))
            n += 1
            if n == batch_size:
                yield np.asarray(X, dtype=np.float64), np.asarray(Y, dtype=np.float64)
                X, Y, n = [], [], 0


__all__ = ["run_training", "MetadataWriterCallback", "BOARD_TRANSFORMATIONS", "one_hot_action",
           "shuffled_hdf5_batch_generator"]

if __name__ == "__main__":
    import sys

    from ..parallel.launch import exit_status
    sys.exit(exit_status(run_training()))
