"""SGF -> HDF5 training-data converter (reference game_converter.py:16-214).

Same output schema and storage layout as the reference so
existing datasets and tools interoperate:
  states       uint8 (N, F, S, S) one-hot planes, chunks (64, F, S, S), LZF
  actions      uint8 (N, 2)        move (x, y),     chunks (1024, 2),    LZF
  file_offsets group: key = path with '/' -> ':', value = [start, n_pairs]
plus a ``features`` attribute listing the planes (the reference's TODO,
game_converter.py:62).  Featurisation runs in native threads; state rows are
streamed straight into the file one compressed chunk at a time (no 1-row
resizes, constant memory), written to a hidden temp file and atomically renamed
on success.  ``compression=None`` writes contiguous datasets
(memory-mappable, for host-streamed training without a decode step).
"""
from __future__ import annotations

import argparse
import os
import sys
import warnings
from typing import Iterable, List, Optional

import numpy as np

from .. import go
from ..features import ALL_NO_LADDER_FEATURES, Preprocess
from ..io import sgf as sgflib
from ..io.h5lite import H5Writer
from ..utils.gorecords import sgf_iter_states


class SizeMismatchError(Exception):
    pass


class GameConverter(object):
    STATE_CHUNK_ROWS = 64     # game_converter.py:71-78
    ACTION_CHUNK_ROWS = 1024  # game_converter.py:79-86

    def __init__(self, features: List[str], threads: int = 8, compression: Optional[str] = "lzf"):
        self.feature_processor = Preprocess(features)
        self.n_features = self.feature_processor.output_dim
        self.features = list(features)
        self.threads = threads
        self.compression = compression

    def convert_game(self, file_name: str, bd_size: int):
        """Yield (planes (1,F,S,S) uint8, move) for every non-pass move."""
        states, moves = self._game_states(file_name, bd_size)
        if not states:
            return
        planes = self.feature_processor.states_to_uint8(states, self.threads)
        for i, mv in enumerate(moves):
            yield planes[i:i + 1], mv

    def _game_states(self, file_name: str, bd_size: int):
        with open(file_name, "r", errors="replace") as fo:
            text = fo.read()
        states, moves = [], []
        err = None
        try:
            for state, move, player in sgf_iter_states(text):
                if state.size != bd_size:
                    raise SizeMismatchError()
                if move is not go.PASS_MOVE:
                    states.append(state.copy())
                    moves.append(move)
        except go.IllegalMove as e:  # keep the prefix, like the reference
            err = e
        if err is not None:
            self._pending_error = err
        return states, moves

    def game_arrays(self, file_name: str, bd_size: int):
        self._pending_error = None
        states, moves = self._game_states(file_name, bd_size)
        planes = self.feature_processor.states_to_uint8(states, self.threads) if states else \
            np.zeros((0, self.n_features, bd_size, bd_size), np.uint8)
        acts = np.array(moves, dtype=np.uint8).reshape(-1, 2)
        return planes, acts, self._pending_error

    def sgfs_to_hdf5(self, sgf_files: Iterable[str], hdf5_file: str, bd_size: int = 19, ignore_errors: bool = True,
                     verbose: bool = False) -> int:
        tmp_file = os.path.join(os.path.dirname(hdf5_file), ".tmp." + os.path.basename(hdf5_file))
        total = 0
        try:
            with H5Writer(tmp_file) as h5f:
                h5f.attrs["features"] = np.array([f.encode() for f in self.features])
                h5f.attrs["board_size"] = np.int64(bd_size)
                chunked = self.compression is not None
                states = h5f.stream_dataset("states", (self.n_features, bd_size, bd_size), np.uint8,
                                            chunk_rows=self.STATE_CHUNK_ROWS if chunked else 0,
                                            compression=self.compression)
                offsets = h5f.create_group("file_offsets")
                all_actions = []
                for file_name in sgf_files:
                    if verbose:
                        print(file_name)
                    start = total
                    n = 0
                    try:
                        planes, acts, err = self.game_arrays(file_name, bd_size)
                        if len(acts):
                            states.append(planes)
                            all_actions.append(acts)
                            n = len(acts)
                            total += n
                        if err is not None:
                            warnings.warn("Illegal Move encountered in %s\n\tdropping the remainder of the game"
                                          % file_name)
                    except sgflib.SGFParseError:
                        warnings.warn("Could not parse %s\n\tdropping game" % file_name)
                    except SizeMismatchError:
                        warnings.warn("Skipping %s; wrong board size" % file_name)
                    except Exception as e:  # noqa: BLE001 - same policy as the reference
                        if ignore_errors:
                            warnings.warn("Unknown exception with file %s\n\t%s" % (file_name, e))
                        else:
                            raise
                    if n > 0:
                        offsets[file_name.replace("/", ":")] = np.array([start, n], dtype=np.int64)
                        if verbose:
                            print("\t%d state/action pairs extracted" % n)
                    elif verbose:
                        print("\t-no usable data-")
                states.finish()
                acts = np.concatenate(all_actions) if all_actions else np.zeros((0, 2), np.uint8)
                if chunked:
                    h5f.create_chunked("actions", acts, self.ACTION_CHUNK_ROWS, self.compression)
                else:
                    h5f.create_dataset("actions", data=acts)
        except Exception:
            if os.path.exists(tmp_file):
                os.remove(tmp_file)
            raise
        os.replace(tmp_file, hdf5_file)
        return total


# reference name
game_converter = GameConverter


def _is_sgf(fname: str) -> bool:
    return fname.strip()[-4:] == ".sgf"


def _walk_all_sgfs(root: str):
    for dirpath, _, files in os.walk(root):
        for filename in sorted(files):
            if _is_sgf(filename):
                yield os.path.join(dirpath, filename)


def _list_sgfs(path: str):
    return (os.path.join(path, f) for f in sorted(os.listdir(path)) if _is_sgf(f))


def run_game_converter(cmd_line_args: Optional[List[str]] = None) -> int:
    parser = argparse.ArgumentParser(
        description="Prepare SGF Go game files for training the neural network model.",
        epilog="Available features are: board, ones, turns_since, liberties, capture_size, self_atari_size, "
               "liberties_after, ladder_capture, ladder_escape, sensibleness, zeros, color")
    parser.add_argument("--features", "-f", help="Comma-separated list of features to compute and store or 'all'",
                        default="all")
    parser.add_argument("--outfile", "-o", help="Destination to write data (hdf5 file)", required=True)
    parser.add_argument("--recurse", "-R", help="Set to recurse through directories searching for SGF files",
                        default=False, action="store_true")
    parser.add_argument("--directory", "-d", help="Directory containing SGF files to process. if not present, "
                        "expects files from stdin", default=None)
    parser.add_argument("--size", "-s", help="Size of the game board. SGFs not matching this are discarded with a "
                        "warning", type=int, default=19)
    parser.add_argument("--threads", type=int, default=8, help="featurizer threads")
    parser.add_argument("--compression", default="lzf", choices=["lzf", "none"],
                        help="lzf: chunked (64,F,S,S) LZF datasets as the reference writes; none: contiguous")
    parser.add_argument("--verbose", "-v", help="Turn on verbose mode", default=False, action="store_true")
    args = parser.parse_args(cmd_line_args)
    if args.features.lower() == "all":
        feature_list = list(ALL_NO_LADDER_FEATURES)
    else:
        feature_list = args.features.split(",")
    if args.verbose:
        print("using features", feature_list)
    converter = GameConverter(feature_list, threads=args.threads,
                              compression=None if args.compression == "none" else "lzf")
    if args.directory:
        files = _walk_all_sgfs(args.directory) if args.recurse else _list_sgfs(args.directory)
    else:
        files = (f.strip() for f in sys.stdin if _is_sgf(f))
    return converter.sgfs_to_hdf5(files, args.outfile, bd_size=args.size, verbose=args.verbose)


if __name__ == "__main__":
    run_game_converter()
