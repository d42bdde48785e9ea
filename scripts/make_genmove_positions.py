"""Write benchmarks/data/lee_sedol_positions.json: the move sequences (our own SGF reader,
utils/gorecords.py) of positions from the four Lee Sedol - AlphaGo game records in the reference's test
data (tests/test_data/sgf/*Lee-Sedol*), every 20th move from move 20 ([x, y, colour] per move, [-1, -1, c] = pass).  The genmove latency benchmark
replays them (the GPU box has no copy of the reference tree)."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from alphago_amd.utils.gorecords import sgf_iter_states  # noqa: E402

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/tests/test_data/sgf"
out = []
for path in sorted(glob.glob(os.path.join(src, "*Lee-Sedol*.sgf"))):
    moves = []
    for state, move, player in sgf_iter_states(open(path).read()):
        moves.append([-1, -1, int(player)] if move is None else [int(move[0]), int(move[1]), int(player)])
    for k in range(20, len(moves), 20):
        out.append({"game": os.path.basename(path), "move_number": k, "moves": moves[:k]})
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks", "data",
                   "lee_sedol_positions.json")
json.dump({"size": 19, "positions": out}, open(dst, "w"))
print(len(out), "positions ->", dst)
