"""cProfile of the single-tree genmove benchmark (host side): top functions by cumulative and by own
time.  Usage: python scripts/r4/genmove_profile.py OUT.txt [--leaves 32]"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "benchmarks"))

out = sys.argv[1]
sys.argv = ["genmove_benchmark.py"] + sys.argv[2:]
import genmove_benchmark  # noqa: E402

pr = cProfile.Profile()
pr.enable()
genmove_benchmark.main()
pr.disable()
s = io.StringIO()
ps = pstats.Stats(pr, stream=s)
ps.sort_stats("cumulative").print_stats(45)
ps.sort_stats("tottime").print_stats(35)
open(out, "w").write(s.getvalue())
print("profile written", out)
