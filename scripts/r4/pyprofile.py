"""cProfile any benchmark script: python scripts/r4/pyprofile.py OUT.txt SCRIPT.py [args...]
(top functions by cumulative and by own time)."""
import cProfile
import io
import os
import pstats
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
out, script = sys.argv[1], sys.argv[2]
sys.argv = [script] + sys.argv[3:]
pr = cProfile.Profile()
pr.enable()
try:
    runpy.run_path(script, run_name="__main__")
finally:
    pr.disable()
    s = io.StringIO()
    ps = pstats.Stats(pr, stream=s)
    ps.sort_stats("cumulative").print_stats(50)
    ps.sort_stats("tottime").print_stats(40)
    open(out, "w").write(s.getvalue())
    print("profile written", out)
