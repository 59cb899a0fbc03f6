"""cProfile of headline bench steps (host-side overhead between kernels)."""
import cProfile, pstats, sys, io, runpy
sys.argv = ["bench.py", "--steps", "2", "--warmup", "1"]
pr = cProfile.Profile()
pr.enable()
try:
    runpy.run_path("bench.py", run_name="__main__")
except SystemExit:
    pass
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
print(s.getvalue())
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue())
