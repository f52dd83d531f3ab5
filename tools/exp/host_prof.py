"""Host-side profile of bench.py's timed steps only: cProfile enabled inside
timed_region, then the per-step functions by cumulative and own time.
Usage: python tools/exp/host_prof.py [out]"""
import cProfile, io, os, pstats, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/host_prof.txt"
sys.argv = ["bench.py", "--steps", "100", "--warmup", "10", "--no-cpu-baseline"]
import bench  # noqa: E402
pr = cProfile.Profile()
_tr = bench.timed_region


def timed_region(*a, **k):
    pr.enable()
    try:
        return _tr(*a, **k)
    finally:
        pr.disable()


bench.timed_region = timed_region
bench.main()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(50)
s2 = io.StringIO()
pstats.Stats(pr, stream=s2).sort_stats("cumulative").print_stats(70)
with open(out, "w") as fh:
    fh.write(s.getvalue() + "\n\n==== cumulative ====\n" + s2.getvalue())
