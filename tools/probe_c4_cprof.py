"""Host profile of the C4 ring (tools/probe_c4.py's loop under cProfile): where the wall time
beyond the kernels goes."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_c4  # noqa: E402

os.environ.setdefault("PROBE_RUNS", "20")
pr = cProfile.Profile()
pr.enable()
probe_c4.main()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
