#!/usr/bin/env python3
"""Host time spent inside CUDAGraph.replay() during config 5's rl_bench (is the period graph
launch the wall-time limiter?).  Prints the rl_bench line, then the replay-call statistics."""
import os
import runpy
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ts = []
_orig = torch.cuda.CUDAGraph.replay


def _timed(self):
    t = time.perf_counter()
    _orig(self)
    ts.append(time.perf_counter() - t)


torch.cuda.CUDAGraph.replay = _timed
sys.argv = [os.path.join(REPO, "tools", "rl_bench.py"), "--algo", "dqn"]
runpy.run_path(sys.argv[0], run_name="__main__")
tail = ts[len(ts) // 2:]
print({"replays": len(ts), "host_us_median": round(1e6 * statistics.median(tail), 1),
       "host_us_p90": round(1e6 * sorted(tail)[int(0.9 * len(tail))], 1)})
