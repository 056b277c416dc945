#!/usr/bin/env python3
"""A/B harness: run bench.py's workload against another build of liblbk8s.so.

    python tools/abtest.py --lib exp/liblbk8s_X.so [bench.py arguments]

Experimental builds (variants of the kernels compiled from modified sources) live under
exp/ (git-ignored, shipped to the GPU box with the snapshot); the product package always
loads its own in-tree liblbk8s.so.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gym-loadbalancing_amd")]


def main():
    argv = sys.argv[1:]
    lib = None
    if "--lib" in argv:
        i = argv.index("--lib")
        lib = os.path.abspath(argv[i + 1])
        del argv[i:i + 2]
    from lbk8s import _native
    if lib:
        _native.LIB_PATH = lib
    import bench
    bench.main(argv + ["--no-cpu-baseline"])
    print("lib:", os.path.basename(lib or _native.LIB_PATH), flush=True)


if __name__ == "__main__":
    main()
