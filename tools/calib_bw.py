#!/usr/bin/env python3
"""Achievable HBM bandwidth on this GPU with torch's own vectorised kernels (calibration
for the roofline: read-only sum, write-only fill, read+write copy, 2 GiB buffers)."""
import json

import torch


def timeit(fn, n=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n / 1e3


def main():
    nbytes = 2 << 30
    x = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda").uniform_()
    y = torch.empty_like(x)
    out = {}
    out["read_GBps"] = nbytes / timeit(lambda: x.sum()) / 1e9
    out["write_GBps"] = nbytes / timeit(lambda: y.fill_(1.0)) / 1e9
    out["copy_GBps"] = 2 * nbytes / timeit(lambda: y.copy_(x)) / 1e9
    print(json.dumps(out))


if __name__ == "__main__":
    main()
