#!/usr/bin/env python3
"""Measured HBM roof on this MI355X: streaming copy / read of a large buffer with
(a) the engine's 16-B copy kernel at several grid sizes, (b) hipMemcpy D2D via
torch, (c) torch's own copy kernel. The stencil's achieved bandwidth is judged
against the best of these, not against the datasheet."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=5):
    import torch
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    import torch
    import heat2d  # noqa: F401
    from heat2d.ops import _native as N
    torch.cuda.set_device(0)
    gb = float(os.environ.get("BW_GB", "8"))
    n = int(gb * 2**30) // 16 * 16
    a = torch.empty(n, dtype=torch.uint8, device="cuda")
    b = torch.empty(n, dtype=torch.uint8, device="cuda")
    a.fill_(1)
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for blocks in (1024, 2048, 4096, 8192, 16384):
        t = timeit(lambda: N.call("heat2d_copy", b.data_ptr(), a.data_ptr(), n, st, blocks))
        res[f"copy16_blocks{blocks}_TBps"] = 2 * n / t / 1e12
        t = timeit(lambda: N.call("heat2d_read", a.data_ptr(), n, sink.data_ptr(), st, blocks))
        res[f"read16_blocks{blocks}_TBps"] = n / t / 1e12
    t = timeit(lambda: b.copy_(a))
    res["torch_copy_TBps"] = 2 * n / t / 1e12
    af = a.view(torch.float32)
    t = timeit(lambda: af.sum())
    res["torch_sum_read_TBps"] = n / t / 1e12
    print(json.dumps({k: round(v, 3) for k, v in res.items()}))


if __name__ == "__main__":
    main()
