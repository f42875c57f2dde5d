"""Do independent branches of one captured HIP graph run concurrently on this ROCm?  Two chains
of latency-bound launches (small matmuls) captured on two streams (fork / join) vs the same
chains captured on one stream; also the eager two-stream form.
usage: python tools/graph_branches.py"""
import time

import torch

dev = torch.device("cuda", 0)
x = [torch.randn(256, 256, device=dev) for _ in range(2)]
w = torch.randn(256, 256, device=dev) * 0.05
N = 200


def chain(i):
    y = x[i]
    for _ in range(N):
        y = torch.tanh(y @ w)
    return y


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


main = torch.cuda.current_stream(dev)
side = torch.cuda.Stream(dev)


def two_streams():
    side.wait_stream(main)
    chain(0)
    with torch.cuda.stream(side):
        chain(1)
    main.wait_stream(side)


def one_stream():
    chain(0)
    chain(1)


graphs = {}
for name, fn in (("one stream", one_stream), ("two streams", two_streams)):
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(main)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):
        fn()  # warm-up on the capture stream
        torch.cuda.synchronize()
        g.capture_begin()
        fn()
        g.capture_end()
    main.wait_stream(cap)
    graphs[name] = g
print(f"eager one stream    {timed(one_stream):9.1f} us")
print(f"eager two streams   {timed(two_streams):9.1f} us")
for name, g in graphs.items():
    print(f"graph {name:12s}  {timed(g.replay):9.1f} us")
