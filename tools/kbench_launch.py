"""Per-kernel floor of a hipGraph replay on this box: N back-to-back tiny
kernels (1-element add) captured in one graph, and N gathers of the S1 size
(8192 x 13 floats), timed over many replays."""
import json
import time

import torch


def timed(fn, reps=200):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


x = torch.zeros(1, device="cuda")
src = torch.randn(13, 8192, device="cuda")
dst = torch.empty(8192, 13, device="cuda")
out = {}
for n in (1, 10, 50):
    out["tiny_add_x%d_us" % n] = 1e6 * timed(lambda: [x.add_(1.0) for _ in range(n)]) / n
    out["gather_8192x13_x%d_us" % n] = 1e6 * timed(lambda: [dst.copy_(src.t()) for _ in range(n)]) / n
print(json.dumps(out))
