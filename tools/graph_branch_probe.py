"""Does a HIP graph run two stream branches concurrently on this ROCm?
Two torch.cuda._sleep kernels (one workgroup each), one per stream, eager vs
captured; concurrent branches take ~1x the sleep, serialized ~2x."""
import time
import torch

torch.cuda.set_device(0)
cyc = 50_000_000
main = torch.cuda.current_stream()
side = torch.cuda.Stream()


def body():
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc)
    torch.cuda._sleep(cyc)
    torch.cuda.current_stream().wait_stream(side)


def t(fn, n=5):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


one = t(lambda: torch.cuda._sleep(cyc))
eager = t(body)
s2 = torch.cuda.Stream()
with torch.cuda.stream(s2):
    body()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
graph = t(g.replay)
print(f"one sleep {one:.2f} ms | two streams eager {eager:.2f} ms | graph {graph:.2f} ms")
