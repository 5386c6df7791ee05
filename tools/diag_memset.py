"""diagnostic: does a zero written by a HIP-graph node survive replays?
variants: buffer allocated inside / before the capture; rr_zero / torch zero_"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"), REPO]
import torch  # noqa: E402

import roadrestore as rr  # noqa: E402
from roadrestore import ops  # noqa: E402

dev = torch.device("cuda:0")
n = 4096
for inside in (True, False):
    for fn in ("rr", "torch"):
        pre = None if inside else torch.empty(n + 64, device=dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            buf = torch.empty(n + 64, device=dev) if inside else pre
            if fn == "rr":
                ops.zero_(buf[:n])
            else:
                buf[:n].zero_()
            buf[n:].fill_(2.0)
        res = []
        for r in range(3):
            buf.fill_(7.0)
            g.replay()
            torch.cuda.synchronize()
            res.append(buf[:n].abs().max().item())
        print(f"inside={inside} {fn}: max after replays {res}")

# other rr kernels as graph nodes: an elementwise op writing a captured output
x = torch.rand(2, 8, 8, 64, device=dev)
sc = torch.rand(64, device=dev)
sh = torch.rand(64, device=dev)
ref = ops.affine_act(x, sc, sh)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    y = ops.affine_act(x, sc, sh)
res = []
for r in range(3):
    y.fill_(7.0)
    g.replay()
    torch.cuda.synchronize()
    res.append((y - ref).abs().max().item())
print("affine_act node: max err after replays", res)
buf = torch.empty(n, device=dev)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    ops.zero_(buf)
for r in range(3):
    buf.fill_(7.0)
    g.replay()
    torch.cuda.synchronize()
    print("zero only, replay", r, buf[:4].tolist(), buf.view(torch.int32)[:4].tolist(), (buf != 0).sum().item())
