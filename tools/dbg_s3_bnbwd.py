import os, sys
sys.path.insert(0, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd")
import torch
import roadrestore as rr
from roadrestore._lib import RR_CONV3X3
ops = rr.ops
dev = torch.device("cuda:0")
def rnd(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)
def nhwc(x): return x.permute(0, 2, 3, 1).contiguous().to(dev, torch.bfloat16)
def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu(); return ((a - b).norm() / b.norm()).item()
n, h, w, C = 16, 64, 64, 64
g2 = nhwc(rnd(n, C, h, w, seed=51))
wt = (rnd(C, C, 3, 3, seed=52) * (1.0 / (3 * C ** 0.5))).to(dev)
_, wd = ops.pack_conv(wt, torch.bfloat16)
t1 = nhwc(rnd(n, C, h, w, seed=53) * 2 + 0.3)
tf = t1.float().reshape(-1, C)
mean = tf.mean(0); inv = 1.0 / torch.sqrt(tf.var(0, unbiased=False) + 1e-5)
gamma = (torch.rand(C, generator=torch.Generator().manual_seed(54)) + 0.5).to(dev)
beta = (torch.rand(C, generator=torch.Generator().manual_seed(55)) - 0.5).to(dev)
s1 = gamma * inv; sh1 = beta - mean * s1
alpha = torch.tensor([0.23], device=dev)
os.environ["RR_STREAM3"] = "0"
da1, _, _ = ops.igemm(RR_CONV3X3, g2, None, n, h, w, wd, C)
ref = ops.bn_backward(da1, t1, mean, inv, gamma, mask_kind=2, aux=t1, aff_s=s1, aff_b=sh1, alpha=alpha)
for rep in range(3):
    for tag in ("0", "1"):
        os.environ["RR_STREAM3"] = tag
        gm, part, rows, arows = ops.igemm_bnbwd(RR_CONV3X3, g2, n, h, w, wd, C, t1, mean, inv, s1, sh1, alpha)
        r = ops.bn_backward_rows(gm, part, rows, arows, t1, mean, inv, gamma)
        torch.cuda.synchronize()
        print(tag, rep, "dt0", rel(r["dt0"], ref["dt0"]), "dg", rel(r["dgamma0"], ref["dgamma0"]), "db", rel(r["dbeta0"], ref["dbeta0"]), "da", rel(r["dalpha"], ref["dalpha"]), "gm-hash", gm.float().sum().item())
# direct gm check vs fp32 computation
os.environ["RR_STREAM3"] = "1"
gm, part, rows, arows = ops.igemm_bnbwd(RR_CONV3X3, g2, n, h, w, wd, C, t1, mean, inv, s1, sh1, alpha)
import torch.nn.functional as F
gx = F.conv2d(g2.float().permute(0,3,1,2), wd.float().view(C,9,C).permute(0,2,1).reshape(C,C,3,3), padding=1) if False else None
os.environ["RR_STREAM3"] = "0"
gm0, _, _, _ = ops.igemm_bnbwd(RR_CONV3X3, g2, n, h, w, wd, C, t1, mean, inv, s1, sh1, alpha)
d = (gm.float() - gm0.float()).abs()
print("gm stream vs tiled: max", d.max().item(), "count>0.01", (d > 0.01).sum().item(), "rel", rel(gm, gm0))
idx = (d == d.max()).nonzero()[:5]
print(idx)
bad = (d > 0.01)
nz = bad.nonzero()
print("bad n:", torch.bincount(nz[:, 0], minlength=n).tolist())
print("bad y mod 2:", torch.bincount(nz[:, 1] % 2).tolist(), "y:", torch.bincount(nz[:, 1], minlength=h).tolist())
print("bad x//16:", torch.bincount(nz[:, 2] // 16).tolist(), "x%16:", torch.bincount(nz[:, 2] % 16, minlength=16).tolist())
print("bad c//16:", torch.bincount(nz[:, 3] // 16).tolist(), "c%16:", torch.bincount(nz[:, 3] % 16, minlength=16).tolist())
# repeatability of the other epilogues
os.environ["RR_STREAM3"] = "1"
x = g2
b = torch.randn(64, device=dev)
outs = []
for rep in range(4):
    y, _, st = ops.igemm(RR_CONV3X3, x, None, n, h, w, wd, 64, bias=b, stats=True)
    y2, _, _ = ops.igemm(RR_CONV3X3, x, None, n, h, w, wd, 64, out=t1.clone(), accumulate=True)
    y3, _, _ = ops.igemm(RR_CONV3X3, x, None, n, h, w, wd, 64, bias=b, act=1)
    outs.append((y.float(), st.double().sum(0), y2.float(), y3.float()))
for k, name in enumerate(["fwd+stats y", "stats", "acc", "relu"]):
    print(name, [ (outs[i][k] - outs[0][k]).abs().max().item() for i in range(1, 4)])
