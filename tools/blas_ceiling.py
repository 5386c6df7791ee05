"""hipBLASLt (torch.matmul bf16) on the im2col GEMM shapes of the cfg3 3x3
convs: the library's rate on the same M x N x K is the practical ceiling the
implicit-GEMM kernels are compared with (no im2col cost counted)."""
import torch

dev = torch.device("cuda:0")
shapes = [  # (M = pixels, N = c_out, K = 9 c_in, layer)
    (32768, 512, 4608, "8x8 c512->512"),
    (32768, 512, 2304, "8x8 c256->512"),
    (131072, 256, 2304, "16x16 c256->256"),
    (131072, 256, 1152, "16x16 c128->256"),
    (524288, 128, 1152, "32x32 c128->128"),
    (524288, 128, 576, "32x32 c64->128"),
    (524288, 64, 1728, "32x32 c192->64"),
    (2097152, 64, 1152, "64x64 c128->64"),
    (2097152, 64, 576, "64x64 c64->64"),
]
for M, N, K, tag in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 20
    s.record()
    for _ in range(it):
        c = a @ b
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / it
    fl = 2.0 * M * N * K
    # also the transposed form (N x K weights times K x M)
    bt = b.t().contiguous()
    s.record()
    for _ in range(it):
        c2 = bt @ a.t()
    e.record()
    torch.cuda.synchronize()
    ms2 = s.elapsed_time(e) / it
    print(f"{tag:18s} M={M:8d} N={N:4d} K={K:5d}  {ms*1e3:8.1f} us {fl/ms/1e9:7.1f} TF/s | "
          f"W@X^T {ms2*1e3:8.1f} us {fl/ms2/1e9:7.1f} TF/s", flush=True)
