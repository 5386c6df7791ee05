"""The C ABI: the library loads without a GPU and exports every entry point
include/roadrestore.h declares; descriptors match the header layout; the
module trees match the reference's state_dict manifests.  No compute calls."""
import ctypes
import os
import re

import pytest

from oracle import seeded as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(REPO, "include", "roadrestore.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rr_[A-Za-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    import roadrestore
    lib = roadrestore.lib()
    declared = header_functions()
    assert len(declared) >= 30
    missing = [n for n in declared if not hasattr(lib.dll, n)]
    assert not missing, missing
    assert set(declared) == set(roadrestore.EXPORTED)
    assert lib.rr_version().startswith(b"roadrestore")


def test_descriptor_layouts(tmp_path):
    """The ctypes mirrors of the C descriptors have the C compiler's layout
    (sizeof / offsetof from include/roadrestore.h, built with gcc here)."""
    import shutil
    import subprocess
    from roadrestore._lib import BnBwdDesc, BnFinalizeDesc, IgemmDesc, PackJob, WgradDesc
    assert ctypes.sizeof(IgemmDesc) == 15 * 4
    assert ctypes.sizeof(WgradDesc) == 9 * 4
    checks = [("rr_bnbwd_desc", BnBwdDesc, ["P", "h", "pool_dy", "pool_idx", "eval", "dbias0", "dbias1"]),
              ("rr_bn_finalize_desc", BnFinalizeDesc, ["count", "part", "momentum", "scale",
                                                       "num_batches_tracked"]),
              ("rr_pack_job", PackJob, ["c_out", "begin"])]
    if shutil.which("gcc") is None:
        pytest.skip("no C compiler")
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "roadrestore.h"', "int main(void) {"]
    for cname, _, fields in checks:
        lines.append(f'  printf("%zu\\n", sizeof({cname}));')
        lines += [f'  printf("%zu\\n", offsetof({cname}, {f}));' for f in fields]
    lines += ["  return 0;", "}"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True,
                                          text=True).stdout.split()]
    want = []
    for _, cls, fields in checks:
        want.append(ctypes.sizeof(cls))
        want += [getattr(cls, f).offset for f in fields]
    assert got == want


def test_status_codes_raise():
    from roadrestore._lib import Lib
    with pytest.raises(RuntimeError, match="EINVAL"):
        Lib.check(-1, "x")


def test_invalid_descriptor_rejected_without_gpu():
    """Validation happens before any launch: a bad descriptor returns EINVAL."""
    import roadrestore
    from roadrestore._lib import IgemmDesc
    lib = roadrestore.lib()
    d = IgemmDesc(0, 0, 0, 8, 8, 64, 0, 64, 0, 0, 0, 0, 0, 0, 0)   # n = 0
    assert lib.rr_igemm(ctypes.byref(d), None, None, None, None, None, None, None, None, None) == -1
    d = IgemmDesc(1, 0, 1, 8, 8, 48, 0, 64, 0, 0, 0, 0, 0, 0, 0)   # c_in not a multiple of 64
    assert lib.rr_igemm(ctypes.byref(d), 1, None, 1, None, 1, None, None, None, None) == -2


@pytest.mark.parametrize("name,cls", [("simpleunet", "SimpleUNet"), ("resunet", "ResUNet")])
def test_module_trees_match_reference(name, cls):
    import roadrestore as rr
    m = getattr(rr, cls)()
    got = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    assert got == S.load_manifest(name)


def test_vgg_trees_match_reference():
    import roadrestore as rr
    got = [[k, list(v.shape)] for k, v in rr.VGGPerceptualLoss().state_dict().items()]
    assert got == S.load_manifest("perceptual")
    got = [[k, list(v.shape)] for k, v in rr.vgg16(num_classes=43).state_dict().items()]
    assert got == S.load_manifest("vgg16")


def test_reference_state_dict_loads():
    import roadrestore as rr
    m = rr.ResUNet()
    m.load_state_dict(S.model_state_dict("resunet"))     # strict: every key and shape


def test_cpu_tensors_rejected():
    import torch
    import roadrestore as rr
    m = rr.ResUNet()
    with pytest.raises(RuntimeError, match="GPU"):
        m(torch.zeros(1, 3, 64, 64))


def test_bn_finalize_out_validated_before_launch():
    """``out=`` must be two contiguous fp32 [C] tensors; checked on the host
    before any launch (no GPU needed)."""
    import torch
    import roadrestore as rr
    st = torch.zeros(4, 8, 2)
    z = torch.zeros(8)
    with pytest.raises(ValueError, match="out"):
        rr.ops.bn_finalize(st, 64, None, z, z, z, z, out=(torch.empty(7), torch.empty(8)))
    with pytest.raises(ValueError, match="out"):
        rr.ops.bn_finalize(st, 64, None, z, z, z, z, out=(torch.empty(8, 2)[:, 0], torch.empty(8)))
    # a bf16 / fp16 out of numel C would be overrun by C fp32 writes
    for dt in (torch.bfloat16, torch.float16):
        with pytest.raises(ValueError, match="out"):
            rr.ops.bn_finalize(st, 64, None, z, z, z, z, out=(torch.empty(8, dtype=dt), torch.empty(8)))
    # gamma / running stats of the wrong dtype or size
    with pytest.raises(ValueError, match="gamma"):
        rr.ops.bn_finalize(st, 64, None, z.double(), z, z, z)
    with pytest.raises(ValueError, match="running_var"):
        rr.ops.bn_finalize(st, 64, None, z, z, z, torch.zeros(9))
    # all-host operands: no host pointer ever reaches a launch
    with pytest.raises(RuntimeError, match="device"):
        rr.ops.bn_finalize(st, 64, None, z, z, z, z, out=(torch.empty(8), torch.empty(8)))


def rr_stat_blocks(d):
    import ctypes as C
    import roadrestore as rr
    return rr.lib().rr_igemm_stat_blocks(C.byref(d))


def test_kernel_selection_for_the_benched_layers():
    """The library reports which kernel owns each cfg3 layer (B = 512, bf16,
    64x64 input) -- host-only queries, no launch: the row-streaming conv and
    weight grad on the 64-channel 64x64 / 32x32 layers, the tap-reuse conv
    (conv3r) on the wider 32x32 .. 8x8 layers and on dec1's 64 + 64 concat
    (64x64 whole-row tiles, one pass), the LDS-halo weight grads on the 16x16 /
    8x8 ones."""
    from roadrestore import ops
    from roadrestore._lib import RR_BF16, RR_CONV3X3, IgemmDesc, WgradDesc
    want = {  # (h, c_in1, c_in2, c_out): (fwd, wgrad)
        (64, 64, 0, 64): ("stream3_kernel<64>", "swgrad_kernel<64>"),
        (64, 64, 64, 64): ("conv3r_kernel<64,64>", "swgrad_kernel<64>"),  # one pass, fp32 sum
        (32, 64, 0, 128): ("conv3r_kernel<32,128>", "swgrad_kernel<32>"),
        (32, 128, 64, 64): ("conv3r_kernel<32,64>", "swgrad_kernel<32>"),
        (16, 256, 0, 256): ("conv3r_kernel<16,128,w8>", "wgrad3_halo_kernel<16>"),
        (16, 256, 128, 128): ("conv3r_kernel<16,128,w8>", "wgrad3_halo_kernel<16>"),
        (8, 512, 0, 512): ("conv3r_kernel<8,128,w8>", "wgrad3_halo_kernel<8>"),
        (8, 512, 0, 256): ("conv3r_kernel<8,128,32,w8>", "wgrad3_halo_kernel<8>"),
    }
    for (h, c1, c2, co), (f, wg) in want.items():
        d = IgemmDesc(RR_BF16, RR_CONV3X3, 512, h, h, c1, c2, co, 0, 0, 0, 1, 0, 1, 0)
        assert ops.igemm_kernel_name(d) == f, (h, c1, c2, co, ops.igemm_kernel_name(d))
        assert ops.wgrad_kernel_name(WgradDesc(RR_BF16, RR_CONV3X3, 512, h, h, c1, c2, co, 0)) == wg
        if f.startswith("conv3r"):     # one BN-statistics partial row per 128 pixels
            assert rr_stat_blocks(d) == 512 * h * h // 128


def test_kernel_selection_odd_batches_stay_on_whole_rows():
    """host-only: a 16x16 / 8x8 map whose pixel count does not
    fill the first pick's 512-pixel tiles takes the 256- or 128-pixel
    whole-row tiles before the row-segment ones; only batches that fill none
    of them drop to segments."""
    from roadrestore import ops
    from roadrestore._lib import RR_BF16, RR_CONV3X3, IgemmDesc
    want = {  # (n, h, c_in, c_out): kernel (LDS-weight K loop)
        (3, 16, 256, 256): "conv3r_kernel<16,128,32,w8>",    # P = 768: 256-pixel tiles
        (512, 16, 256, 256): "conv3r_kernel<16,128,w8>",     # the benched batch: 512
        (1, 8, 512, 512): "conv3r_kernel<s1,128,w8>",        # P = 64: no whole-row tile fits
        (3, 8, 512, 512): "conv3r_kernel<s1,128,w8>",        # P = 192
        (2, 8, 512, 512): "conv3r_kernel<8,128,32>",         # P = 128: 4-wave 128-pixel tiles
        (1, 16, 64, 64): "conv3r_kernel<16,64,32>",          # P = 256, 64 channels
    }
    for (n, h, ci, co), f in want.items():
        d = IgemmDesc(RR_BF16, RR_CONV3X3, n, h, h, ci, 0, co, 0, 0, 0, 1, 0, 1, 0)
        assert ops.igemm_kernel_name(d) == f, (n, h, ci, co, ops.igemm_kernel_name(d))


def test_kernel_selection_at_the_reference_geometry():
    """host-only: the 3x3 convs of the reference's 224x224 pipeline and its
    112 / 56 / 28 / 14 maps (14:202-205, 17:66, 18:28-32) take the
    row-segment tiles of the tap-reuse conv (32-column segments above W = 16,
    16-column at 14x14), one statistics row per wave row of a tile (the
    row-streaming kernel's column strips have no statistics epilogue)"""
    from roadrestore import ops
    from roadrestore._lib import RR_BF16, RR_CONV3X3, IgemmDesc
    want = {  # (h, c_in1, c_in2, c_out): (kernel, rows per image)
        (224, 64, 0, 64): ("conv3r_kernel<s2,64>", 7 * 14 * 4),
        (224, 64, 64, 64): ("conv3r_kernel<s2,64>", 7 * 14 * 4),
        (112, 64, 0, 128): ("conv3r_kernel<s2,128>", 4 * 14 * 2),
        (56, 128, 0, 256): ("conv3r_kernel<s2,128>", 2 * 7 * 2),
        (28, 256, 0, 512): ("conv3r_kernel<s2,128,w8>", 1 * 2 * 4),
        (14, 512, 0, 512): ("conv3r_kernel<s1,128,w8>", 1 * 1 * 2),
    }
    for (h, c1, c2, co), (f, rows) in want.items():
        d = IgemmDesc(RR_BF16, RR_CONV3X3, 16, h, h, c1, c2, co, 0, 0, 0, 1, 0, 1, 0)
        assert ops.igemm_kernel_name(d) == f, (h, ops.igemm_kernel_name(d))
        assert rr_stat_blocks(d) == 16 * rows, (h, rr_stat_blocks(d))


def test_igemm_ex_kernel_selection():
    """host-only: rr_igemm_ex's fused PReLU / residual epilogues run on the
    tap-reuse conv or, for the 64 -> 64 maps it takes, the row-streaming
    kernel (column strips at 224); other descriptors report "unsupported" (the
    engine then keeps the activation pass)"""
    from roadrestore import ops
    from roadrestore._lib import RR_ACT_POOL, RR_ACT_PRELU, RR_ACT_RES, RR_BF16, RR_CONV3X3, RR_F32, IgemmDesc

    def name(dt, h, c, act, bnbwd=False):
        return ops.igemm_kernel_name(IgemmDesc(dt, RR_CONV3X3, 4, h, h, c, 0, c, 0, act, 0, 1, 0, 0, 0),
                                     bnbwd=bnbwd)
    assert name(RR_BF16, 224, 64, RR_ACT_PRELU) == "stream3_kernel<s32>"
    assert name(RR_BF16, 224, 64, 1 | RR_ACT_RES | RR_ACT_POOL) == "stream3_kernel<s32>"
    assert name(RR_BF16, 224, 128, RR_ACT_PRELU) == "conv3r_kernel<s2,128>"
    assert name(RR_BF16, 16, 256, 1 | RR_ACT_RES).startswith("conv3r_kernel<16,128")
    assert name(RR_F32, 224, 64, RR_ACT_PRELU) == "unsupported"
    assert name(RR_BF16, 224, 64, RR_ACT_PRELU, bnbwd=True) == "unsupported"


def _s1name(mode, n, h, w, c1, c2, co, split=0, act=0, acc=0, bias=0, mask=0, stats=0, nchw_=0):
    from roadrestore import ops
    from roadrestore._lib import RR_BF16, IgemmDesc
    return ops.igemm_kernel_name(IgemmDesc(RR_BF16, mode, n, h, w, c1, c2, co, split, act, acc,
                                           bias, mask, stats, nchw_))


def test_stream1_benched_shapes_selected():
    """host-only: the cfg3 (B = 512) 1x1 / convT layers the planner gives to
    the streaming kernel"""
    from roadrestore._lib import RR_CONV1X1, RR_CONVT_DOWN, RR_CONVT_UP
    assert _s1name(RR_CONV1X1, 512, 32, 32, 64, 0, 128, bias=1, stats=1) == "stream1_kernel<4,2>"
    assert _s1name(RR_CONV1X1, 512, 64, 64, 64, 64, 64, bias=1, stats=1) == "stream1_kernel<4,4>"
    assert _s1name(RR_CONV1X1, 512, 64, 64, 64, 0, 128, split=64, acc=1) == "stream1_kernel<8,2>"
    assert _s1name(RR_CONV1X1, 512, 64, 64, 64, 0, 3, bias=1, nchw_=1) == "stream1_kernel<1,2>"
    assert _s1name(RR_CONVT_UP, 512, 32, 32, 64, 0, 256, bias=1) == "stream1_kernel<8,2>"
    assert _s1name(RR_CONVT_DOWN, 512, 32, 32, 64, 0, 64, mask=1).startswith("igemm_kernel")
    # 8x8 maps (P = 32768) stay on the tiled kernel
    assert _s1name(RR_CONV1X1, 512, 8, 8, 256, 0, 512, bias=1, stats=1).startswith("igemm_kernel")


def test_custom_ops_registered_with_fake_shapes():
    """The hot path is registered as PyTorch custom ops (torch.ops.rr.*) with
    fake kernels: shapes propagate without a device (torch.compile / meta
    tracing), and every op the modules call exists."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    import roadrestore as rr
    from roadrestore import torch_ops
    assert all(hasattr(torch.ops.rr, n) for n in torch_ops.OPS)
    s = str(torch.ops.rr.resunet_forward.default._schema)
    assert s.startswith("rr::resunet_forward(Tensor x, Tensor[] params,"), s
    res, su, blk, vgg = rr.ResUNet(), rr.SimpleUNet(), rr.ResidualBlock(64, 128), rr.vgg16()
    with FakeTensorMode(allow_non_fake_inputs=True):
        x = torch.empty(2, 3, 36, 52, device="cuda")
        out, h = torch.ops.rr.resunet_forward(x, list(res.parameters()), res._op_key, True)
        assert out.shape == (2, 3, 36, 52) and h.dtype == torch.int64
        out, _ = torch.ops.rr.simple_unet_forward(torch.empty(2, 3, 64, 64, device="cuda"),
                                                  list(su.parameters()), su._op_key, False)
        assert out.shape == (2, 3, 64, 64)
        out, _ = torch.ops.rr.resblock_forward(torch.empty(2, 64, 16, 16, device="cuda"),
                                               list(blk.parameters()), blk._op_key, False)
        assert out.shape == (2, 128, 16, 16)
        lg = torch.ops.rr.vgg16_logits(torch.empty(5, 3, 224, 224, device="cuda"),
                                       list(vgg.parameters()), vgg._op_key)
        assert lg.shape == (5, 43) and lg.dtype == torch.float32
        assert torch.ops.rr.nearest_resize(torch.empty(2, 4, 6, 128, device="cuda"), 9, 13).shape \
            == (2, 9, 13, 128)
        u8 = torch.ops.rr.to_uint8_hwc(torch.empty(2, 3, 8, 8, device="cuda"), True)
        assert u8.shape == (2, 8, 8, 3) and u8.dtype == torch.uint8
        assert torch.ops.rr.argmax_rows(torch.empty(7, 43, device="cuda")).shape == (7,)
        loss, _ = torch.ops.rr.unified_loss(torch.empty(2, 3, 8, 8, device="cuda"),
                                            torch.empty(2, 3, 8, 8, device="cuda"), 0, 0.1, 1.0,
                                            True)
        assert loss.shape == ()
        g = torch.ops.rr.perceptual_loss_backward(torch.empty((), device="cuda"),
                                                  torch.empty((), dtype=torch.int64),
                                                  torch.empty(2, 3, 8, 8, device="cuda"))
        assert g.shape == (2, 3, 8, 8)


def test_saved_forward_state_lives_with_its_handle():
    """The forward state table (torch_ops._SAVED) holds an entry only while
    its handle tensor lives: the autograd node keeps the handle, so a graph
    dropped without a backward frees the state; a handle never kept (no
    backward possible) frees it at once; the backward pops it."""
    import gc
    from roadrestore import torch_ops as T
    n0 = T.saved_state_count()
    hs = [T._stash(("state", i)) for i in range(50)]
    assert T.saved_state_count() == n0 + 50
    del hs
    gc.collect()
    assert T.saved_state_count() == n0
    h = T._stash("x")
    assert T._unstash(h) == "x" and T.saved_state_count() == n0
    with pytest.raises(RuntimeError, match="already consumed"):
        T._unstash(h)
    del h
    gc.collect()
    assert T.saved_state_count() == n0


def test_stream3_column_strips_selected(monkeypatch):
    """host-only: the row-streaming kernel's column-strip mode -- 32-wide
    strips of any 32-multiple width above 64 (the reference's 224) -- for the
    plain / bias / ReLU and eval flag sets; the training epilogues stay on the
    tap-reuse conv's row-segment tiles, and RR_PATH stream3_strips=0 hands the
    wide maps back to them"""
    from rrpath import set_path
    from roadrestore import ops
    from roadrestore._lib import RR_BF16, RR_CONV3X3, IgemmDesc

    def name(n, h, w, c1=64, c2=0, co=64, stats=0, mask=0, bnbwd=False):
        return ops.igemm_kernel_name(IgemmDesc(RR_BF16, RR_CONV3X3, n, h, w, c1, c2, co, 0, 0, 0, 1, mask,
                                               stats, 0), bnbwd=bnbwd)
    assert name(2, 224, 224) == "stream3_kernel<s32>"
    assert name(10, 40, 224) == "stream3_kernel<s32>"
    assert name(5, 128, 128) == "stream3_kernel<s32>"
    assert name(2, 224, 224, stats=1) == "conv3r_kernel<s2,64>"    # training epilogues: tap-reuse
    assert name(2, 224, 224, mask=1) == "conv3r_kernel<s2,64>"
    assert name(2, 224, 224, bnbwd=True) == "conv3r_kernel<s2,64>"
    assert name(16, 64, 64, stats=1) == "stream3_kernel<64>"
    assert name(4, 104, 160) == "stream3_kernel<s32>"
    assert name(16, 64, 64) == "stream3_kernel<64>"
    assert name(1, 224, 224) == "conv3r_kernel<s2,64>"        # P < 256 steps of 256 pixels
    assert name(2, 220, 224) == "conv3r_kernel<s2,64>"        # h % 8: no whole steps
    assert name(8, 112, 112) == "conv3r_kernel<s2,64>"        # 112 % 32: no strip width
    assert name(2, 224, 224, 64, 64) == "conv3r_kernel<s2,64>"   # concat: one tap-reuse pass
    set_path(monkeypatch, "stream3_strips", "0")
    assert name(2, 224, 224) == "conv3r_kernel<s2,64>"
    assert name(16, 64, 64) == "stream3_kernel<64>"
