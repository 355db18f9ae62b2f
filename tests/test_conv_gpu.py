"""Implicit-GEMM convolution kernels (csrc/kernels/conv.hip) vs a PyTorch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

import dtg  # noqa: F401
from dtg import ops
from dtg.ops import conv as conv_ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CASES = [
    # N, C, K, H, R, stride, pad
    (4, 64, 64, 14, 3, 1, 1),
    (2, 128, 128, 28, 3, 2, 1),
    (3, 64, 128, 9, 3, 1, 1),      # odd spatial size, partial tiles
    (2, 256, 512, 14, 1, 2, 0),    # 1x1 stride-2 downsample
    (2, 128, 64, 7, 3, 1, 1),      # skinny N (fwd) / skinny C (dgrad)
    (2, 64, 128, 7, 3, 2, 1),      # strided dgrad, odd size: unequal residue classes, skinny C
    (2, 128, 64, 9, 1, 2, 0),      # 1x1/s2 dgrad, odd size: odd residue classes get no tap (zeros)
    (2, 64, 64, 10, 3, 3, 1),      # stride 3
    (2, 64, 64, 12, 5, 2, 2),      # 5x5 stride 2
]


@pytest.mark.parametrize("N,C,K,H,R,st,pad", CASES)
def test_conv_fwd_bwd(N, C, K, H, R, st, pad):
    g = torch.Generator(device="cpu").manual_seed(N * 1000 + C + K + H)
    x = torch.randn(N, C, H, H, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, generator=g) * (2.0 / (C * R * R)) ** 0.5).to(DEV, torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    x.requires_grad_()
    w.requires_grad_()
    y = ops.conv2d(x, w, st, pad)
    yr = F.conv2d(xr, wr, None, st, pad)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    gy = torch.randn(yr.shape, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(gy)
    yr.backward(gy.float())
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2


def test_conv_direct_grad_into_flat_buffer():
    from dtg.models.layers import Conv2d
    from dtg.parallel import FlatParams
    torch.manual_seed(0)
    m = Conv2d(64, 128, 3, 1, 1).to(DEV)
    ref_w = m.weight.detach().clone().float()
    flat = FlatParams(m)
    x = torch.randn(2, 64, 10, 10, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for _ in range(2):  # accumulates (beta = 1) across two backwards
        m(x).float().square().sum().backward()
    xr = x.float().requires_grad_()
    wr = m.weight.detach().float().requires_grad_()
    F.conv2d(xr, wr, None, 1, 1).square().sum().backward()
    g = m.weight.grad
    assert g.data_ptr() >= flat.groups["compute"].grad.data_ptr()
    assert _rel(g, 2 * wr.grad) < 3e-2
    assert ref_w.shape == g.shape


@pytest.mark.parametrize("R,st,pad,H", [(3, 2, 1, 56), (1, 2, 0, 28), (3, 2, 1, 15)])
def test_conv_dgrad_strided_accumulate(R, st, pad, H):
    """Residue-class dgrad with beta = 1 into an existing buffer (the ResNet projection path)."""
    from dtg.ops._native import lib
    g = torch.Generator(device="cpu").manual_seed(R * 100 + H)
    N, C, K = 2, 128, 256
    P = (H + 2 * pad - R) // st + 1
    dy = torch.randn(N, P, P, K, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(K, R, R, C, generator=g) * 0.05).to(DEV, torch.bfloat16)
    base = torch.randn(N, H, H, C, generator=g).to(DEV, torch.bfloat16)
    out = base.clone()
    lib().conv_dgrad(dy, w, H, H, st, pad, out=out, beta=1.0)
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                     st, pad).permute(0, 2, 3, 1)
    assert _rel(out, base.float() + ref) < 1e-2
    fresh = lib().conv_dgrad(dy, w, H, H, st, pad)
    assert _rel(fresh, ref) < 1e-2


@pytest.mark.parametrize("pairs", ["1", "0"])
@pytest.mark.parametrize("N,C,K,H,R,st,pad", [(2, 3, 64, 32, 7, 2, 3), (2, 3, 64, 23, 7, 2, 3), (3, 4, 128, 16, 3, 1, 1),
                                              (2, 3, 64, 224, 7, 2, 3), (2, 2, 64, 31, 5, 2, 2)])
def test_conv_c8_stem(N, C, K, H, R, st, pad, pairs, monkeypatch):
    """Few-channel input (the ResNet stem): implicit-GEMM fwd + wgrad on the input padded to 8 channels,
    or (stride 2, <= 4 channels, pairs=1) packed as pixel pairs (ops/conv.py stem_pairs)."""
    monkeypatch.setattr(conv_ops, "_PAIRS", pairs != "0")
    g = torch.Generator(device="cpu").manual_seed(7 + H)
    x = torch.randn(N, C, H, H, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, generator=g) * (2.0 / (C * R * R)) ** 0.5).to(DEV, torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last).requires_grad_()
    y = ops.conv2d(x, w, st, pad)
    assert "ConvC8" in type(y.grad_fn).__name__
    wr = w.detach().float().requires_grad_()
    yr = F.conv2d(x.float(), wr, None, st, pad)
    assert y.shape == yr.shape and _rel(y, yr) < 1e-2
    gy = torch.randn(yr.shape, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(gy)
    yr.backward(gy.float())
    assert _rel(w.grad, wr.grad) < 2e-2


@pytest.mark.parametrize("N,C,H,W,pad,S", [(2, 3, 224, 224, 3, 7), (3, 3, 23, 29, 3, 7), (2, 2, 31, 31, 2, 5),
                                           (1, 4, 12, 14, 1, 3), (1, 1, 10, 10, 0, 4)])
def test_stem_pack_pairs_matches_pad(N, C, H, W, pad, S):
    """The one-pass pixel-pair packing kernel (stem.hip) equals the F.pad form of ops/conv.py stem_pairs."""
    from dtg.ops.conv import stem_pairs
    g = torch.Generator(device="cpu").manual_seed(H + W)
    x = torch.randn(N, C, H, W, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, C, S, S, generator=g).bfloat16()
    ref, wref, _ = stem_pairs(x, w, 2, pad)          # CPU: F.pad
    got, wgot, _ = stem_pairs(x.to(DEV), w.to(DEV), 2, pad)
    assert got.shape == ref.shape and torch.equal(got.cpu(), ref)
    assert torch.equal(wgot.cpu(), wref)




@pytest.mark.parametrize("N", [1, 3])
def test_stem_stream_conv_matches_tiled(N):
    """The streaming stem conv (gemm_expand.hip stem_stream_bn_kernel: persistent workgroups, all weights in
    registers, gathered 64-row blocks through a 3-deep LDS-DMA ring) equals the tiled implicit GEMM on ResNet's
    pixel-pair stem at 224 x 224 (fewer blocks than workgroups at N = 1), output and BN statistics, and the fp32
    conv."""
    from dtg.ops.conv import stem_pairs
    from dtg.ops._native import lib
    L = lib()
    g = torch.Generator(device="cpu").manual_seed(11)
    x = torch.randn(N, 3, 224, 224, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x8, w8, (rk, sk) = stem_pairs(x, w, 2, 3)
    out = []
    for on in (0, 1):
        L.stem_stream_set(on)
        try:
            y, part = L.conv_fwd_c8(x8, w8, rk, sk, 2, 0, True, stride_w=1)
        finally:
            L.stem_stream_set(1)
        out.append((y.float(), part.view(-1, 2, 64).sum(0)))
    (yt, pt), (ys, ps) = out
    assert _rel(ys, yt) < 1e-3
    assert _rel(ps[0], pt[0]) < 1e-3 and _rel(ps[1], pt[1]) < 1e-3
    ref = F.conv2d(x.float(), w.float(), None, 2, 3).permute(0, 2, 3, 1)
    assert _rel(ys.view_as(ref), ref) < 1e-2
    yf = ys.reshape(-1, 64)
    assert _rel(ps[0], yf.sum(0)) < 1e-3


@pytest.mark.parametrize("N,H", [(3, 56), (2, 28), (2, 30), (40, 56), (75, 28)])
def test_conv_fwd_bn_halo_64(N, H):
    """conv_fwd_bn for ResNet's stage-1 3x3 (64 -> 64, stride 1, pad 1): H % 4 == 0 runs the direct halo-tile conv
    (csrc/kernels/conv_halo.hip), H = 30 the implicit GEMM; output against the fp32 conv, the BN-statistics partials
    against the stored output's column sums and sums of squares.  N = 40 at 56x56 (560 bands) and N = 75 at 28x28
    (525 bands) make every persistent workgroup walk 2-3 bands through the double-buffered halo, as at b1024."""
    from dtg.ops._native import lib
    L = lib()
    g = torch.Generator(device="cpu").manual_seed(21 + H)
    x = torch.randn(N, H, H, 64, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, generator=g) * 0.05).to(DEV, torch.bfloat16)
    y, part = L.conv_fwd_bn(x, w, 1, 1)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2
    p = part.view(-1, 2, 64).sum(0)
    yf = y.float().reshape(-1, 64)
    assert _rel(p[0], yf.sum(0)) < 1e-3 and _rel(p[1], (yf * yf).sum(0)) < 1e-3


@pytest.mark.parametrize("N,beta,bf16_out", [(2, 0.0, False), (19, 1.0, False), (3, 0.0, True)])
def test_conv_wgrad_halo_64(N, beta, bf16_out):
    """conv_wgrad for ResNet's stage-1 3x3 (64 -> 64, s1, p1, 56x56) runs the persistent halo-tile weight gradient
    (csrc/kernels/conv_halo.hip, one fp32 slab per workgroup + the split-K reduce): against the fp32 conv2d_weight and
    the implicit-GEMM wgrad (conv_halo_wgrad_set(0)).  N = 19: 266 bands over 256 workgroups (some walk two);
    beta = 1 accumulates into an existing gradient; bf16_out writes a bf16 dw."""
    from dtg.ops._native import lib
    L = lib()
    g = torch.Generator(device="cpu").manual_seed(60 + N)
    x = torch.randn(N, 56, 56, 64, generator=g).to(DEV, torch.bfloat16)
    dy = torch.randn(N, 56, 56, 64, generator=g).to(DEV, torch.bfloat16)
    dw0 = torch.randn(64, 3, 3, 64, generator=g).to(DEV)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 64, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      padding=1).permute(0, 2, 3, 1) + beta * dw0
    outs = []
    for halo in (1, 0):
        dw = dw0.clone().to(torch.bfloat16 if bf16_out else torch.float32)
        L.conv_halo_wgrad_set(halo)
        try:
            L.conv_wgrad(dy, x, dw, beta, 1, 1)
        finally:
            L.conv_halo_wgrad_set(1)
        assert _rel(dw, ref) < (1e-2 if bf16_out else 2e-3)
        outs.append(dw.float())
    assert _rel(outs[0], outs[1]) < (1e-2 if bf16_out else 2e-3)


@pytest.mark.parametrize("N,H,C,K,beta", [(40, 28, 128, 128, 0.0), (64, 14, 256, 256, 1.0), (64, 7, 512, 512, 0.0),
                                          (12, 28, 64, 128, 0.0), (20, 14, 256, 128, 0.0), (9, 7, 128, 512, 1.0)])
def test_conv_wgrad_lin_halo(N, H, C, K, beta):
    """conv_wgrad for the 3x3 / s1 / p1 layers of ResNet stages 2-4 (28x28 x 128, 14x14 x 256, 7x7 x 512) runs the
    linear-halo weight gradient (csrc/kernels/conv_halo.hip conv3x3_lin_wgrad_kernel: the batch as one tall image
    with shared zero rows / columns, 64 x 576 blocks per workgroup, XCD-grouped channel-block pairs): against the fp32
    conv2d_weight and the implicit-GEMM wgrad (conv_lin_wgrad_set(0)).  The first three shapes put 2-4 bands on
    every persistent workgroup (the pipelined next-band staging); the others cover C != K block pairs."""
    from dtg.ops._native import lib
    L = lib()
    g = torch.Generator(device="cpu").manual_seed(70 + N + H + C + K)
    x = torch.randn(N, H, H, C, generator=g).to(DEV, torch.bfloat16)
    dy = torch.randn(N, H, H, K, generator=g).to(DEV, torch.bfloat16)
    dw0 = torch.randn(K, 3, 3, C, generator=g).to(DEV)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (K, C, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      padding=1).permute(0, 2, 3, 1) + beta * dw0
    outs = []
    for on in (1, 256, 0):  # 128 workgroups (default), 256 (conv_lin_wgrad_set(256): other XCD slot mapping), implicit
        dw = dw0.clone()
        L.conv_lin_wgrad_set(on)
        try:
            L.conv_wgrad(dy, x, dw, beta, 1, 1)
        finally:
            L.conv_lin_wgrad_set(1)
        assert _rel(dw, ref) < 2e-3, (on, _rel(dw, ref))
        outs.append(dw)
    assert _rel(outs[0], outs[2]) < 2e-3 and _rel(outs[1], outs[2]) < 2e-3
