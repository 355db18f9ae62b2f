"""BatchNorm statistics fused into the GEMM / implicit-GEMM epilogues (csrc/include/dtg/bn_epi.cuh)
against plain fp32 PyTorch references of the same math."""
import pytest
import torch
import torch.nn.functional as F

import dtg  # noqa: F401
from dtg.ops._native import lib

pytestmark = pytest.mark.gpu
SLOTS = 32


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _bn_stats(part, n):
    p = part.view(SLOTS, 2, n).sum(0)
    return p[0], p[1]


def _bwd_ref(g, x, mean, inv, gamma, beta):
    """dp = g * [relu(bn(x)) > 0], sum(dp), sum(dp * xhat) in fp32."""
    sc = gamma * inv
    sf = beta - mean * sc
    xf = x.float()
    dp = torch.where(xf * sc + sf > 0, g, torch.zeros_like(g))
    xhat = (xf - mean) * inv
    return dp, dp.sum(0), (dp * xhat).sum(0)


def _chan(n, dev, g):
    mean = (torch.randn(n, generator=g) * 0.3).to(dev)
    inv = (torch.rand(n, generator=g) + 0.5).to(dev)
    gamma = (torch.rand(n, generator=g) + 0.5).to(dev)
    beta = (torch.randn(n, generator=g) * 0.2).to(dev)
    return mean, inv, gamma, beta


# (M, N, K): skinny (256x64), 128x128, 64x256 and the 2-stage short-grid tiles, plus ragged M
@pytest.mark.parametrize("M,N,K", [(4096, 64, 256), (2048, 128, 512), (1024, 256, 64), (640, 512, 2048),
                                   (1000, 192, 128)])
def test_gemm_bn_fwd_stats(M, N, K):
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    a = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = torch.randn(N, K, generator=g).mul_(K ** -0.5).to(dev, torch.bfloat16)
    out, part = lib().gemm_bn(a, w, 1)
    ref = a.float() @ w.float().t()
    assert _rel(out, ref) < 1e-2
    s, q = _bn_stats(part, N)
    of = out.float()
    assert _rel(s, of.sum(0)) < 1e-3
    assert _rel(q, (of * of).sum(0)) < 1e-3


# the persistent streaming expand kernel (csrc/kernels/gemm_expand.hip: K in {64, 128, 256}, N % 256 == 0,
# M % 64 == 0, M * N >= 2^24): one, two and four 256-column slices, a row-block count that does not divide the grid
@pytest.mark.parametrize("M,N,K", [(65536, 256, 64), (32768, 512, 128), (64 * 1031, 256, 64), (16384, 1024, 64),
                                   (20480, 1024, 128), (16384, 1024, 256), (64 * 1031, 256, 256), (32768, 512, 256)])
def test_gemm_bn_expand_stats(M, N, K):
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(1)
    a = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = torch.randn(N, K, generator=g).mul_(K ** -0.5).to(dev, torch.bfloat16)
    L = lib()
    out, part = L.gemm_bn(a, w, 1)
    ref = a.float() @ w.float().t()
    assert _rel(out, ref) < 1e-2
    s, q = _bn_stats(part, N)
    of = out.float()
    assert _rel(s, of.sum(0)) < 1e-4
    assert _rel(q, (of * of).sum(0)) < 1e-4
    # identical outputs to the tiled 128x128 path (same bf16 rounding of the same fp32 sums up to MFMA order)
    L.gemm_bn_force_cfg(1)
    try:
        out1, part1 = L.gemm_bn(a, w, 1)
    finally:
        L.gemm_bn_force_cfg(0)
    assert _rel(out, out1) < 2e-3
    s1, q1 = _bn_stats(part1, N)
    assert _rel(s, s1) < 1e-3 and _rel(q, q1) < 1e-4


@pytest.mark.parametrize("M,N,K", [(4096, 64, 256), (2048, 128, 512), (1024, 256, 128), (1000, 192, 64)])
def test_gemm_bn_bwd_stats(M, N, K):
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(1)
    dy = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = torch.randn(K, N, generator=g).mul_(K ** -0.5).to(dev, torch.bfloat16)  # stored [K, N] (dgrad)
    x = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    mean, inv, gamma, beta = _chan(N, dev, g)
    dp, part = lib().gemm_bn(dy, w, 2, x, mean, inv, gamma, beta)
    gref = dy.float() @ w.float()
    dpr, sr, qr = _bwd_ref(gref, x, mean, inv, gamma, beta)
    assert _rel(dp, dpr) < 1e-2
    s, q = _bn_stats(part, N)
    assert _rel(s, sr) < 1e-2
    assert _rel(q, qr) < 1e-2
    # the same reduction with the relu mask read from packed bits (mode 3 without accumulation)
    dp3, part3 = lib().gemm_bn(dy, w, 3, x, mean, inv, gamma, beta, mask=_pack_mask(x, mean, inv, gamma, beta))
    assert _rel(dp3, dpr) < 1e-2
    s3, q3 = _bn_stats(part3, N)
    assert _rel(s3, sr) < 1e-2 and _rel(q3, qr) < 1e-2


def _pack_mask(x, mean, inv, gamma, beta):
    """uint8 [M, C/8]: bit k of byte j = relu mask of column 8j+k (gamma*xhat + beta > 0)."""
    m = ((x.float() - mean) * inv * gamma + beta > 0).to(torch.int32).view(x.shape[0], -1, 8)
    return (m << torch.arange(8, device=x.device, dtype=torch.int32)).sum(-1).to(torch.uint8).contiguous()


# the 1x1 / stride-2 projection from 256 channels on the streaming expand kernel with a row gather
# (gemm_expand.hip conv1x1_s2_expand_bn; M * K >= 2^24 and M % 64 == 0): against fp32 and the implicit-GEMM conv
@pytest.mark.parametrize("N,H,K", [(48, 56, 512), (96, 28, 1024), (2048, 8, 512)])
def test_conv1x1_s2_expand_bn(N, H, K):
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(3)
    C = 256
    x = torch.randn(N, H, H, C, generator=g).to(dev, torch.bfloat16)
    w = torch.randn(K, 1, 1, C, generator=g).mul_(C ** -0.5).to(dev, torch.bfloat16)
    L = lib()
    y, part = L.conv_fwd_bn(x, w, 2, 0)
    yr = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), stride=2).permute(0, 2, 3, 1)
    assert _rel(y, yr) < 1e-2
    yf = y.float().reshape(-1, K)
    s, q = _bn_stats(part, K)
    assert _rel(s, yf.sum(0)) < 1e-4 and _rel(q, (yf * yf).sum(0)) < 1e-4
    L.gemm_expand_s2_set(0)
    try:
        y0, part0 = L.conv_fwd_bn(x, w, 2, 0)
    finally:
        L.gemm_expand_s2_set(1)
    assert _rel(y, y0) < 2e-3
    s0, q0 = _bn_stats(part0, K)
    assert _rel(s, s0) < 1e-3 and _rel(q, q0) < 1e-4


@pytest.mark.parametrize("C,K,H,R,st,pad", [(64, 64, 14, 3, 1, 1), (64, 64, 16, 3, 1, 1), (128, 128, 14, 3, 2, 1),
                                            (64, 256, 8, 1, 1, 0),
                                            (256, 512, 7, 3, 1, 1)])
def test_conv_bn_fwd_and_dgrad_stats(C, K, H, R, st, pad):
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(2)
    N = 4
    x = torch.randn(N, C, H, H, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, R, R, generator=g).mul_((C * R * R) ** -0.5).to(dev, torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    L = lib()
    y, part = L.conv_fwd_bn(x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1), st, pad)
    yr = F.conv2d(x.float(), w.float(), stride=st, padding=pad).permute(0, 2, 3, 1)
    assert _rel(y, yr) < 1e-2
    yf = y.float().reshape(-1, K)
    s, q = _bn_stats(part, K)
    assert _rel(s, yf.sum(0)) < 1e-3 and _rel(q, (yf * yf).sum(0)) < 1e-3
    # dgrad through BN(x)->relu of the conv INPUT x (channels C)
    dy = torch.randn(yr.shape, generator=g).to(dev, torch.bfloat16).contiguous()
    mean, inv, gamma, beta = _chan(C, dev, g)
    xin = x.permute(0, 2, 3, 1).contiguous()
    dp, part = L.conv_dgrad_bn(dy, w.permute(0, 2, 3, 1).contiguous(), H, H, st, pad, xin.view(-1, C), mean, inv,
                               gamma, beta)
    gref = torch.nn.grad.conv2d_input((N, C, H, H), w.float(), dy.permute(0, 3, 1, 2).float(), stride=st,
                                      padding=pad).permute(0, 2, 3, 1).reshape(-1, C)
    dpr, sr, qr = _bwd_ref(gref, xin.view(-1, C), mean, inv, gamma, beta)
    assert _rel(dp.view(-1, C), dpr) < 1e-2
    s, q = _bn_stats(part, C)
    assert _rel(s, sr) < 1e-2 and _rel(q, qr) < 1e-2
    if st == 1 or R == 3:  # relu mask from packed bits (what the fused bottleneck passes)
        bits = _pack_mask(xin.view(-1, C), mean, inv, gamma, beta)
        dp3, part3 = L.conv_dgrad_bn(dy, w.permute(0, 2, 3, 1).contiguous(), H, H, st, pad, xin.view(-1, C), mean,
                                     inv, gamma, beta, bits=bits)
        assert _rel(dp3.view(-1, C), dpr) < 1e-2
        s3, q3 = _bn_stats(part3, C)
        assert _rel(s3, sr) < 1e-2 and _rel(q3, qr) < 1e-2


@pytest.mark.parametrize("N,H,grid,shift", [(2, 56, 1, 0.0), (3, 28, 1, 0.0), (40, 56, 1, 0.0), (40, 56, 192, 0.0),
                                             (5, 56, 1, 64.0)])
def test_conv_dgrad_bn_halo_64(N, H, grid, shift):
    """conv_dgrad_bn with packed mask bits for ResNet's stage-1 3x3 (64 -> 64, s1, p1) runs the direct halo-tile
    data gradient (csrc/kernels/conv_halo.hip, EPI 1): against the fp32 reference and against the implicit-GEMM
    dgrad (conv_halo_dgrad_set(0)) with the same epilogue.  N = 40 at 56x56 is 560 bands: every one of the 256
    persistent workgroups walks 2-3 bands through the double-buffered halo (the benchmark's b1024 walks ~56);
    grid 192 (conv_halo_dgrad_set(192)) gives uneven runs of 2 and 3 bands; shift 64 puts the BN input's mean at
    64x its standard deviation, where a raw-moment sum(dp * x) - mean * sum(dp) would cancel."""
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(40 + H + N)
    C = 64
    L = lib()
    w = (torch.randn(C, 3, 3, C, generator=g) * (9 * C) ** -0.5).to(dev, torch.bfloat16)
    dy = torch.randn(N, H, H, C, generator=g).to(dev, torch.bfloat16)
    xin = (torch.randn(N * H * H, C, generator=g) + shift).to(dev, torch.bfloat16)
    mean, inv, gamma, beta = _chan(C, dev, g)
    if shift:  # the BN's own batch statistics of xin
        mean = xin.float().mean(0)
        inv = xin.float().var(0, unbiased=False).add(1e-5).rsqrt()
    bits = _pack_mask(xin, mean, inv, gamma, beta)
    gref = torch.nn.grad.conv2d_input((N, C, H, H), w.float().permute(0, 3, 1, 2), dy.permute(0, 3, 1, 2).float(),
                                      padding=1).permute(0, 2, 3, 1).reshape(-1, C)
    dpr, sr, qr = _bwd_ref(gref, xin, mean, inv, gamma, beta)
    outs = []
    for halo in (grid, 0):
        L.conv_halo_dgrad_set(halo)
        try:
            dp, part = L.conv_dgrad_bn(dy, w, H, H, 1, 1, xin, mean, inv, gamma, beta, bits=bits)
        finally:
            L.conv_halo_dgrad_set(1)
        assert _rel(dp.view(-1, C), dpr) < 1e-2
        s, q = _bn_stats(part, C)
        assert _rel(s, sr) < 1e-2 and _rel(q, qr) < 1e-2
        outs.append((dp.float(), s, q))
    assert _rel(outs[0][0], outs[1][0]) < 5e-3
    assert _rel(outs[0][1], outs[1][1]) < 5e-3 and _rel(outs[0][2], outs[1][2]) < 5e-3


@pytest.mark.parametrize("res", [False, True])
def test_bn_part_matches_unfused(res):
    """bn_fwd_part / bn_bwd_part (statistics from an epilogue) equal bn_fwd_train / bn_bwd."""
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(3)
    M, K, N = 3136, 128, 256
    a = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = torch.randn(N, K, generator=g).mul_(K ** -0.5).to(dev, torch.bfloat16)
    L = lib()
    y, part = L.gemm_bn(a, w, 1)
    gamma = (torch.rand(N, generator=g) + 0.5).to(dev)
    beta = (torch.randn(N, generator=g) * 0.1).to(dev)
    r = torch.randn(M, N, generator=g).to(dev, torch.bfloat16) if res else None
    rm0, rv0 = torch.zeros(N, device=dev), torch.ones(N, device=dev)
    rm1, rv1 = rm0.clone(), rv0.clone()
    o0, m0, i0 = L.bn_fwd_train(y, r, gamma, beta, rm0, rv0, 0.1, 1e-5, True)
    o1, m1, i1 = L.bn_fwd_part(y, part, r, gamma, beta, rm1, rv1, 0.1, 1e-5, True)
    assert _rel(m1, m0) < 1e-4 and _rel(i1, i0) < 1e-4
    assert _rel(rm1, rm0) < 1e-4 and _rel(rv1, rv0) < 1e-4
    assert _rel(o1, o0) < 1e-2
    # backward: reference bn_bwd on the unmasked gradient vs bn_bwd_part on (masked dp, reduced here)
    do = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    dx0, _, dg0, db0 = L.bn_bwd(do, o0, y, gamma, m0, i0, True, False, None, None)
    dp = torch.where(o0 > 0, do, torch.zeros_like(do))
    xhat = (y.float() - m0) * i0
    pr = torch.zeros(SLOTS, 2, N, device=dev)
    pr[0, 0] = dp.float().sum(0)
    pr[0, 1] = (dp.float() * xhat).sum(0)
    dx1, _, dg1, db1 = L.bn_bwd_part(dp, y, pr.view(-1), gamma, m0, i0, False, None, None)
    assert _rel(dg1, dg0) < 1e-3 and _rel(db1, db0) < 1e-3
    assert _rel(dx1, dx0) < 1e-2


def test_bn_fwd2_part_matches_two_passes():
    """relu(bn3(y3) + bn_d(yd)) in one pass == bn_d applied, then bn3 with the residual."""
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(4)
    M, K, N = 2048, 128, 256
    L = lib()
    a = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w3 = torch.randn(N, K, generator=g).mul_(K ** -0.5).to(dev, torch.bfloat16)
    wd = torch.randn(N, K, generator=g).mul_(K ** -0.5).to(dev, torch.bfloat16)
    ch = lambda: ((torch.rand(N, generator=g) + 0.5).to(dev), (torch.randn(N, generator=g) * 0.1).to(dev))  # noqa
    (g3, b3), (gd, bd) = ch(), ch()
    outs = []
    for fused in (False, True):
        y3, p3 = L.gemm_bn(a, w3, 1)
        yd, pd = L.gemm_bn(a, wd, 1)
        rm3, rv3, rmd, rvd = (torch.zeros(N, device=dev), torch.ones(N, device=dev), torch.zeros(N, device=dev),
                              torch.ones(N, device=dev))
        if fused:
            o, m3, i3, md, idd = L.bn_fwd2_part(y3, p3, g3, b3, rm3, rv3, yd, pd, gd, bd, rmd, rvd, 0.1, 1e-5)
        else:
            idn, md, idd = L.bn_fwd_part(yd, pd, None, gd, bd, rmd, rvd, 0.1, 1e-5, False)
            o, m3, i3 = L.bn_fwd_part(y3, p3, idn, g3, b3, rm3, rv3, 0.1, 1e-5, True)
        outs.append((o, m3, i3, md, idd, rm3, rv3, rmd, rvd))
    for x, y in zip(outs[1], outs[0]):
        assert _rel(x, y) < 1e-2


def _pack_bits(t):
    b = (t.float() > 0).to(torch.uint8).view(t.shape[0], -1, 8)
    w = (1 << torch.arange(8, device=t.device, dtype=torch.int32)).to(torch.uint8)
    return (b * w).sum(-1).to(torch.uint8)


def test_mode3_packed_mask_bits():
    """bn_fwd_part emits the packed relu mask of its output; gemm_bn mode 3 gives identical results with
    the packed mask and with the bf16 tensor it was packed from (and accumulates into `out`)."""
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(5)
    M, K, N = 1536, 128, 256
    L = lib()
    a = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = torch.randn(N, K, generator=g).mul_(K ** -0.5).to(dev, torch.bfloat16)
    y, part = L.gemm_bn(a, w, 1)
    res = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    gamma, beta = (torch.rand(N, generator=g) + 0.5).to(dev), (torch.randn(N, generator=g) * 0.1).to(dev)
    bits = torch.empty(M, N // 8, device=dev, dtype=torch.uint8)
    out, m, i = L.bn_fwd_part(y, part, res, gamma, beta, torch.zeros(N, device=dev), torch.ones(N, device=dev), 0.1,
                              1e-5, True, bits=bits)
    assert torch.equal(bits, _pack_bits(out))
    dy = torch.randn(M, 64, generator=g).to(dev, torch.bfloat16)
    w1 = torch.randn(64, N, generator=g).mul_(0.125).to(dev, torch.bfloat16)
    acc0 = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    r = []
    for mask in (out, bits):
        o = acc0.clone()
        dp, q = L.gemm_bn(dy, w1, 3, y, m, i, gamma, beta, mask=mask, out=o)
        r.append((o, q))
    assert torch.equal(r[0][0], r[1][0]) and torch.allclose(r[0][1], r[1][1], rtol=1e-4, atol=1e-3)
    ref = torch.where(out.float() > 0, dy.float() @ w1.float() + acc0.float(), torch.zeros(M, N, device=dev))
    assert _rel(r[1][0], ref) < 1e-2


# ---- BN backward dx pass fused with the producing conv's weight gradient (bn_dx_wgrad.hip) ---------------
@pytest.mark.parametrize("dual", [False, True])
@pytest.mark.parametrize("gdtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,CI", [(256, 64), (512, 128)])
def test_bn_dx_wgrad_fused(dual, gdtype, C, CI):
    """BN backward dx pass fused with dW += dx^T act (csrc/kernels/bn_dx_wgrad.hip): dx equal to the unfused pass
    up to fma contraction, dW against fp32 torch on the fused pass's bf16 dx, accumulated (beta = 1) into a fp32 or
    bf16 gradient."""
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(3)
    M = 8192 + 32 * 37  # not a multiple of the grid: workgroups end after different block counts
    L = lib()
    assert L.bn_dx_wgrad_ok(M, C, CI) and not L.bn_dx_wgrad_ok(M, C, CI // 2 + 8)
    assert not L.bn_dx_wgrad_ok(M + 8, C, CI)
    dp = torch.randn(M, C, generator=g).to(dev, torch.bfloat16)
    x = torch.randn(M, C, generator=g).to(dev, torch.bfloat16)
    x2 = torch.randn(M, C, generator=g).to(dev, torch.bfloat16)
    act = torch.rand(M, CI, generator=g).to(dev, torch.bfloat16)

    def chan():
        mean, inv, gamma, _ = _chan(C, dev, g)
        part = torch.zeros(SLOTS, 2, C, device=dev)
        part[0, 0] = torch.randn(C, generator=g).to(dev) * 10
        part[0, 1] = torch.randn(C, generator=g).to(dev) * 10
        return mean, inv, gamma, part.view(-1)

    m1, i1, g1, p1 = chan()
    m2, i2, g2, p2 = chan()
    w0 = (torch.randn(C, CI, generator=g) * 0.1).to(dev, gdtype)
    wgrad = w0.clone()
    z = lambda: torch.zeros(C, device=dev)  # noqa: E731
    if dual:
        ref = L.bn_bwd2_part(dp, x, p1.clone(), g1, m1, i1, z(), z(), x2, p2.clone(), g2, m2, i2, z(), z())
        out = L.bn_bwd2_part(dp, x, p1.clone(), g1, m1, i1, z(), z(), x2, p2.clone(), g2, m2, i2, z(), z(),
                             wact=act, wgrad=wgrad)
        assert _rel(out[1], ref[1]) < 1e-3  # the same fp32 expression up to fma contraction, rounded to bf16
    else:
        ref = L.bn_bwd_part(dp, x, p1.clone(), g1, m1, i1, False, z(), z())
        out = L.bn_bwd_part(dp, x, p1.clone(), g1, m1, i1, False, z(), z(), wact=act, wgrad=wgrad)
    assert _rel(out[0], ref[0]) < 1e-3
    want = w0.float() + out[0].float().t() @ act.float()
    assert _rel(wgrad, want) < (1e-4 if gdtype == torch.float32 else 5e-3)


def test_bn_dx_wgrad_fused_two_weights():
    """Dual form with the projection shortcut's weight gradient too: dW += dx^T act, dW2 += dx2^T act2."""
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(5)
    M, C, CI = 8192, 256, 64
    L = lib()
    dp, x, x2 = (torch.randn(M, C, generator=g).to(dev, torch.bfloat16) for _ in range(3))
    act, act2 = (torch.rand(M, CI, generator=g).to(dev, torch.bfloat16) for _ in range(2))
    chans = []
    for _ in range(2):
        mean, inv, gamma, _ = _chan(C, dev, g)
        part = torch.zeros(SLOTS, 2, C, device=dev)
        part[0] = torch.randn(2, C, generator=g).to(dev) * 10
        chans.append((mean, inv, gamma, part.view(-1)))
    (m1, i1, g1, p1), (m2, i2, g2, p2) = chans
    z = lambda: torch.zeros(C, device=dev)  # noqa: E731
    w, w2 = torch.zeros(C, CI, device=dev), torch.zeros(C, CI, device=dev)
    ref = L.bn_bwd2_part(dp, x, p1.clone(), g1, m1, i1, z(), z(), x2, p2.clone(), g2, m2, i2, z(), z())
    out = L.bn_bwd2_part(dp, x, p1.clone(), g1, m1, i1, z(), z(), x2, p2.clone(), g2, m2, i2, z(), z(),
                         wact=act, wgrad=w, wact2=act2, wgrad2=w2)
    assert _rel(out[0], ref[0]) < 1e-3 and _rel(out[1], ref[1]) < 1e-3
    assert _rel(w, out[0].float().t() @ act.float()) < 1e-4
    assert _rel(w2, out[1].float().t() @ act2.float()) < 1e-4
