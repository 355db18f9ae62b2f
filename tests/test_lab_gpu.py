"""Lab-extension kernels (dtg._lab, csrc/lab: NOT part of the production _C) against fp32 torch.

These are A/B candidates and negative results kept for the tools (tools/gemm_ab.py, gemm_sweep.py,
epi_gemm_ab.py, gemm5_ab.py): the 256x128 8-wave ring and the rest of the forced tile table
(gemm_forced*.hip), the 256x256 8-phase GEMM and its persistent form (gemm8.hip), the round-5 main-loop lab
(gemm5.hip) and the transposed fused BN dx + weight gradient
(bn_dxT_wgrad.hip).  Marked ``lab`` (not ``gpu``): the production GPU
suite does not load the lab extension.  Run with ``python -m pytest tests/test_lab_gpu.py -m lab`` on a GPU box
after ``python tools/build_ext.py --only lab``.
"""
import pytest
import torch
import torch.nn.functional as F

import dtg  # noqa: F401

pytestmark = pytest.mark.lab


def _lab():
    from dtg.ops._native import lab
    return lab()


def _gemm(cfg, A, a_kc, B, b_kc, bias=None, act=0, out_dtype=torch.bfloat16, split_k=1, aux=None, aux_mode=0):
    M = A.shape[0] if a_kc else A.shape[1]
    N = B.shape[0] if b_kc else B.shape[1]
    out = torch.empty(M, N, device=A.device, dtype=out_dtype)
    assert _lab().gemm_cfg(cfg, A, a_kc, B, b_kc, out, 1.0, 0.0, bias, act, split_k, aux, aux_mode)
    return out


def _rel(x, r):
    return ((x.float() - r).norm() / r.norm()).item()


@pytest.mark.parametrize("M,N,K", [(1024, 768, 512), (1000, 520, 328), (512, 256, 4096)])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False), (False, True)])
def test_gemm_big_tile_ring(M, N, K, a_kc, b_kc):
    """256x128 / 8-wave / 3-slot counted-vmcnt pipeline (forced configuration 8) vs fp32 torch."""
    torch.manual_seed(0)
    A = torch.randn((M, K) if a_kc else (K, M), device="cuda").bfloat16()
    B = torch.randn((N, K) if b_kc else (K, N), device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda")
    ref = (A.float() if a_kc else A.float().t()) @ (B.float().t() if b_kc else B.float()) + bias
    assert _rel(_gemm(8, A, a_kc, B, b_kc, bias=bias, out_dtype=torch.float32), ref) < 1e-2
    assert _rel(_gemm(8, A, a_kc, B, b_kc, bias=bias, out_dtype=torch.float32, split_k=3), ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(512, 512, 64), (512, 768, 128), (1024, 512, 192), (768, 1024, 1024),
                                   (1000, 600, 328), (256, 256, 512)])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False), (False, True)])
def test_gemm_8phase(M, N, K, a_kc, b_kc):
    """256x256 8-wave 8-phase kernel (forced configuration 99) vs fp32 torch: 1, 2, 3 and many K-tiles, ragged
    edges, all four operand layouts, bias + GELU epilogue, split-K slabs."""
    torch.manual_seed(0)
    A = torch.randn((M, K) if a_kc else (K, M), device="cuda").bfloat16()
    B = torch.randn((N, K) if b_kc else (K, N), device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda")
    ref = (A.float() if a_kc else A.float().t()) @ (B.float().t() if b_kc else B.float()) + bias
    assert _rel(_gemm(99, A, a_kc, B, b_kc, bias=bias, out_dtype=torch.float32), ref) < 1e-2
    refg = F.gelu(ref, approximate="tanh")
    assert _rel(_gemm(99, A, a_kc, B, b_kc, bias=bias, act=2), refg) < 2e-2
    if K >= 256:
        assert _rel(_gemm(99, A, a_kc, B, b_kc, bias=bias, out_dtype=torch.float32, split_k=2), ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 128), (8192, 2048, 768), (8192, 3072, 128), (6144, 3072, 192)])
@pytest.mark.parametrize("b_kc", [True, False])
def test_gemm_8phase_persistent(M, N, K, b_kc):
    """Persistent 256x256 8-phase kernel (forced configuration 98, gemm8.hip gemm8p_kernel) vs fp32 torch: one
    and many K-tiles per tile, a partial last round of tiles, both B layouts, and its four register epilogues
    (plain, bias, bias + GELU with GELU' saved, x saved GELU')."""
    torch.manual_seed(0)
    A = torch.randn(M, K, device="cuda").bfloat16()
    B = torch.randn((N, K) if b_kc else (K, N), device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda")
    ref = A.float() @ (B.float().t() if b_kc else B.float())
    assert _rel(_gemm(98, A, True, B, b_kc), ref) < 1e-2
    assert _rel(_gemm(98, A, True, B, b_kc, bias=bias), ref + bias) < 1e-2
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    pre = ref + bias
    assert _rel(_gemm(98, A, True, B, b_kc, bias=bias, act=2, aux=aux, aux_mode=3), F.gelu(pre, approximate="tanh")) < 2e-2
    p = pre.clone().requires_grad_()
    F.gelu(p, approximate="tanh").backward(torch.ones_like(p))
    assert _rel(aux, p.grad) < 2e-2
    sav = (torch.rand(M, N, device="cuda") + 0.5).bfloat16()
    assert _rel(_gemm(98, A, True, B, b_kc, aux=sav, aux_mode=4), ref * sav.float()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(2048, 768, 768), (1024, 1536, 3072), (512, 192, 64), (256, 384, 128)])
@pytest.mark.parametrize("sched", [0, 1])
def test_gemm5_matches_fp32_reference(M, N, K, sched):
    """Round-5 main-loop lab (csrc/lab/gemm5.hip, hipBLASLt-style VGPR-staged schedule): C = A B^T vs fp32, one,
    two and many K-tiles (the peeled tail iterations)."""
    torch.manual_seed(0)
    A = torch.randn(M, K, device="cuda").bfloat16()
    B = torch.randn(N, K, device="cuda").bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert _lab().gemm5(A, B, out, sched)
    assert _rel(out, A.float() @ B.float().t()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(2048, 768, 768), (1024, 1536, 3072), (256, 192, 64), (10240, 1536, 128)])
@pytest.mark.parametrize("epi", ["plain", "bias", "gelu_aux", "fp32"])
def test_gemm5p_matches_fp32_reference(M, N, K, epi):
    """Persistent v5 (one K-stream per workgroup across its tiles, register-bounced epilogue): several tiles per
    workgroup (10240 x 1536 is 320 tiles on 256 workgroups), one-K-tile tiles, and the epilogues: plain, + bias, + bias / GELU
    with GELU'(pre) saved, and the generic fp32 path."""
    torch.manual_seed(0)
    A = torch.randn(M, K, device="cuda").bfloat16()
    B = torch.randn(N, K, device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda")
    ref = A.float() @ B.float().t()
    out = torch.empty(M, N, device="cuda", dtype=torch.float32 if epi == "fp32" else torch.bfloat16)
    if epi == "plain" or epi == "fp32":
        assert _lab().gemm5p(A, B, out)
        assert _rel(out, ref) < 1e-2
    elif epi == "bias":
        assert _lab().gemm5p(A, B, out, bias)
        assert _rel(out, ref + bias) < 1e-2
    else:
        aux = torch.empty_like(out)
        assert _lab().gemm5p(A, B, out, bias, 2, aux, 3)
        pre = (ref + bias).requires_grad_()
        g = F.gelu(pre, approximate="tanh")
        assert _rel(out, g) < 2e-2
        g.backward(torch.ones_like(g))
        assert _rel(aux, pre.grad) < 2e-2


@pytest.mark.parametrize("C,CI", [(64, 256), (128, 256), (128, 512)])
def test_bn_dxT_wgrad_matches_fp32_reference(C, CI):
    """Transposed fused BN dx pass + weight gradient (csrc/lab/bn_dxT_wgrad.hip): dx = a dp + bx x + c per channel
    against fp32 torch, and wgrad += dx^T act on the kernel's bf16 dx; the row count is not a multiple of the grid,
    so the persistent workgroups end after different block counts."""
    g = torch.Generator().manual_seed(7)
    dev = torch.device("cuda")
    M = 8192 + 32 * 37
    dp, x = (torch.randn(M, C, generator=g).to(dev, torch.bfloat16) for _ in range(2))
    act = torch.rand(M, CI, generator=g).to(dev, torch.bfloat16)
    coef = torch.randn(3, C, generator=g).to(dev)
    w0 = torch.randn(C, CI, generator=g).to(dev)
    w = w0.clone()
    dx = _lab().bn_dxT_wgrad(dp, x, coef.view(-1), act, w)
    ref = coef[0] * dp.float() + coef[1] * x.float() + coef[2]
    assert _rel(dx, ref) < 1e-2
    assert _rel(w, w0 + dx.float().t() @ act.float()) < 1e-4
