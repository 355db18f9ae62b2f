"""Numerics of every hand-written HIP kernel against a plain PyTorch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

import dtg  # noqa: F401
from dtg import ops
from dtg.ops import optim_kernels as K

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_native_loaded():
    lib = ops.lib()
    assert hasattr(lib, "gemm") and hasattr(lib, "bn_fwd_train")


# ---------------------------------------------------------------- GEMM
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 512), (200, 136, 96), (64, 1000, 2048)])
def test_gemm_layouts(a_kc, b_kc, M, N, K):
    if (not a_kc and M % 8) or (not b_kc and N % 8):
        pytest.skip("MN-contiguous operand needs multiple of 8")
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K)
    A = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    B = torch.randn(K, N, generator=g).to(DEV, torch.bfloat16)
    ref = A.float() @ B.float()
    a = A if a_kc else A.t().contiguous()          # [M,K] or [K,M]
    b = B.t().contiguous() if b_kc else B          # [N,K] or [K,N]
    out = ops.gemm(a, a_kc, b, b_kc, out_dtype=torch.float32, split_k=1)
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-5, _rel(out, ref)


def test_gemm_identity_asymmetric():
    # A = I with an asymmetric B catches a transposed C write
    M = N = K = 128
    A = torch.eye(M, device=DEV, dtype=torch.bfloat16)
    B = (torch.arange(K * N, device=DEV).reshape(K, N) % 251).to(torch.bfloat16)
    out = ops.gemm(A, True, B, False, out_dtype=torch.float32)
    assert torch.equal(out, B.float())


def test_gemm_splitk_bias_act():
    g = torch.Generator(device="cpu").manual_seed(3)
    M, N, K = 96, 64, 8192
    A = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    W = torch.randn(N, K, generator=g).to(DEV, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(DEV)
    ref = torch.relu(A.float() @ W.float().t() + bias)
    for sk in (1, 4, 0):
        out = ops.gemm(A, True, W, True, bias=bias, act="relu", split_k=sk, out_dtype=torch.float32)
        assert _rel(out, ref) < 1e-5
    out = ops.gemm(A, True, W, True, bias=bias, act="relu")
    assert out.dtype == torch.bfloat16 and _rel(out, ref) < 1e-2


def test_gemm_beta_accumulate():
    g = torch.Generator(device="cpu").manual_seed(4)
    A = torch.randn(256, 128, generator=g).to(DEV, torch.bfloat16)
    B = torch.randn(128, 192, generator=g).to(DEV, torch.bfloat16)
    C = torch.randn(256, 192, generator=g).to(DEV)
    ref = 0.5 * (A.float() @ B.float()) + 2.0 * C
    ops.gemm(A, True, B, False, out=C, alpha=0.5, beta=2.0)
    assert _rel(C, ref) < 1e-5


def test_linear_autograd():
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(48, 256, generator=g).to(DEV, torch.bfloat16).requires_grad_()
    w = torch.randn(96, 256, generator=g).mul(0.05).to(DEV, torch.bfloat16).requires_grad_()
    b = torch.randn(96, generator=g).to(DEV).requires_grad_()
    for act in (None, "relu", "gelu"):
        y = ops.linear(x, w, b, act)
        gy = torch.randn_like(y)
        y.backward(gy)
        xr, wr, br = x.detach().float().requires_grad_(), w.detach().float().requires_grad_(), b.detach().clone().requires_grad_()
        yr = F.linear(xr, wr, br)
        yr = F.relu(yr) if act == "relu" else (F.gelu(yr, approximate="tanh") if act == "gelu" else yr)
        yr.backward(gy.float())
        assert _rel(y, yr) < 1e-2
        assert _rel(x.grad, xr.grad) < 2e-2
        assert _rel(w.grad, wr.grad) < 2e-2
        assert _rel(b.grad, br.grad) < 1e-2
        x.grad = w.grad = b.grad = None


# ---------------------------------------------------------------- BatchNorm
@pytest.mark.parametrize("C,HW", [(64, 56), (256, 14), (2048, 7), (96, 9)])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_bn_act(C, HW, res, relu):
    g = torch.Generator(device="cpu").manual_seed(C + HW)
    N = 8
    x = (torch.randn(N, C, HW, HW, generator=g) * 2 + 0.5).to(DEV, torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()
    r = torch.randn(N, C, HW, HW, generator=g).to(DEV, torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_() if res else None
    w = (torch.rand(C, generator=g) + 0.5).to(DEV).requires_grad_()
    b = torch.randn(C, generator=g).to(DEV).requires_grad_()
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    y = ops.batch_norm_act(x, w, b, rm, rv, True, 0.1, 1e-5, r, relu)
    gy = torch.randn(y.shape, generator=g).to(DEV, torch.bfloat16)
    y.backward(gy)
    xr = x.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if res else None
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    rm2, rv2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    yr = F.batch_norm(xr, rm2, rv2, wr, br, True, 0.1, 1e-5)
    if res:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    yr.backward(gy.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 1e-2
    assert _rel(b.grad, br.grad) < 1e-2
    if res:
        assert _rel(r.grad, rr.grad) < 1e-2
    assert _rel(rm, rm2) < 1e-3 and _rel(rv, rv2) < 1e-3
    # inference path uses running stats
    yi = ops.batch_norm_act(x.detach(), w.detach(), b.detach(), rm, rv, False, 0.1, 1e-5,
                            r.detach() if res else None, relu)
    yir = F.batch_norm(x.detach().float(), rm, rv, w.detach(), b.detach(), False, 0.1, 1e-5)
    if res:
        yir = yir + r.detach().float()
    if relu:
        yir = F.relu(yir)
    assert _rel(yi, yir) < 1e-2


# ---------------------------------------------------------------- softmax xent
@pytest.mark.parametrize("B,V,dt", [(256, 1000, torch.bfloat16), (64, 10, torch.float32), (40, 30522, torch.bfloat16),
                                    (48, 30528, torch.bfloat16)])
def test_softmax_xent(B, V, dt):
    """V % 8 == 0 bf16 rows take the 16-byte vector kernels; the backward reads the upstream gradient
    (here 0.5: the loss is scaled) on the device."""
    g = torch.Generator(device="cpu").manual_seed(B + V)
    logits = (torch.randn(B, V, generator=g) * 3).to(DEV, dt).requires_grad_()
    labels = torch.randint(0, V, (B,), generator=g).to(DEV)
    labels[::7] = -1  # ignored rows
    nv = int((labels >= 0).sum())
    loss = ops.softmax_cross_entropy(logits, labels, num_valid=nv)
    (loss * 0.5).backward()
    lr_ = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(lr_, labels, ignore_index=-1, reduction="sum") / nv
    (ref * 0.5).backward()
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1, abs(ref.item()))
    assert _rel(logits.grad, lr_.grad) < 1e-2


# ---------------------------------------------------------------- optimizer applies
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kind", ["sgd", "momentum", "adagrad", "adam"])
def test_optim_apply(kind, gdt):
    n = 100003  # odd: exercises the scalar tail
    g0 = torch.Generator(device="cpu").manual_seed(11)
    w = torch.randn(n, generator=g0)
    grad = torch.randn(n, generator=g0).to(gdt)
    hyper = torch.tensor([0.05, 3.0])
    st = [torch.rand(n, generator=g0) for _ in range(2)]
    res = {}
    for dev in ("cpu", DEV):
        W = w.clone().to(dev)
        G = grad.clone().to(dev)
        H = hyper.to(dev)
        S = [s.clone().to(dev) for s in st]
        mir = torch.empty(n, dtype=torch.bfloat16, device=dev)
        if kind == "sgd":
            K.sgd(W, G, H, mir, wd=0.01, gscale=0.5, zero_grad=True)
        elif kind == "momentum":
            K.momentum(W, G, S[0], H, mir, mu=0.9, wd=1e-4, nesterov=True, gscale=0.5, zero_grad=True)
        elif kind == "adagrad":
            K.adagrad(W, G, S[0], H, mir, eps=0.0, gscale=0.5, zero_grad=True)
        else:
            K.adam(W, G, S[0], S[1], H, mir, wd=0.01, gscale=0.5, zero_grad=True)
        res[dev] = (W.cpu(), mir.cpu(), G.cpu(), [s.cpu() for s in S])
    (wc, mc, gc, sc), (wg, mg, gg, sg) = res["cpu"], res[DEV]
    assert torch.allclose(wg, wc, rtol=1e-5, atol=1e-6)
    assert torch.equal(mg, wg.to(torch.bfloat16))
    assert gg.abs().sum() == 0
    for a, b in zip(sg, sc):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)


def test_axpby():
    a = torch.randn(1001, device=DEV)
    g = torch.randn(1001, device=DEV, dtype=torch.bfloat16)
    ref = 0.5 * a + 2.0 * g.float()
    K.axpby(a, g, 0.5, 2.0)
    assert torch.allclose(a, ref, atol=1e-6)


@pytest.mark.parametrize("shape,k,s,pad", [((4, 64, 112, 112), 3, 2, 1), ((8, 32, 28, 28), 2, 2, 0),
                                           ((2, 16, 15, 13), 3, 2, 1)])
def test_maxpool_fwd_bwd(shape, k, s, pad):
    from dtg.ops.pool import max_pool2d
    torch.manual_seed(0)
    x = torch.randn(shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xr = x.float().requires_grad_()
    xd = x.clone().requires_grad_()
    y = max_pool2d(xd, k, s, pad)
    yr = torch.nn.functional.max_pool2d(xr, k, s, pad)
    assert torch.equal(y.float(), yr)
    dy = torch.randn(yr.shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    yr.backward(dy.float())
    assert torch.allclose(xd.grad.float(), xr.grad, atol=1e-2, rtol=1e-2)


def test_global_avg_pool():
    from dtg.ops.pool import global_avg_pool
    torch.manual_seed(0)
    x = torch.randn(8, 2048, 7, 7, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xd = x.clone().requires_grad_()
    y = global_avg_pool(xd)
    assert torch.allclose(y.float(), x.float().mean(dim=(2, 3)), atol=1e-2)
    dy = torch.randn(8, 2048, device="cuda").bfloat16()
    y.backward(dy)
    assert torch.allclose(xd.grad.float(), (dy.float() / 49)[:, :, None, None].expand(8, 2048, 7, 7), atol=1e-3)


@pytest.mark.parametrize("cin,cout,k,stride,pad,hw", [(1, 32, 5, 1, 2, 28), (32, 64, 5, 1, 2, 14), (3, 64, 7, 2, 3, 32),
                                                     (16, 24, 3, 2, 1, 15)])
def test_conv_im2col_bias_relu(cin, cout, k, stride, pad, hw):
    from dtg.ops.conv import conv2d_bias_act
    torch.manual_seed(0)
    x = torch.randn(4, cin, hw, hw, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, k, k, device="cuda") * 0.1).bfloat16()
    b = torch.randn(cout, device="cuda")
    xd, wd, bd = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    xr, wr, br = x.float().requires_grad_(), w.float().requires_grad_(), b.clone().requires_grad_()
    y = conv2d_bias_act(xd, wd, bd, stride, pad, "relu")
    yr = F.relu(F.conv2d(xr, wr, br, stride, pad))
    rel = lambda a, r: ((a.float() - r).norm() / (r.norm() + 1e-12)).item()  # noqa: E731
    assert rel(y, yr) < 1e-2
    dy = torch.randn_like(yr)
    y.backward(dy.bfloat16())
    yr.backward(dy)
    assert rel(xd.grad, xr.grad) < 2e-2
    assert rel(wd.grad, wr.grad) < 2e-2
    assert rel(bd.grad, br.grad) < 2e-2


def test_mnist_cnn_trains_on_gpu():
    from dtg.models.mnist import MnistCNN, synthetic_mnist
    from dtg.parallel import MirroredStrategy
    from dtg.optim import FusedSGD
    torch.manual_seed(0)
    s = MirroredStrategy()
    with s.scope():
        m = MnistCNN().to(s.device)
    tr = s.distribute(m, lambda f: FusedSGD(f, lr=0.01, momentum=0.9))
    for i in range(60):
        x, y = synthetic_mnist(128, s.device, seed=i)
        tr.step(lambda: ops.softmax_cross_entropy(m(x), y))
    x, y = synthetic_mnist(512, s.device, seed=999)
    with torch.no_grad():
        acc = (m(x).argmax(1) == y).float().mean().item()
    assert acc > 0.9, acc


@pytest.mark.parametrize("M,N,K,a_kc,b_kc", [(64, 256, 8192, False, False), (64, 576, 4096, False, False),
                                             (48, 300, 512, True, True), (64, 1024, 256, True, False)])
def test_gemm_short_m_tiles(M, N, K, a_kc, b_kc):
    """M <= 64 (64-channel weight gradients) runs on 64x256 tiles, with and without split-K."""
    torch.manual_seed(0)
    A = torch.randn((M, K) if a_kc else (K, M), device="cuda").bfloat16()
    B = torch.randn((N, K) if b_kc else (K, N), device="cuda").bfloat16()
    ref = (A.float() if a_kc else A.float().t()) @ (B.float().t() if b_kc else B.float())
    for sk in (1, 0):
        out = ops.gemm(A, a_kc, B, b_kc, out_dtype=torch.float32, split_k=sk)
        assert ((out - ref).norm() / ref.norm()).item() < 1e-2, sk


