"""End-to-end ResNet training on the GPU through dtg's kernels."""
import pytest
import torch

import dtg  # noqa: F401
from dtg import ops
from dtg.ops import conv as conv_ops
from dtg.models import resnet
from dtg.parallel import FlatParams, DataParallel
from dtg.optim import FusedSGD

pytestmark = pytest.mark.gpu


def test_resnet_tiny_loss_decreases():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet.resnet18_like_tiny(10).to(dev).to(memory_format=torch.channels_last)
    flat = FlatParams(model)
    dp = DataParallel(flat)
    opt = FusedSGD(flat, lr=0.05, momentum=0.9)
    x, y = resnet.synthetic_batch(32, dev, torch.bfloat16, 32, 10, seed=1)
    losses = []
    for _ in range(30):
        loss = ops.softmax_cross_entropy(model(x), y)
        loss.backward()
        dp.finish()
        opt.step(dp.grad_scale)
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < 0.5 * losses[0], losses


@pytest.mark.parametrize("cin,width,stride", [(64, 64, 1), (256, 64, 1), (256, 128, 2), (512, 128, 1)])
@pytest.mark.parametrize("flat", [False, True])
@pytest.mark.parametrize("bn_fuse", [True, False])
def test_fused_bottleneck_matches_layerwise(cin, width, stride, flat, bn_fuse, monkeypatch):
    """The hand-written bottleneck backward (with and without BN statistics fused into the conv
    epilogues) equals the layer-by-layer autograd path."""
    from dtg.models.resnet import Bottleneck
    from dtg.models import resnet_fused
    monkeypatch.setattr(resnet_fused, "_FUSE", bn_fuse)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    blocks = []
    for fused in (False, True):
        torch.manual_seed(0)
        b = Bottleneck(cin, width, stride).to(dev).to(memory_format=torch.channels_last)
        for bn in (b.c1.bn, b.c2.bn, b.c3.bn):
            bn.weight.data.uniform_(0.5, 1.5)  # c3 is zero-initialised: make the branch matter
        b.fused = fused
        b.train()
        if flat:
            FlatParams(b)
        else:
            for p in b.parameters():
                if p.dim() > 1:
                    p.data = p.data.to(torch.bfloat16)
        blocks.append(b)
    g = torch.Generator(device="cpu").manual_seed(1)
    x0 = torch.randn(4, cin, 14, 14, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = None
    outs, grads = [], []
    for b in blocks:
        x = x0.clone().requires_grad_()
        y = b(x)
        if gy is None:
            gy = torch.randn(y.shape, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y.backward(gy)
        outs.append(y.float())
        grads.append([x.grad.float()] + [p.grad.float().clone() for p in b.parameters()])
    rel = lambda a, b: ((a - b).norm() / (b.norm() + 1e-12)).item()  # noqa: E731
    assert rel(outs[1], outs[0]) < 1e-2
    for ga, gb in zip(grads[1], grads[0]):
        assert rel(ga, gb) < 3e-2, rel(ga, gb)
    for ba, bb in zip(blocks[1].buffers(), blocks[0].buffers()):
        assert torch.allclose(ba, bb, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("sub2", [True, False])
def test_bn3_link_chain_matches_unlinked(sub2, monkeypatch):
    """Three chained blocks (projection, identity, strided projection).  With the BN3 link each block's
    BN3 statistics are reduced by the NEXT block's last dgrad epilogue (mode 3); without it, by the
    block's own reduction pass.  Both runs share the same forward bit for bit (the link only changes
    backward), so their gradients must agree to summation-order noise.  (Against the layer-wise
    reference a 3-block chain differs by a few % through ReLU-mask flips of near-zero activations,
    which is why the per-block test above is the fused-vs-layerwise check.)"""
    from dtg.models.resnet import Bottleneck
    from dtg.models import resnet_fused
    monkeypatch.setattr(resnet_fused, "_FUSE", True)
    monkeypatch.setattr(resnet_fused, "_SUB2", sub2)  # strided projection dgrad: even rows only (no zero fill)
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(1)
    x0 = torch.randn(4, 64, 16, 16, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = None
    outs, grads = [], []
    for link in (False, True):
        monkeypatch.setattr(resnet_fused, "_LINK", link)
        torch.manual_seed(0)
        bl = torch.nn.Sequential(Bottleneck(64, 64, 1), Bottleneck(256, 64, 1), Bottleneck(256, 128, 2))
        bl = bl.to(dev).to(memory_format=torch.channels_last)
        for b in bl:
            for bn in (b.c1.bn, b.c2.bn, b.c3.bn):
                bn.weight.data.uniform_(0.5, 1.5)
        bl.train()
        FlatParams(bl)
        x = x0.clone().requires_grad_()
        y = bl(x)
        if gy is None:
            gy = torch.randn(y.shape, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y.backward(gy)
        outs.append(y.float())
        grads.append([x.grad.float()] + [p.grad.float().clone() for p in bl.parameters()])
    rel = lambda a, b: ((a - b).norm() / (b.norm() + 1e-12)).item()  # noqa: E731
    assert rel(outs[1], outs[0]) == 0.0
    errs = [rel(ga, gb) for ga, gb in zip(grads[1], grads[0])]
    assert max(errs) < 1e-2, errs


def test_resnet50_step_matches_reference_direction():
    """One ResNet-50 step on a small batch: finite loss, grads flow into the flat buffer."""
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
    flat = FlatParams(model)
    x, y = resnet.synthetic_batch(4, dev, torch.bfloat16, 224, 1000)
    loss = ops.softmax_cross_entropy(model(x), y)
    loss.backward()
    g = flat.groups["compute"].grad
    assert torch.isfinite(loss).item()
    assert torch.isfinite(g.float()).all().item() and g.float().abs().sum().item() > 0


def test_wgrad_side_stream_matches_main_stream(monkeypatch):
    """parallel/overlap.py: weight gradients on the side stream (opt-in) give the same gradients as on the
    main stream, and backward() returns with them finished (the end-of-backward join)."""
    from dtg.models.resnet import Bottleneck
    from dtg.models import resnet_fused
    from dtg.parallel import overlap
    monkeypatch.setattr(resnet_fused, "_FUSE", True)
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(2)
    x0 = torch.randn(8, 64, 16, 16, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy, grads = None, []
    was = overlap._ON
    try:
        for side in (False, True):
            overlap.set_enabled(side)
            torch.manual_seed(0)
            bl = torch.nn.Sequential(Bottleneck(64, 64, 1), Bottleneck(256, 64, 1), Bottleneck(256, 128, 2))
            bl = bl.to(dev).to(memory_format=torch.channels_last)
            bl.train()
            FlatParams(bl)
            x = x0.clone().requires_grad_()
            y = bl(x)
            if gy is None:
                gy = torch.randn(y.shape, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
            y.backward(gy)
            assert not overlap._pending  # joined by the end-of-backward callback
            grads.append([x.grad.float()] + [p.grad.float().clone() for p in bl.parameters()])
    finally:
        overlap.set_enabled(was)
    rel = lambda a, b: ((a - b).norm() / (b.norm() + 1e-12)).item()  # noqa: E731
    errs = [rel(ga, gb) for ga, gb in zip(grads[1], grads[0])]
    assert max(errs) < 1e-2, errs


@pytest.mark.parametrize("size", [64, 60])
@pytest.mark.parametrize("pairs", ["1", "0"])
@pytest.mark.parametrize("flat", [False, True])
def test_fused_stem_matches_unfused(flat, pairs, size, monkeypatch):
    """conv7x7/2 -> BN -> ReLU -> maxpool3x3/2 as one node (csrc/kernels/stem.hip: BN statistics from the
    conv epilogue, BN+ReLU+pool in one pass, gather-form backward) equals the op-by-op path: output,
    running statistics and the conv / gamma / beta gradients.  size 64 (conv output 32x32, a multiple of
    4 rows) runs the LDS-banded backward, size 60 (30x30) the per-pixel gather form."""
    from dtg.models.layers import ConvBN
    from dtg.models import resnet_fused
    from dtg.ops.pool import max_pool2d
    monkeypatch.setattr(conv_ops, "_PAIRS", pairs != "0")  # pixel-pair (ops/conv.py stem_pairs) or 8-channel stem conv
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(4, 3, size, size, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for fused in (False, True):
        monkeypatch.setattr(resnet_fused, "_STEM", fused)
        torch.manual_seed(0)
        stem = ConvBN(3, 64, 7, 2, 3).to(dev)
        stem.bn.weight.data.uniform_(0.5, 1.5)
        stem.bn.bias.data.uniform_(-0.3, 0.3)
        if flat:
            FlatParams(stem)
        else:
            stem.conv.weight.data = stem.conv.weight.data.to(torch.bfloat16)
        stem.train()
        assert resnet_fused.stem_ok(stem, x) == fused
        y = resnet_fused.stem_pool(stem, x) if fused else max_pool2d(stem(x), 3, 2, 1)
        gy = torch.randn(y.shape, generator=g.manual_seed(7)).to(dev)
        (y.float() * gy).sum().backward()
        res.append([t.detach().float().clone() for t in (y, stem.bn.running_mean, stem.bn.running_var,
                                                          stem.conv.weight.grad, stem.bn.weight.grad,
                                                          stem.bn.bias.grad)])
    names = ["out", "running_mean", "running_var", "dW", "dgamma", "dbeta"]
    for name, a, b in zip(names, *res):
        assert a.shape == b.shape, name
        err = ((a - b).norm() / (a.norm() + 1e-6)).item()
        assert err < 2e-2, (name, err)


@pytest.mark.gpu
@pytest.mark.parametrize("size", [64, 60])
def test_stem_pooled_statistics_pass(size, monkeypatch):
    """The stem backward's BN statistics pass at pooled resolution (the forward saves y at each window's argmax,
    stem_bwd_pooled_stats_kernel) gives the gradients of the pixel-resolution gather pass up to summation order."""
    from dtg.models.layers import ConvBN
    from dtg.models import resnet_fused
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(4, 3, size, size, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for yam in (False, True):
        monkeypatch.setattr(resnet_fused, "_STEM_YAM", yam)
        torch.manual_seed(0)
        stem = ConvBN(3, 64, 7, 2, 3).to(dev)
        stem.bn.weight.data.uniform_(0.5, 1.5)
        stem.bn.bias.data.uniform_(-0.3, 0.3)
        stem.conv.weight.data = stem.conv.weight.data.to(torch.bfloat16)
        stem.train()
        xx = x.detach().clone().requires_grad_(False)
        y = resnet_fused.stem_pool(stem, xx)
        gy = torch.randn(y.shape, generator=g.manual_seed(7)).to(dev)
        (y.float() * gy).sum().backward()
        res.append([t.detach().float().clone() for t in (y, stem.conv.weight.grad, stem.bn.weight.grad,
                                                          stem.bn.bias.grad)])
    for name, a, b in zip(["out", "dW", "dgamma", "dbeta"], *res):
        err = ((a - b).norm() / (a.norm() + 1e-6)).item()
        assert err < 2e-3, (name, err)


def _bf(t):
    """Round to bf16 and back: what dtg stores between kernels."""
    return t.to(torch.bfloat16).to(torch.float32)


def _ref_cbn(P, x, pre, stride=1, pad=0, relu=True, res=None, bf16=False, round_out=True):
    """conv -> training-mode BN (-> + res) (-> relu) in fp32 torch.  ``bf16``: round where dtg stores bf16 --
    the conv output (the BN statistics are taken over the stored values) and the block output; a BN output
    that feeds a fused sum (the projection shortcut) is not rounded (``round_out=False``)."""
    import torch.nn.functional as F
    r = _bf if bf16 else (lambda t: t)
    y = r(F.conv2d(x, P[pre + ".conv.weight"], None, stride, pad))
    y = F.batch_norm(y, None, None, P[pre + ".bn.weight"], P[pre + ".bn.bias"], True, 0.0, 1e-5)
    if res is not None:
        y = y + res
    if relu:
        y = F.relu(y)
    return r(y) if round_out else y


def _ref_block(P, h, pre, blk, bf16=False, drop_residual=False):
    st = blk.c2.conv.stride
    idn = _ref_cbn(P, h, pre + ".down", st, 0, relu=False, bf16=bf16, round_out=False) if blk.down is not None else h
    t = _ref_cbn(P, h, pre + ".c1", bf16=bf16)
    t = _ref_cbn(P, t, pre + ".c2", st, 1, bf16=bf16)
    return _ref_cbn(P, t, pre + ".c3", relu=True, res=None if drop_residual else idn, bf16=bf16)


def _ref_resnet_loss(model, params32, x32, y, drop_residual=None, bf16=False):
    """Plain fp32 PyTorch ResNet (F.conv2d / F.batch_norm in training mode) over ``params32``: the
    model's own weights as fp32 leaves.  ``drop_residual``: index of a block whose identity branch is
    left out (the negative control).  ``bf16``: round every tensor dtg stores in bf16 (conv outputs, BN
    outputs, block outputs, pooled features, logits) -- autograd then rounds the matching gradients too --
    so the comparison measures dtg's accumulation-order noise, not bf16 storage."""
    import torch.nn.functional as F
    P = params32
    r = _bf if bf16 else (lambda t: t)
    h = _ref_cbn(P, x32, "stem", 2, 3, bf16=bf16)
    h = F.max_pool2d(h, 3, 2, 1)
    for i, blk in enumerate(model.blocks):
        h = _ref_block(P, h, "blocks.%d" % i, blk, bf16=bf16, drop_residual=(i == drop_residual))
    h = r(h.mean(dim=(2, 3)))
    logits = r(F.linear(h, P["fc.weight"], P["fc.bias"]))
    return F.cross_entropy(logits, y)


def _ref_params(model, bf16, noise=0.0, seed=11):
    """fp32 leaves of the model's parameters; ``bf16``: conv / FC weights rounded as dtg's bf16 compute
    mirror holds them (BN parameters stay fp32 as in dtg)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    P = {}
    for n, p in model.named_parameters():
        t = p.detach().float().contiguous().clone()
        if noise:
            t = t * (1 + noise * torch.randn(t.shape, generator=g).to(t.device))
        if bf16 and p.dim() > 1:
            t = _bf(t)
        P[n] = t.requires_grad_()
    return P


def _seed_bn(model):
    from dtg.models.layers import BatchNorm2d
    for name, m in model.named_modules():
        if isinstance(m, BatchNorm2d):  # zero-init c3 gammas would hide every residual branch
            m.weight.data.uniform_(*((0.1, 0.3) if name.endswith("c3.bn") else (0.8, 1.2)))
            m.bias.data.uniform_(-0.2, 0.2)


_rel = lambda a, b: ((a - b).norm() / (b.norm() + 1e-12)).item()  # noqa: E731
_med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731


def test_resnet50_full_network_matches_fp32_reference():
    """The whole fused ResNet-50 (stem node, 16 bottleneck nodes with the cross-block BN3 link, pools, FC,
    softmax-xent) against plain fp32 PyTorch with identical weights.

    End to end, a 50-layer ReLU network is chaotic: the fp32 reference's own gradients move by ~27 % (median
    per tensor) under 2^-9 relative weight noise, and a bf16-storage-emulating fp32 reference lands just as far
    from dtg (26.5 %, round 4: the spread is accumulation-order noise amplified through ReLU masks and small-sample
    BN, not bf16 storage).  So the end-to-end gradients are held relative to that noise floor, and the tight
    check is per block, teacher-forced: every bottleneck of the real network, given dtg's own block input and
    the output gradient dtg's backward handed it, is recomputed in fp32 torch with dtg's bf16 storage points
    emulated -- its parameter gradients and input gradient must agree to accumulation-order noise.  Negative
    controls: the end-to-end reference without one residual branch, and a teacher-forced block whose reference
    drops its residual, must disagree far more."""
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet.resnet50(100).to(dev).to(memory_format=torch.channels_last)
    _seed_bn(model)
    FlatParams(model)
    model.train()
    x, y = resnet.synthetic_batch(16, dev, torch.bfloat16, 64, 100, seed=3)
    # capture every block's input and the gradient its backward received (teacher forcing)
    b_in, b_gout = {}, {}

    def fwd_hook(i):
        def h(mod, inp, out):
            b_in[i] = inp[0].detach().float().clone()

            def gh(gr):
                b_gout[i] = gr.detach().float().clone()
            out.register_hook(gh)
        return h
    hooks = [blk.register_forward_hook(fwd_hook(i)) for i, blk in enumerate(model.blocks)]
    loss = ops.softmax_cross_entropy(model(x), y)
    loss.backward()
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    names = [n for n, _ in model.named_parameters()]
    got = {n: p.grad.float() for n, p in model.named_parameters()}

    def reference(drop=None, noise=0.0, bf16=False):
        P = _ref_params(model, bf16, noise)
        ref = _ref_resnet_loss(model, P, x.float(), y, drop_residual=drop, bf16=bf16)
        ref.backward()
        return ref.item(), {n: P[n].grad for n in names}

    ref_loss, ref_g = reference()
    _, noisy_g = reference(noise=2 ** -9)
    _, bad_g = reference(drop=8)  # a layer3 identity block without its skip connection
    e_dtg = {n: _rel(got[n], ref_g[n]) for n in names}
    e_noise = _med([_rel(noisy_g[n], ref_g[n]) for n in names])
    e_bad = _med([_rel(got[n], bad_g[n]) for n in names])
    # per block, teacher-forced
    P = _ref_params(model, True)
    e_blk, e_dx, bad_blk = {}, [], None
    for i, blk in enumerate(model.blocks):
        pre = "blocks.%d" % i
        for drop in ((False, True) if i == 8 else (False,)):
            for t in P.values():
                t.grad = None
            xi = b_in[i].clone().requires_grad_()
            _ref_block(P, xi, pre, blk, bf16=True, drop_residual=drop).backward(b_gout[i])
            errs = {n: _rel(got[n], P[n].grad) for n in names if n.startswith(pre + ".")}
            if drop:
                bad_blk = _med(errs.values())
                continue
            e_blk.update(errs)
            if i > 0:  # the input gradient is the gradient block i-1's output received -- already masked by
                # block i-1's relu in block i's conv1 dgrad epilogue (the cross-block BN3 link): compare masked
                mk = (b_in[i] > 0).float()
                e_dx.append(_rel(b_gout[i - 1] * mk, xi.grad * mk))
    worst = sorted(e_blk.items(), key=lambda kv: -kv[1])[:4]
    print("loss %.6f fp32 ref %.6f | end to end: median grad rel-err %.4f, fp32 ref under 2^-9 weight noise %.4f, "
          "without one residual %.4f | teacher-forced blocks: params median %.4f max %.4f %s, input grads median "
          "%.4f max %.4f, block 8 without its residual %.4f"
          % (loss.item(), ref_loss, _med(e_dtg.values()), e_noise, e_bad, _med(e_blk.values()), worst[0][1],
             worst[0][0], _med(e_dx), max(e_dx), bad_blk))
    assert abs(loss.item() - ref_loss) < 2e-3 * abs(ref_loss)
    assert _med(e_dtg.values()) < 1.6 * e_noise + 0.02
    assert e_bad > 2.0 * _med(e_dtg.values())
    assert _med(e_blk.values()) <= 3e-2 and max(e_blk.values()) <= 0.15, worst
    assert _med(e_dx) <= 3e-2 and max(e_dx) <= 0.1, e_dx
    assert bad_blk > 5 * _med(e_blk.values())


def test_bottleneck_chain_matches_fp32_reference():
    """Three fused bottleneck nodes in a row -- a projection block (stride 1), an identity block and a strided
    projection block, linked through the cross-block BN3 reduction -- against F.conv2d / F.batch_norm in fp32
    with dtg's bf16 storage points emulated: output, input gradient and every parameter gradient."""
    from dtg.models.resnet import Bottleneck
    torch.manual_seed(0)
    dev = torch.device("cuda")
    chain = torch.nn.Module()
    chain.blocks = torch.nn.Sequential(Bottleneck(128, 64, 1), Bottleneck(256, 64, 1), Bottleneck(256, 128, 2))
    chain = chain.to(dev).to(memory_format=torch.channels_last)
    _seed_bn(chain)
    FlatParams(chain)
    chain.train()
    g = torch.Generator(device="cpu").manual_seed(2)
    x0 = torch.randn(16, 128, 28, 28, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = None
    x = x0.clone().requires_grad_()
    out = chain.blocks(x)
    gy = torch.randn(out.shape, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out.backward(gy)
    torch.cuda.synchronize()
    names = [n for n, _ in chain.named_parameters()]

    def reference(drop=None):
        P = _ref_params(chain, True)
        xr = x0.float().requires_grad_()
        h = xr
        for i, blk in enumerate(chain.blocks):
            h = _ref_block(P, h, "blocks.%d" % i, blk, bf16=True, drop_residual=(i == drop))
        h.backward(gy.float())
        return h.detach(), xr.grad, {n: P[n].grad for n in names}

    ref_out, ref_dx, ref_g = reference()
    _, _, bad_g = reference(drop=1)
    e = {n: _rel(p.grad.float(), ref_g[n]) for n, p in chain.named_parameters()}
    e_out, e_dx = _rel(out.float(), ref_out), _rel(x.grad.float(), ref_dx)
    e_bad = _med([_rel(p.grad.float(), bad_g[n]) for n, p in chain.named_parameters()])
    worst = sorted(e.items(), key=lambda kv: -kv[1])[:4]
    print("chain: out %.4f dx %.4f | param grads median %.4f max %.4f %s | without the identity residual %.4f"
          % (e_out, e_dx, _med(e.values()), worst[0][1], worst[0][0], e_bad))
    # three chained blocks already amplify the accumulation-order noise ~10x over one teacher-forced block
    # (round 4: 0.34 % median per block in the full network, 3.6 % here), so the chain bounds are 2x looser
    assert e_out < 1e-2 and e_dx < 6e-2
    assert _med(e.values()) <= 6e-2 and max(e.values()) <= 0.15, worst
    assert e_bad > 5 * _med(e.values())


def test_wgrad_side_stream_accumulates_into_existing_grad(monkeypatch):
    """Parameters WITHOUT flat gradient buffers, two backward passes (the second adds into existing .grad,
    as gradient accumulation does): the side-stream wgrads must be finished before autograd's
    AccumulateGrad adds them on the main stream.  Side stream vs main stream must agree."""
    from dtg.models.resnet import Bottleneck
    from dtg.models import resnet_fused
    from dtg.parallel import overlap
    monkeypatch.setattr(resnet_fused, "_FUSE", True)
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(5)
    x0 = torch.randn(16, 256, 28, 28, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    was = overlap._ON
    try:
        for side in (False, True):
            overlap.set_enabled(side)
            torch.manual_seed(0)
            bl = torch.nn.Sequential(Bottleneck(256, 64, 1), Bottleneck(256, 128, 2)).to(dev)
            bl = bl.to(memory_format=torch.channels_last)
            for p in bl.parameters():
                if p.dim() > 1:
                    p.data = p.data.to(torch.bfloat16)
            bl.train()
            for it in range(2):
                y = bl(x0.clone().requires_grad_())
                gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(it)).to(dev, torch.bfloat16)
                y.backward(gy.contiguous(memory_format=torch.channels_last))
            torch.cuda.synchronize()
            res.append([p.grad.float().clone() for p in bl.parameters()])
    finally:
        overlap.set_enabled(was)
    rel = lambda a, b: ((a - b).norm() / (b.norm() + 1e-12)).item()  # noqa: E731
    errs = [rel(a, b) for a, b in zip(res[1], res[0])]
    assert max(errs) < 1e-2, errs


@pytest.mark.parametrize("N,H", [(4, 112), (3, 30), (2, 58)])
def test_stem_pool_rows_kernel_matches_row_parallel(N, H):
    """The row-walking stem BN + ReLU + 3x3/2 max-pool forward (stem.hip stem_pool_fwd_rows_kernel: a thread walks a
    segment of pooled rows and carries the shared input row in registers) equals the row-parallel kernel bit for
    bit -- outputs, argmax indices (ties: many ReLU zeros and repeated values, first maximum in window order) and
    the saved y at the argmax -- including a segment shorter than the 14-row default (H = 30 -> 15 pooled rows)."""
    import torch.nn.functional as F
    from dtg.ops._native import lib
    dev = torch.device("cuda")
    L = lib()
    C = 64
    g = torch.Generator(device="cpu").manual_seed(H)
    y = (torch.randint(-4, 5, (N, H, H, C), generator=g).float() * 0.5).to(dev, torch.bfloat16)
    yf = y.float().view(-1, C)
    part = torch.zeros(32, 2, C, device=dev)
    part[0, 0] = yf.sum(0)
    part[0, 1] = (yf * yf).sum(0)
    gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
    beta = (torch.rand(C, generator=g) - 0.5).to(dev)
    res = {}
    for on in (0, 1):
        L.stem_pool_rows_set(on)
        try:
            rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
            res[on] = L.stem_bn_pool_fwd(y, part, gamma, beta, rm, rv, 0.1, 1e-5, 3, 2, 1, save_yam=True)
        finally:
            L.stem_pool_rows_set(1)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
    # and against torch: max_pool2d(relu(bn(y)))
    mean, var = yf.mean(0), yf.var(0, unbiased=False)
    a = torch.relu((y.float() - mean) / torch.sqrt(var + 1e-5) * gamma + beta).bfloat16().float()
    ref = F.max_pool2d(a.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.allclose(res[1][0].float(), ref, atol=2e-2, rtol=1e-2)
