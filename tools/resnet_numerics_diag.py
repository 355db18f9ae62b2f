#!/usr/bin/env python3
"""Per-parameter gradient agreement of the whole ResNet-50 (dtg fused, dtg layer-wise) against an fp32
PyTorch reference with the same weights, plus the reference's own sensitivity to bf16-sized weight noise
(how chaotic the network's gradients are at this init).  Diagnostic for tests/test_resnet_gpu.py.

    python tools/resnet_numerics_diag.py [--batch 8] [--image 96] [--gamma uniform|ones]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402

import dtg  # noqa: E402,F401
from dtg import ops  # noqa: E402
from dtg.models import resnet, resnet_fused  # noqa: E402
from dtg.models.layers import BatchNorm2d  # noqa: E402
from dtg.parallel import FlatParams  # noqa: E402
from test_resnet_gpu import _ref_resnet_loss  # noqa: E402


def init_bn(model, mode):
    """BN affine init: "uniform" gammas 0.5-1.5 everywhere (chaotic gradients at small batch); "small3"
    gammas 0.8-1.2 except the last BN of every residual branch at 0.1-0.3 (near-identity blocks, so
    gradients are well conditioned but every branch still contributes)."""
    for name, m in model.named_modules():
        if isinstance(m, BatchNorm2d):
            if mode == "small3" and name.endswith("c3.bn"):
                m.weight.data.uniform_(0.1, 0.3)
            elif mode == "small3":
                m.weight.data.uniform_(0.8, 1.2)
            else:
                m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--image", type=int, default=96)
    ap.add_argument("--gamma", default="uniform", help="uniform | small3 (residual-branch gammas 0.1-0.3)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = resnet.resnet50(100).to(dev).to(memory_format=torch.channels_last)
    init_bn(model, a.gamma)
    FlatParams(model)
    model.train()
    x, y = resnet.synthetic_batch(a.batch, dev, torch.bfloat16, a.image, 100, seed=3)
    names = [n for n, _ in model.named_parameters()]
    state = {k: v.clone() for k, v in model.state_dict().items()}

    def dtg_grads(fused):
        model.load_state_dict(state)
        for p in model.parameters():
            p.grad.zero_()
        for b in model.blocks:
            b.fused = fused
        resnet_fused._STEM = fused
        loss = ops.softmax_cross_entropy(model(x), y)
        loss.backward()
        torch.cuda.synchronize()
        return loss.item(), {n: p.grad.float().clone() for n, p in model.named_parameters()}

    def ref_grads(noise=0.0, dtype=torch.float32):
        g = torch.Generator(device="cpu").manual_seed(11)
        P = {}
        for n, p in model.named_parameters():
            t = p.detach().to(dtype).contiguous().clone()
            if noise:
                t = t * (1 + noise * torch.randn(t.shape, generator=g).to(dev, dtype))
            P[n] = t.requires_grad_()
        loss = _ref_resnet_loss(model, P, x.to(dtype), y)
        loss.backward()
        return loss.item(), {n: P[n].grad.float() for n in names}

    rel = lambda u, v: ((u - v).norm() / (v.norm() + 1e-12)).item()  # noqa: E731
    r64 = ref_grads(dtype=torch.float64)
    runs = {"ref32": ref_grads(), "ref32_noise2^-9": ref_grads(2 ** -9), "dtg_fused": dtg_grads(True),
            "dtg_layerwise": dtg_grads(False)}
    print("loss fp64 ref %.6f" % r64[0])
    for k, (l, g) in runs.items():
        e = [rel(g[n], r64[1][n]) for n in names]
        se = sorted(e)
        print("%-18s loss %.6f  grad rel-err vs fp64: median %.4f  p90 %.4f  max %.4f" % (
            k, l, se[len(se) // 2], se[int(len(se) * 0.9)], se[-1]))
    f, lw = runs["dtg_fused"][1], runs["dtg_layerwise"][1]
    print("per-parameter (backward order, every 6th): name  fused-vs-ref32  layerwise-vs-ref32  fused-vs-layerwise")
    r32 = runs["ref32"][1]
    for n in list(reversed(names))[::6]:
        print("  %-28s %.4f %.4f %.4f" % (n, rel(f[n], r32[n]), rel(lw[n], r32[n]), rel(f[n], lw[n])))


if __name__ == "__main__":
    main()
