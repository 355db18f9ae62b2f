#!/usr/bin/env python3
"""Per-call roofline of one ResNet-50 (or BERT) training step: every native GEMM / conv / BN call is
bracketed by device events, its FLOPs and compulsory HBM bytes are computed from the shapes, and
the table shows achieved TFLOP/s, TB/s and the fraction of the roofline bound
max(flops / 2.5 PF, bytes / 8 TB/s) it reaches -- the list of what is worth optimising next.

    python tools/layer_roofline.py [--model resnet|bert] [--batch 256] [--top 40] [--json out.json]
"""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TF = 2500.0   # dense bf16 MFMA, TFLOP/s
PEAK_BW = 8.0      # HBM3E, TB/s


def _nb(t):
    return 0 if t is None else t.numel() * t.element_size()


def _gemm_cost(args, kw):
    A, a_kc, B, b_kc, out = args[:5]
    beta = args[6] if len(args) > 6 else kw.get("beta", 0.0)
    M = A.shape[0] if a_kc else A.shape[1]
    K = A.shape[1] if a_kc else A.shape[0]
    N = B.shape[0] if b_kc else B.shape[1]
    by = _nb(A) + _nb(B) + _nb(out) * (2 if beta else 1)
    return f"gemm {M}x{N}x{K}{' +C' if beta else ''}", 2.0 * M * N * K, by


def _conv_geo(x, w, st, pad):
    n, h, wd, c = x.shape
    k, r, s = w.shape[0], w.shape[1], w.shape[2]
    return n, h, wd, c, k, r, s, (h + 2 * pad - r) // st + 1, (wd + 2 * pad - s) // st + 1


def _conv_fwd_cost(args, kw):
    x, w, st, pad = args[:4]
    n, h, wd, c, k, r, s, p, q = _conv_geo(x, w, st, pad)
    return (f"conv_fwd {r}x{s}/{st} {h}x{wd} C{c}->K{k}", 2.0 * n * p * q * k * r * s * c,
            _nb(x) + _nb(w) + n * p * q * k * 2)


def _conv_dgrad_cost(args, kw):
    dy, w, H, W, st, pad = args[:6]
    beta = kw.get("beta", args[7] if len(args) > 7 else 0.0)
    n, p, q, k = dy.shape
    r, s, c = w.shape[1], w.shape[2], w.shape[3]
    return (f"conv_dgrad {r}x{s}/{st} {H}x{W} K{k}->C{c}{' +C' if beta else ''}", 2.0 * n * p * q * k * r * s * c,
            _nb(dy) + _nb(w) + n * H * W * c * 2 * (2 if beta else 1))


def _conv_wgrad_cost(args, kw):
    dy, x, dw = args[:3]
    n, p, q, k = dy.shape
    r, s, c = dw.shape[1], dw.shape[2], dw.shape[3]
    return (f"conv_wgrad {r}x{s} {x.shape[1]}x{x.shape[2]} C{c} K{k}", 2.0 * n * p * q * k * r * s * c,
            _nb(dy) + _nb(x) + 2 * _nb(dw))


def _bn_fwd_cost(args, kw):
    x, res = args[0], args[1]
    return (f"bn_fwd {tuple(x.shape)}{' +res' if res is not None else ''}", 0.0,
            2 * _nb(x) + _nb(res) + _nb(x))


def _bn_bwd_cost(args, kw):
    dy, y, x = args[:3]
    want_dres = args[7] if len(args) > 7 else False
    return (f"bn_bwd {tuple(dy.shape)}{' relu' if y is not None else ''}{' +dres' if want_dres else ''}", 0.0,
            2 * (_nb(dy) + _nb(y) + _nb(x)) + _nb(dy) * (2 if want_dres else 1))


def _gemm_bn_cost(args, kw):
    A, B, mode = args[:3]
    M, K = A.shape
    N = B.shape[0] if mode == 1 else B.shape[1]
    by = _nb(A) + _nb(B) + M * N * 2 * (1 if mode == 1 else 2)  # mode 2 also reads the BN input
    return f"gemm_bn{mode} {M}x{N}x{K}", 2.0 * M * N * K, by


def _conv_fwd_bn_cost(args, kw):
    lab, fl, by = _conv_fwd_cost(args, kw)
    return lab.replace("conv_fwd", "conv_fwd_bn"), fl, by


def _conv_dgrad_bn_cost(args, kw):
    lab, fl, by = _conv_dgrad_cost(args[:6], {})
    return lab.replace("conv_dgrad", "conv_dgrad_bn"), fl, by + _nb(args[6])


def _bn_fwd_part_cost(args, kw):
    x, res = args[0], args[2]
    return f"bn_fwd_part {tuple(x.shape)}{' +res' if res is not None else ''}", 0.0, 2 * _nb(x) + _nb(res)


def _bn_bwd_part_cost(args, kw):
    dp, x = args[:2]
    return f"bn_bwd_part {tuple(dp.shape)}", 0.0, 3 * _nb(dp)


COSTS = {"gemm_bn": _gemm_bn_cost, "conv_fwd_bn": _conv_fwd_bn_cost, "conv_dgrad_bn": _conv_dgrad_bn_cost,
         "bn_fwd_part": _bn_fwd_part_cost, "bn_bwd_part": _bn_bwd_part_cost, "gemm": _gemm_cost, "conv_fwd": _conv_fwd_cost, "conv_dgrad": _conv_dgrad_cost,
         "conv_wgrad": _conv_wgrad_cost, "bn_fwd_train": _bn_fwd_cost, "bn_bwd": _bn_bwd_cost}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", default="")
    ap.add_argument("--conv-stages", default="", help="LDS ring depth of conv fwd,dgrad,wgrad, e.g. 1,1,2")
    a = ap.parse_args()
    import torch
    import dtg  # noqa: F401
    from dtg import ops
    from dtg.ops._native import lib

    L = lib()
    if a.conv_stages:
        for i, v in enumerate(a.conv_stages.split(",")):
            L.conv_set_stages(i, int(v))
    dev = torch.device("cuda")
    records = []
    active = [False]

    def wrap(name, fn, cost):
        def w(*args, **kw):
            if not active[0]:
                return fn(*args, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*args, **kw)
            e1.record()
            records.append((cost(args, kw), e0, e1))
            return r
        return w

    for name, cost in COSTS.items():
        setattr(L, name, wrap(name, getattr(L, name), cost))

    from dtg.parallel import FlatParams
    torch.manual_seed(0)
    if a.model == "bert":
        from dtg.models import bert
        from dtg.optim import FusedAdam
        cfg = bert.BertConfig.base()
        model = bert.BertForPreTraining(cfg).to(dev)
        flat = FlatParams(model)
        opt = FusedAdam(flat, lr=1e-4)
        batch = bert.synthetic_batch(a.batch or 64, 128, cfg, dev)

        def step():
            model(*batch).backward()
            opt.step()
    else:
        from dtg.models import resnet
        from dtg.optim import FusedSGD
        model = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
        flat = FlatParams(model)
        opt = FusedSGD(flat, lr=0.1, momentum=0.9)
        x, y = resnet.synthetic_batch(a.batch or 256, dev)

        def step():
            ops.softmax_cross_entropy(model(x), y).backward()
            opt.step()
    model.train()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record()
    for _ in range(5):
        step()
    c1.record()
    torch.cuda.synchronize()
    clean_ms = c0.elapsed_time(c1) / 5
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    active[0] = True
    t0.record()
    step()
    t1.record()
    active[0] = False
    torch.cuda.synchronize()
    total = t0.elapsed_time(t1) * 1e3
    agg = collections.OrderedDict()
    for (label, fl, by), e0, e1 in records:
        us = e0.elapsed_time(e1) * 1e3
        a_ = agg.setdefault(label, [0, 0.0, 0.0, 0.0])
        a_[0] += 1
        a_[1] += us
        a_[2] += fl
        a_[3] += by
    rows = []
    for label, (n, us, fl, by) in agg.items():
        bound = max(fl / (PEAK_TF * 1e12), by / (PEAK_BW * 1e12)) * 1e6
        rows.append({"op": label, "calls": n, "us": us, "tflops": fl / us / 1e6 if us else 0.0,
                     "tbps": by / us / 1e6 if us else 0.0, "bound_us": bound, "eff": bound / us if us else 0.0,
                     "lost_us": us - bound})
    rows.sort(key=lambda r: -r["lost_us"])
    covered = sum(r["us"] for r in rows)
    print(f"uninstrumented step {clean_ms:.2f} ms (conv stages {a.conv_stages or 'default'})")
    print(f"step {total:.0f} us; instrumented ops {covered:.0f} us; roofline bound of those "
          f"{sum(r['bound_us'] for r in rows):.0f} us")
    print(f"{'op':52s} {'calls':>5s} {'us':>8s} {'TF/s':>7s} {'TB/s':>6s} {'eff':>5s} {'lost us':>8s}")
    for r in rows[:a.top]:
        print(f"{r['op'][:52]:52s} {r['calls']:5d} {r['us']:8.1f} {r['tflops']:7.1f} {r['tbps']:6.2f} "
              f"{r['eff']:5.2f} {r['lost_us']:8.1f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"step_us": total, "clean_ms": clean_ms, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
