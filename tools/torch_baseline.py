#!/usr/bin/env python3
"""Same-hardware comparator for bench.py: the stock PyTorch-ROCm path on ONE MI355X.

The reference publishes no throughput numbers, so the number dtg has to beat on
the GPU is what a user of plain PyTorch-ROCm gets for the same training step:

* ``--model resnet50``: a torchvision-architecture ResNet-50 written with ``torch.nn`` (torchvision
  is not installed here), channels_last, bf16 autocast over fp32 master weights (MIOpen convs and
  batch-norm, hipBLASLt FC), ``torch.optim.SGD(momentum=0.9, foreach)``; batch 256 of 224x224.
* ``--model bert``: HuggingFace ``BertForPreTraining`` (BERT-base config, random init, SDPA
  attention), bf16 autocast over fp32 weights, ``torch.optim.AdamW(fused=True)``; batch 64 x 128
  with 20 masked positions per sequence, MLM + NSP loss.

Same synthetic-data shapes, same warmup/timed-steps bracketing (device synchronize on both sides)
as bench.py; prints one JSON line.  ``--compile`` additionally wraps the model in torch.compile
where the image has a working inductor backend.

    python tools/torch_baseline.py --model resnet50 --steps 20 --warmup 5
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride, down):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, width * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(width * 4)
        self.down = None
        if down:
            self.down = nn.Sequential(nn.Conv2d(cin, width * 4, 1, stride, bias=False), nn.BatchNorm2d(width * 4))

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return F.relu(y + idt)


class ResNet50(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        layers, cin = [], 64
        for width, blocks, stride in [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]:
            for i in range(blocks):
                layers.append(Bottleneck(cin, width, stride if i == 0 else 1, i == 0))
                cin = width * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(2048, classes)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x))), 3, 2, 1)
        x = self.layers(x)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def build(a, dev):
    g = torch.Generator(device="cpu").manual_seed(0)
    if a.model == "bert":
        from transformers import BertConfig, BertForPreTraining
        cfg = BertConfig(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                         intermediate_size=3072, max_position_embeddings=512, attn_implementation="sdpa")
        model = BertForPreTraining(cfg).to(dev)
        b, s, p = a.batch or 64, a.seq, 20
        ids = torch.randint(0, cfg.vocab_size, (b, s), generator=g).to(dev)
        tt = torch.zeros(b, s, dtype=torch.long, device=dev)
        tt[:, s // 2:] = 1
        am = torch.ones(b, s, dtype=torch.long, device=dev)
        labels = torch.full((b, s), -100, dtype=torch.long)
        for i in range(b):
            pos = torch.randperm(s, generator=g)[:p]
            labels[i, pos] = torch.randint(0, cfg.vocab_size, (p,), generator=g)
        labels = labels.to(dev)
        nsp = torch.randint(0, 2, (b,), generator=g).to(dev)
        opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01, fused=True)

        def loss_fn(m):
            return m(input_ids=ids, token_type_ids=tt, attention_mask=am, labels=labels,
                     next_sentence_label=nsp).loss
        return model, opt, loss_fn, b, "sequences/sec", "BERT-base (MLM+NSP, HF transformers)"
    model = ResNet50().to(dev).to(memory_format=torch.channels_last)
    b = a.batch or 256
    x = torch.randn(b, 3, a.image, a.image, generator=g).to(dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (b,), generator=g).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=True)

    def loss_fn(m):
        return F.cross_entropy(m(x), y)
    return model, opt, loss_fn, b, "images/sec", "ResNet-50 (torch.nn, channels_last)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "bert"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--compile", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    # MIOpen find step (per conv shape, first call): without it MIOpen's immediate mode falls back to
    # workspace-free solvers that are ~50x slower on these NHWC bf16 shapes
    torch.backends.cudnn.benchmark = True
    model, opt, loss_fn, batch, unit, name = build(a, dev)
    model.train()
    run = torch.compile(model) if a.compile else model

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = loss_fn(run)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    t0 = time.perf_counter()
    state = {"i": 0}

    def heartbeat():  # MIOpen compiles its kernels on first use (minutes on a fresh box): say so
        while True:
            time.sleep(30)
            print(f"  ... warmup step {state['i']} running, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
    import threading
    threading.Thread(target=heartbeat, daemon=True).start()
    for i in range(a.warmup):
        state["i"] = i
        step()
        torch.cuda.synchronize()
        print(f"warmup step {i} done at {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"comparator": "pytorch-rocm " + torch.__version__ + (" +compile" if a.compile else " eager"),
                      "model": name, "value": round(batch * a.steps / dt, 2), "unit": unit,
                      "ms_per_step": round(dt / a.steps * 1e3, 3), "batch": batch, "steps": a.steps,
                      "warmup": a.warmup, "dtype": "bf16 autocast (fp32 master)", "data": "synthetic",
                      "final_loss": float(loss.float().item())}), flush=True)


if __name__ == "__main__":
    main()
