#!/usr/bin/env python3
"""YARDSTICK ONLY (never part of the product path): the same ResNet-50 training step written with
stock PyTorch-ROCm modules (nn.Conv2d → MIOpen, nn.BatchNorm2d, torch.optim.SGD), channels_last,
bf16 autocast.  Used to put the native-kernel numbers of bench.py in context on the same box.

  python bench/yardstick_torch.py --batch 256 --steps 10 --warmup 3
"""
import argparse
import json
import time

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    def __init__(self, cin, w, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, w, 1, bias=False)
        self.b1 = nn.BatchNorm2d(w)
        self.c2 = nn.Conv2d(w, w, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(w)
        self.c3 = nn.Conv2d(w, w * 4, 1, bias=False)
        self.b3 = nn.BatchNorm2d(w * 4)
        self.down = None
        if stride != 1 or cin != w * 4:
            self.down = nn.Sequential(nn.Conv2d(cin, w * 4, 1, stride, bias=False),
                                      nn.BatchNorm2d(w * 4))

    def forward(self, x):
        sc = x if self.down is None else self.down(x)
        y = torch.relu(self.b1(self.c1(x)))
        y = torch.relu(self.b2(self.c2(y)))
        return torch.relu(self.b3(self.c3(y)) + sc)


class ResNet50(nn.Module):
    def __init__(self):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64),
                                  nn.ReLU(), nn.MaxPool2d(3, 2, 1))
        layers, cin = [], 64
        for i, n in enumerate((3, 4, 6, 3)):
            w = 64 * 2 ** i
            for j in range(n):
                layers.append(Bottleneck(cin, w, 2 if (j == 0 and i > 0) else 1))
                cin = w * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(2048, 1000)

    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(x.mean((2, 3)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = ResNet50().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev)
    lossf = nn.CrossEntropyLoss()

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = lossf(m(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"yardstick": "pytorch-rocm (MIOpen) resnet50 bf16 autocast channels_last",
                      "images_per_sec": round(a.batch * a.steps / el, 1),
                      "ms_per_step": round(el / a.steps * 1e3, 2), "batch": a.batch}))


if __name__ == "__main__":
    main()
