#!/usr/bin/env python3
"""A/B: one forward of B windows on one stream vs the batch split into S shards
forwarded concurrently on S streams (one vp3d handle each), so the last partial
round of 256x256 tiles of one shard's layer overlaps the next layer of another.

    VP3D_BIG_MIN_TILES=128 python tools/split_streams.py [--batch 8192]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "dynamic-camera-augmented-videopose3d_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

from common.models.TemporalModel import TemporalModelOptimized1f  # noqa: E402
from vp3d_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B = a.batch
    sd = None
    models = []
    for i in range(4):
        m = TemporalModelOptimized1f(17, 2, 17, [3] * 5, channels=1024)
        if sd is None:
            sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed=0)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        m.eval().cuda()
        models.append(m)
    lifters = [m.native_lifter(dev) for m in models]
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = (torch.rand((B, 243, 17, 2), generator=g, device=dev) - 0.5).contiguous()
    y = torch.empty((B, 1, 17, 3), device=dev)
    y_ref = torch.empty_like(y)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    main_s = torch.cuda.current_stream(dev)

    def single():
        lifters[0].forward(x, a.dtype, out=y)

    def split(S):
        def f():
            ev = torch.cuda.Event()
            ev.record(main_s)
            n = B // S
            for i in range(S):
                streams[i].wait_event(ev)
                with torch.cuda.stream(streams[i]):
                    lifters[i].forward(x[i * n:(i + 1) * n], a.dtype, out=y[i * n:(i + 1) * n])
            for i in range(S):
                main_s.wait_stream(streams[i])
        return f

    def run(name, fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        while time.perf_counter() - t < 0.5:  # clocks up
            fn()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(f"{name:28s} {dt * 1e3:7.3f} ms/step  {B / dt / 1e6:6.3f} M poses/s", flush=True)

    with torch.no_grad():
        for S in (1, 2, 4):
            for L in lifters[:S]:
                L.reserve(B // S, 243, a.dtype)
        run("single stream", single)
        y_ref.copy_(y)
        for S in (2, 4):
            y.zero_()
            run(f"split x{S}", split(S))
            d = (y - y_ref).abs().max().item()
            print(f"   max |split - single| = {d:.3e}", flush=True)
        run("single stream again", single)
        run("split x2 again", split(2))


if __name__ == "__main__":
    main()
