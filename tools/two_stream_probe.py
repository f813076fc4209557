#!/usr/bin/env python3
"""Probe: does splitting a small per-GPU batch into two halves on two HIP streams (two
lifter workspaces) fill the fractional tile rounds of the B = 8,192 step (config 4 at
N = 8)?  Times one forward_windows of B windows against two of B/2 on two streams
(fork/join by events), bf16, Optimized1f 243-RF, 1024 ch.  Measurement only.

    python tools/two_stream_probe.py [B ...]
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dynamic-camera-augmented-videopose3d_amd"))
sys.path.insert(0, REPO)


def main():
    from common.models.TemporalModel import TemporalModelOptimized1f
    from vp3d_amd import synth
    from vp3d_amd.pipeline import SyntheticWindowPool

    sizes = [int(a) for a in sys.argv[1:]] or [8192, 16384, 65536]
    dev = torch.device("cuda", 0)
    FW = [3, 3, 3, 3, 3]
    models = []
    for _ in range(2):
        m = TemporalModelOptimized1f(17, 2, 17, FW, channels=1024)
        sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed=0)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        models.append(m.eval().cuda())
    RF = models[0].receptive_field()
    pad = (RF - 1) // 2
    pool = SyntheticWindowPool(1000, dev, cameras=False)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for B in sizes:
        pairs = torch.from_numpy(pool.global_pairs(B)).to(dev)
        h = B // 2
        lifters = [m.native_lifter(dev) for m in models]
        lifters[0].reserve(B, RF, "bf16")
        lifters[1].reserve(B - h, RF, "bf16")
        y = torch.empty((B, 1, 17, 3), device=dev)
        y2 = torch.empty((B, 1, 17, 3), device=dev)
        pa, pb = pairs[:h].contiguous(), pairs[h:].contiguous()

        def one():
            lifters[0].forward_windows(pool.seqs, pairs, RF, pad, dtype="bf16", out=y)

        def two():
            cur = torch.cuda.current_stream(dev)
            ev = torch.cuda.Event()
            ev.record(cur)
            for s, lf, p, o in ((s1, lifters[0], pa, y2[:h]), (s2, lifters[1], pb, y2[h:])):
                s.wait_event(ev)
                with torch.cuda.stream(s):
                    lf.forward_windows(pool.seqs, p, RF, pad, dtype="bf16", out=o)
            for s in (s1, s2):
                e = torch.cuda.Event()
                e.record(s)
                cur.wait_event(e)

        res = {}
        for name, fn in (("one", one), ("two", two), ("one", one), ("two", two)):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            n = max(5, int(20 * 65536 / B))
            t = time.perf_counter()
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / n * 1e3
            res.setdefault(name, []).append(ms)
        same = bool(torch.equal(y, y2))
        print(f"B={B}: one stream {' / '.join(f'{v:.4f}' for v in res['one'])} ms "
              f"({B / min(res['one']) * 1e3 / 1e6:.3f} M poses/s); two streams "
              f"{' / '.join(f'{v:.4f}' for v in res['two'])} ms ({B / min(res['two']) * 1e3 / 1e6:.3f} M poses/s); "
              f"outputs equal: {same}", flush=True)


if __name__ == "__main__":
    main()
