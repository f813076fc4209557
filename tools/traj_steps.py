#!/usr/bin/env python3
"""Per-step wall time of the config-3 (trajectory) step in several modes, to separate
host overhead, device time and the bench's event instrumentation.

    python tools/traj_steps.py [--batch 8192]
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
from vp3d_amd.pipeline import SyntheticTrajectoryBatcher  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    m = TemporalModelOptimized1f(23, 2, 17, [3] * 5, channels=1024)
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed=0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.eval().cuda()
    RF, B = m.receptive_field(), a.batch
    pipe = SyntheticTrajectoryBatcher(B, RF, seed=1000, device=dev)
    lifter = m.native_lifter(dev)
    lifter.reserve(B, RF, a.dtype)
    y = torch.empty((B, 1, 17, 3), device=dev)

    def cams():
        pipe.next_pairs()

    def fwd(p):
        lifter.forward_windows(pipe.seqs, p, RF, pipe.pad, concat_cams=True, dtype=a.dtype, out=y)

    p0 = pipe.pairs[0]

    def run(name, fn, n=20):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name:40s} {(t2 - t0) / n * 1e3:8.3f} ms/step (host issue {(t1 - t0) / n * 1e3:7.3f} ms)",
              flush=True)

    with torch.no_grad():
        run("camera_matrices only", cams)
        run("forward_windows only (fixed pairs)", lambda: fwd(p0))
        run("full step (cams + next pairs + fwd)", lambda: fwd(pipe.next_pairs()))
        run("full step again", lambda: fwd(pipe.next_pairs()))
        xg = pipe.gather(p0).contiguous()
        run("materialised gather + lifter.forward", lambda: lifter.forward(xg, a.dtype, out=y))
        lifter.profile(True)
        lifter.profile_layers([1])
        run("full step, events around block1_k3", lambda: fwd(pipe.next_pairs()))
        lifter.profile(False)
        lifter.profile_layers(None)
        run("full step (after profiling)", lambda: fwd(pipe.next_pairs()))
        # bench.py's exact sequence: all-layer event pass, read, then block1_k3 only
        lifter.profile(True)
        lifter.profile_layers(None)
        lifter.profile_reset()
        for _ in range(10):
            fwd(pipe.next_pairs())
        lifter.profile_read()
        lifter.profile_layers([1])
        lifter.profile_reset()
        run("bench sequence: block1_k3 events", lambda: fwd(pipe.next_pairs()))
        lifter.profile_reset()
        lifter.profile_layers(None)
        run("bench sequence: all-layer events", lambda: fwd(pipe.next_pairs()))
        lifter.profile(False)
        run("after", lambda: fwd(pipe.next_pairs()))


if __name__ == "__main__":
    main()
