#!/usr/bin/env python3
"""Where does the 16-bit error of the trajectory-conditioned (46-ch) Optimized1f path
come from?  CPU emulation of the native 16-bit arithmetic (A and W rounded to the
16-bit type, f32 accumulation, f32 BN affine in the epilogue, activations rounded to
the 16-bit type), with stages selectively kept in f32.

    python tools/bf16_error_study.py [--dtype bf16] [--B 32] [--traj]

Not a test: a numerics study whose output is quoted in DESIGN.md.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dynamic-camera-augmented-videopose3d_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle.temporal_ref import lifter_forward  # noqa: E402
from vp3d_amd import synth  # noqa: E402


def keys_shapes(jin, fw, C, jout=17):
    ks = [("expand_conv.weight", (C, jin * 2, fw[0]))]
    for n in ("expand_bn",):
        ks += [(f"{n}.weight", (C,)), (f"{n}.bias", (C,)), (f"{n}.running_mean", (C,)),
               (f"{n}.running_var", (C,)), (f"{n}.num_batches_tracked", ())]
    for i, w in enumerate(fw[1:]):
        ks.append((f"layers_conv.{2 * i}.weight", (C, C, w)))
        ks.append((f"layers_conv.{2 * i + 1}.weight", (C, C, 1)))
    for i in range(2 * (len(fw) - 1)):
        n = f"layers_bn.{i}"
        ks += [(f"{n}.weight", (C,)), (f"{n}.bias", (C,)), (f"{n}.running_mean", (C,)),
               (f"{n}.running_var", (C,)), (f"{n}.num_batches_tracked", ())]
    ks += [("shrink.weight", (jout * 3, C, 1)), ("shrink.bias", (jout * 3,))]
    return ks


def emulate(sd, x, fw, dt, exact=(), split_a=(), eps=1e-5):
    """Optimized1f forward, layer l computed with A, W rounded to `dt` unless l in `exact`;
    l in `split_a`: A carried as hi + lo (two MFMAs), W still rounded."""
    r = (lambda t: t.to(dt).float())
    sdt = {k: torch.from_numpy(np.asarray(v)).float() for k, v in sd.items() if not k.endswith("tracked")}

    def fold(name):
        inv = 1.0 / torch.sqrt(sdt[name + ".running_var"] + eps)
        sc = sdt[name + ".weight"] * inv
        return sc, sdt[name + ".bias"] - sdt[name + ".running_mean"] * sc

    def conv(h, wname, layer, stride):
        W = sdt[wname]
        if layer in exact:
            return F.conv1d(h, W, None, stride=stride)
        Wr = r(W)
        if layer in split_a:
            hi = r(h)
            lo = r(h - hi)
            return F.conv1d(hi, Wr, None, stride=stride) + F.conv1d(lo, Wr, None, stride=stride)
        return F.conv1d(r(h), Wr, None, stride=stride)

    def act(h, layer):
        return h if layer in exact else r(h)

    B, T = x.shape[:2]
    h = torch.from_numpy(x).reshape(B, T, -1).permute(0, 2, 1).contiguous()
    sc, sh = fold("expand_bn")
    h = act(F.relu(conv(h, "expand_conv.weight", 0, fw[0]) * sc[:, None] + sh[:, None]), 0)
    for i, w in enumerate(fw[1:]):
        res = h[:, :, w // 2::w]
        sc, sh = fold(f"layers_bn.{2 * i}")
        l1 = 1 + 2 * i
        h = act(F.relu(conv(h, f"layers_conv.{2 * i}.weight", l1, w) * sc[:, None] + sh[:, None]), l1)
        sc, sh = fold(f"layers_bn.{2 * i + 1}")
        l2 = 2 + 2 * i
        h = act(res + F.relu(conv(h, f"layers_conv.{2 * i + 1}.weight", l2, 1) * sc[:, None] + sh[:, None]), l2)
    L = 2 * (len(fw) - 1) + 1
    Wsh = sdt["shrink.weight"] if L in exact else r(sdt["shrink.weight"])
    h = F.conv1d(h, Wsh, sdt["shrink.bias"])
    return h.permute(0, 2, 1).reshape(B, h.shape[2], -1, 3).numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--C", type=int, default=1024)
    ap.add_argument("--traj", action="store_true")
    ap.add_argument("--bench-data", action="store_true", help="config-3 bench windows (large dolly offsets)")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    fw = [3, 3, 3, 3, 3]
    jin = 23 if a.traj else 17
    sd = synth.lifter_state_dict(keys_shapes(jin, fw, a.C), seed=0)
    x2 = synth.normalized_windows(1, "study", a.B, 243)
    if a.traj and a.bench_data:
        # the config-3 bench workload (vp3d_amd.pipeline.SyntheticTrajectoryBatcher, seed 1000)
        rng = np.random.RandomState(1000)
        n_seq, L = 64, 2048
        seqs = []
        for i in range(4):
            trk = synth.keypoint_tracks(1000, f"traj{i}", L)
            kp = (trk / 1280 * 2 - np.array([1, 720 / 1280])).astype(np.float32).reshape(L, 34)
            E = synth.camera_extrinsics(1000, f"traj{i}", L)
            K = np.diag([1.5625, 1.5625, 1.0])
            ke = (K @ E).astype(np.float32).reshape(L, 12)
            seqs.append(np.concatenate([kp, ke], axis=1))
        wins = []
        for b in range(a.B):
            s, st = rng.randint(0, 4), rng.randint(0, L)
            idx = np.clip(np.arange(st - 121, st + 122), 0, L - 1)
            wins.append(seqs[s][idx])
        x = np.stack(wins).reshape(a.B, 243, 23, 2)
        print("input |max| kps %.3f cams %.3f" % (np.abs(x.reshape(a.B, 243, 46)[..., :34]).max(),
                                                  np.abs(x.reshape(a.B, 243, 46)[..., 34:]).max()))
    elif a.traj:
        E = synth.camera_extrinsics(2, "study", 243 + a.B)
        K = np.diag([1.5625, 1.5625, 1.0]).astype(np.float32)
        ke = (K.astype(np.float64) @ E).astype(np.float32).reshape(-1, 12)
        cams = np.stack([ke[b:b + 243] for b in range(a.B)])
        x = np.concatenate([x2.reshape(a.B, 243, 34), cams], axis=-1).reshape(a.B, 243, 23, 2)
    else:
        x = x2
    x = np.ascontiguousarray(x, dtype=np.float32)
    ref = lifter_forward(sd, x, fw, strided=True, dtype=torch.float64).numpy()
    gt = synth.gt_poses(3, "study_gt", a.B, 17).reshape(ref.shape)
    print("output |max| %.3f m, rms %.3f m" % (np.abs(ref).max(), np.sqrt(np.mean(ref ** 2))))

    def rep(name, y):
        mp = lambda v: float(np.mean(np.linalg.norm(v.astype(np.float64) - gt, axis=-1)))
        print(f"{name:40s} max|d| {np.abs(y - ref).max() * 1e3:8.3f} mm   dMPJPE {abs(mp(y) - mp(ref)) * 1e3:.5f} mm",
              flush=True)

    nl = 2 * (len(fw) - 1) + 2
    rep("all 16-bit", emulate(sd, x, fw, dt))
    rep("expand A split hi+lo", emulate(sd, x, fw, dt, split_a=(0,)))
    rep("expand exact (f32)", emulate(sd, x, fw, dt, exact=(0,)))
    rep("expand exact + b1 k3 A split", emulate(sd, x, fw, dt, exact=(0,), split_a=(1,)))
    rep("all but expand exact", emulate(sd, x, fw, dt, exact=tuple(range(1, nl))))
    rep("all exact (f32 emulation)", emulate(sd, x, fw, dt, exact=tuple(range(nl))))


if __name__ == "__main__":
    main()
