#!/usr/bin/env python3
"""Numerics study for the split-fp16 ("f16x3") GEMM path: CPU emulation of the
arithmetic the native kernels use, against the fp32 oracle.

Every 16-bit operand pair carries an f32 value x as hi = f16(x), lo = f16((x - hi) * 2^11);
weights are pre-scaled by a per-layer power of two s (max |W s| in [2^14, 2^15)), so
    W s ~= Wh + Wl,   Wh = f16(W s),  Wl = f16(W s - Wh)
and one conv is three 16-bit MFMA products accumulated in f32:
    acc = A_hi . Wh  +  A_lo . f16(Wh * 2^-11)  +  A_hi . Wl      (= s * A . W + O(2^-22))
followed by the f32 epilogue relu(acc * (scale / s) + shift) [+ residual], the output
stored again as a (hi, lo) pair.  The block-4 1x1 writes f32 and the shrink runs the
exact f32 GEMM.

    python tools/split_f16_study.py [--B 64] [--traj]
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

sys.path.insert(0, os.path.join(REPO, "tools"))
from bf16_error_study import keys_shapes  # noqa: E402

h16 = lambda t: t.to(torch.float16).float()  # noqa: E731


LO_SCALE = 1.0  # 2^11: lo carried scaled (kernel variant A); 1: unscaled lo (interleaved variant)


def split(x):
    hi = h16(x)
    return hi, h16((x - hi) * LO_SCALE)


W3 = False  # a third weight half: W s = Wh + Wl + W3 exactly, and a 4th product A_hi . W3


def wsplit(W):
    e = 14 - int(np.floor(np.log2(float(W.abs().max()))))
    Ws = W * (2.0 ** e)
    Wh = h16(Ws)
    Wl = h16(Ws - Wh)
    return Wh, h16(Wh / LO_SCALE), Wl, (h16(Ws - Wh - Wl) if W3 else None), 2.0 ** -e


def emulate(sd, x, fw, eps=1e-5):
    sdt = {k: torch.from_numpy(np.asarray(v)).float() for k, v in sd.items() if not k.endswith("tracked")}

    def fold(name):
        inv = 1.0 / torch.sqrt(sdt[name + ".running_var"] + eps)
        sc = sdt[name + ".weight"] * inv
        return sc, sdt[name + ".bias"] - sdt[name + ".running_mean"] * sc

    def conv(pair, wname, stride):
        hi, lo = pair
        Wh, Wh11, Wl, Wr, inv_s = wsplit(sdt[wname])
        acc = F.conv1d(hi, Wh, None, stride=stride)
        acc = acc + F.conv1d(lo, Wh11, None, stride=stride)
        acc = acc + F.conv1d(hi, Wl, None, stride=stride)
        if Wr is not None:
            acc = acc + F.conv1d(hi, Wr, None, stride=stride)
        return acc, inv_s

    def bn_relu(acc, inv_s, name):
        sc, sh = fold(name)
        return F.relu(acc * (sc * inv_s)[:, None] + sh[:, None])

    def join(p):
        return p[0] + p[1] / LO_SCALE

    B, T = x.shape[:2]
    h = torch.from_numpy(x).reshape(B, T, -1).permute(0, 2, 1).contiguous()
    acc, s = conv(split(h), "expand_conv.weight", fw[0])
    hp = split(bn_relu(acc, s, "expand_bn"))
    nb = len(fw) - 1
    for i, w in enumerate(fw[1:]):
        res = join(hp)[:, :, w // 2::w]
        acc, s = conv(hp, f"layers_conv.{2 * i}.weight", w)
        mid = split(bn_relu(acc, s, f"layers_bn.{2 * i}"))
        acc, s = conv(mid, f"layers_conv.{2 * i + 1}.weight", 1)
        out = res + bn_relu(acc, s, f"layers_bn.{2 * i + 1}")
        hp = split(out) if i + 1 < nb else (out, None)
    y = F.conv1d(hp[0], sdt["shrink.weight"], sdt["shrink.bias"])
    return y.permute(0, 2, 1).reshape(B, -1, 17, 3).numpy()


def dolly_windows(B, seed=1000, n_seq=64, L=2048, W=243):
    """vp3d_amd.pipeline.SyntheticWindowPool(cameras=True) windows on the host: normalised
    random-walk tracks + K.E (CMU K, yaw + dolly extrinsics), edge-clamped."""
    pairs = np.random.RandomState(seed + 1)
    seqs = pairs.randint(0, n_seq, size=B)
    starts = pairs.randint(0, L, size=B)
    K = np.diag([1.5625, 1.5625, 1.0]).astype(np.float32)
    out = np.zeros((B, W, 46), np.float32)
    cache = {}
    for b in range(B):
        i = int(seqs[b])
        if i not in cache:
            trk = synth.keypoint_tracks(seed, f"pool{i}", L)
            kps = (trk / 1280 * 2 - np.array([1, 720 / 1280])).astype(np.float32).reshape(L, 34)
            ke = (K @ synth.camera_extrinsics(seed, f"pool{i}", L)).astype(np.float32).reshape(L, 12)
            cache[i] = np.concatenate([kps, ke], axis=1)
        f = np.clip(np.arange(W) + starts[b] - (W - 1) // 2, 0, L - 1)
        out[b] = cache[i][f]
    return out.reshape(B, W, 23, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--traj", action="store_true")
    ap.add_argument("--lo-scale", type=float, default=1.0)
    ap.add_argument("--dolly", action="store_true", help="the bench's config-3 windows (K.E up to ~22 m)")
    ap.add_argument("--w3", action="store_true", help="three weight halves, four products")
    a = ap.parse_args()
    global LO_SCALE, W3
    LO_SCALE, W3 = a.lo_scale, a.w3
    fw = [3, 3, 3, 3, 3]
    jin = 23 if (a.traj or a.dolly) else 17
    sd = synth.lifter_state_dict(keys_shapes(jin, fw, 1024), seed=0)
    if a.dolly:
        x = dolly_windows(a.B)
    else:
        x = synth.normalized_windows(1, "x64_243", a.B, 243, n_joints=jin)
    ref = lifter_forward(sd, x, fw, strided=True).numpy()
    ref64 = lifter_forward(sd, x, fw, strided=True, dtype=torch.float64).numpy()
    y = emulate(sd, x, fw)
    gt = synth.gt_poses(3, "gt", a.B, 17).reshape(ref.shape)

    def mp(v):
        return float(np.mean(np.linalg.norm(v.astype(np.float64) - gt, axis=-1)))
    print(f"rms out {np.sqrt(np.mean(ref ** 2)):.4f} m")
    print(f"split vs fp32 oracle: max {np.abs(y - ref).max() * 1e3:.3e} mm  dMPJPE {abs(mp(y) - mp(ref)) * 1e3:.3e} mm")
    print(f"split vs f64:         max {np.abs(y - ref64).max() * 1e3:.3e} mm  dMPJPE {abs(mp(y) - mp(ref64)) * 1e3:.3e} mm")
    print(f"fp32 oracle vs f64:   max {np.abs(ref - ref64).max() * 1e3:.3e} mm  dMPJPE {abs(mp(ref) - mp(ref64)) * 1e3:.3e} mm")
    r64 = ref64.astype(np.float64)
    rr = float(np.sum(r64 * r64))
    for name, v in (("split", y), ("fp32 oracle", ref)):
        d = v.astype(np.float64) - r64
        print(f"{name:12s} vs f64: scale eps {np.sum(d * r64) / rr * 2 ** 24:+.2f} x 2^-24, "
              f"rms {np.sqrt(np.sum(d * d) / rr) * 2 ** 24:.2f} x 2^-24")


if __name__ == "__main__":
    main()
