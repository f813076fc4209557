"""Where one served frame's latency goes (config 5, layer-pipelined serve form).

Serves frames one at a time (post -> wait) with VP3D_STREAM_TRACE set, then reads the
per-workgroup device clocks (vp3d_stream_trace) and prints, per frame and then as medians,
the time from the expand role seeing the frame to each role's LAST workgroup having its
input complete / its output stored, plus the host wall time of the whole round trip.

    python tools/stream_latency.py [--frames 64] [--channels 1024] [--out gpurun_out/x.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dynamic-camera-augmented-videopose3d_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--channels", type=int, default=1024)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    os.environ["VP3D_STREAM_TRACE"] = str(a.frames)
    from common.models.TemporalModel import TemporalModel
    from vp3d_amd import synth
    from vp3d_amd.stream import CausalStream

    dev = torch.device("cuda", 0)
    model = TemporalModel(17, 2, 17, [3, 3, 3, 3, 3], causal=True, channels=a.channels)
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()], seed=0)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.eval().cuda()
    st = CausalStream(model.native_lifter(dev), "fp16")
    assert st.mode == "pipe", st.mode
    frames = np.random.RandomState(0).uniform(-1, 1, (a.frames, 17 * 2)).astype(np.float32)
    wall, native = [], []
    with st.serve(idle_ms=200.0) as sv:
        for i in range(a.frames):
            t0 = time.perf_counter_ns()
            sv.step(frames[i])
            wall.append((time.perf_counter_ns() - t0) * 1e-3)
            native.append(sv.last_latency_us)
    clk, first = st.trace()
    st.close()
    names = ["expand"] + [f"{k}{b}" for b in range(1, (len(first) - 3) // 2 + 1) for k in ("k", "p")] + ["shrink"]
    rows = []
    for s in range(a.frames):
        t_exp = clk[first[0]:first[1], s, 0]
        if not t_exp.all():
            continue
        base = int(t_exp.min())
        r = {"wall_us": wall[s], "native_us": native[s]}
        for i, n in enumerate(names):
            c = clk[first[i]:first[i + 1], s].astype(np.int64)
            if not c[:, 0].all():
                break
            outs = c[:, 1:9]
            outs = outs[outs > 0]  # waves that recorded a store
            # (last input, last store of any wave, first input, first store)
            r[n] = ((int(c[:, 0].max()) - base) / 100.0, (int(outs.max()) - base) / 100.0,
                    (int(c[:, 0].min()) - base) / 100.0, (int(outs.min()) - base) / 100.0)
        # shader clock of wave 0 between its input and output marks, every workgroup
        cl = clk[:, s].astype(np.int64)
        ok = (cl[:, 1] > cl[:, 0]) & (cl[:, 10] > cl[:, 9])
        if ok.any():
            r["sclk_mhz"] = float(np.median((cl[ok, 10] - cl[ok, 9]) / ((cl[ok, 1] - cl[ok, 0]) / 100.0)))
        rows.append(r)
    skip = min(8, len(rows) // 2)  # first frames: weights to VGPRs, clocks up
    steady = rows[skip:]
    med = {k: float(np.median([r[k] for r in steady])) for k in ("wall_us", "native_us")}
    for n in names:
        if all(n in r for r in steady):
            med[n] = tuple(float(np.median([r[n][k] for r in steady])) for k in range(4))
    print("role: input complete / output stored by the LAST (first) workgroup or wave of the role, us after the "
          f"first expand workgroup had the frame (median of {len(steady)} frames)")
    prev = 0.0
    for n in names:
        if n in med:
            i, o, i0, o0 = med[n]
            print(f"  {n:7s} in {i:7.2f} ({i0:6.2f})  out {o:7.2f} ({o0:6.2f})   "
                  f"(hand-off {i - prev:5.2f}, compute {o - i:5.2f})")
            prev = o
    sc = [r["sclk_mhz"] for r in steady if "sclk_mhz" in r]
    if sc:
        med["sclk_mhz"] = float(np.median(sc))
        print(f"  shader clock while a workgroup computes a frame: {med['sclk_mhz']:.0f} MHz (s_memtime / s_memrealtime)")
    print(f"  host wall (post -> pose in host memory): library {med['native_us']:.2f} us, "
          f"with the Python call {med['wall_us']:.2f} us")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"median": med, "frames": rows, "names": names, "role_first_wg": first.tolist()}, f, indent=1)


if __name__ == "__main__":
    main()
