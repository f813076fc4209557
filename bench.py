#!/usr/bin/env python3
"""Headline benchmark: 3D poses/s of the 243-frame-RF, 17-joint, 1024-channel
TemporalModelOptimized1f lifter on MI355X (BASELINE.json config 2; config 4
when launched with N > 1 ranks: the window batch is sharded, no collective).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--dtype bf16]

One step = one eval-mode forward of B independent 243-frame windows that are
already resident in HBM (B poses out).  Every rank processes its own B windows
(weak scaling); `value` = N*B*K / max-over-ranks(wall time of K steps).

Besides the JSON contract fields the line carries
  roofline      dominant kernel (block-1 k3 conv GEMM) FLOP per launch / its average
                HIP-event duration on the launch stream during the timed steps
  cpu_baseline  the oracle (the reference's torch-CPU op sequence) on this host
  parity        MPJPE delta vs the oracle on a window subset, fp32 and the timed dtype
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "dynamic-camera-augmented-videopose3d_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "3D poses/sec, 243-frame RF, 17 joints, 1024ch; MPJPE vs ref"
FW = [3, 3, 3, 3, 3]
CHANNELS = 1024
JOINTS = 17
PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3}  # MI355X dense (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="windows per GPU per step (8192; 1024 with --train)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--traj", action="store_true",
                    help="config 3: camera-trajectory conditioned input (46 ch) with the "
                         "on-device window gather inside the timed step")
    ap.add_argument("--stream", action="store_true",
                    help="config 5: causal streaming, one frame per step, hipGraph replay "
                         "(use --dtype fp16 and a large --steps)")
    ap.add_argument("--train", action="store_true",
                    help="training iteration (f32): TemporalModel train mode + backward + Adam; "
                         "--batch defaults to 1024 windows (run.py's batch_size)")
    ap.add_argument("--sequence", action="store_true",
                    help="sequence mode: dilated TemporalModel over one long sequence (run.py --evaluate "
                         "shape); --batch = output poses per step (default 65536)")
    ap.add_argument("--seq-model", choices=["transformer", "lstm"], default=None,
                    help="sliding-window eval of CoupledTransformer / CoupledLSTM (f32); --batch = poses "
                         "per step (default 16384)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="approximate CPU-baseline sample duration (0 disables)")
    ap.add_argument("--parity-windows", type=int, default=32)
    ap.add_argument("--settle-seconds", type=float, default=0.5,
                    help="untimed steps after --warmup until the device has run this long")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = 1024 if args.train else (16384 if args.seq_model else 65536 if args.sequence else 8192)
    return args


def synth_windows(B, T, jin, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    base = (torch.rand((B, 1, jin, 2), generator=g, device=device) - 0.5) * 1.2
    steps = torch.randn((B, T, jin, 2), generator=g, device=device) * 0.003
    return (base + torch.cumsum(steps, dim=1)).contiguous()


def stream_main(args, world, rank, dev):
    """Config 5: causal TemporalModel, one frame in / one pose out per step, the
    10-kernel step replayed from a hipGraph; HBM-bound weight streaming."""
    from common.models.TemporalModel import TemporalModel
    from oracle.temporal_ref import lifter_forward
    from vp3d_amd import synth
    from vp3d_amd.stream import CausalStream

    model = TemporalModel(JOINTS, 2, JOINTS, FW, causal=True, channels=CHANNELS)
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()], seed=0)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.eval().cuda()
    st = CausalStream(model.native_lifter(dev), args.dtype)
    s = torch.cuda.Stream(dev)
    fq, pr = st.io_tensors()
    Q = st.queue_len
    G = Q  # steps per graph launch: the whole frame queue
    # a synthetic clip fills the device frame queue; every step reads its own slot
    fq.copy_(synth_windows(1, Q, JOINTS, 1000 + rank, dev)[0].reshape(Q, -1))
    st.capture(s, steps=G)
    n_launch = max(1, -(-args.steps // G))
    n_warm = max(1, -(-args.warmup // G))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        for _ in range(n_warm):
            st.replay(s)
        s.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(s)
        for _ in range(n_launch):
            st.replay(s)
        ev1.record(s)
        s.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    args.steps = n_launch * G  # steps actually timed (whole graphs)
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank != 0:
        return
    # algorithmic bytes per step: every weight of the stack once (unpadded), step dtype
    wbytes = {"fp32": 4, "bf16": 2, "fp16": 2}[args.dtype]
    n_w = sum(v.size for k, v in sd.items() if (k.startswith("layers_conv") or k.startswith("expand_conv")
                                                 or k == "shrink.weight") and k.endswith("weight"))
    step_bytes = n_w * wbytes
    step_s = ev_ms * 1e-3 / args.steps
    achieved = step_bytes / step_s / 1e9
    # parity: first 64 frames of a stream vs the whole-sequence causal evaluation
    T = 64
    xs = synth_windows(1, T, JOINTS, 7, dev)
    st.reset()
    outs = torch.stack([st.step(xs[0, t]).clone() for t in range(T)]).cpu().numpy()
    pad = (RF_FULL - 1) // 2
    xp = torch.cat([xs[:, :1].expand(1, 2 * pad, -1, -1), xs], dim=1).cpu()
    ref = lifter_forward(sd, xp, FW, causal=True).numpy()[0]
    gt = synth.gt_poses(3, "stream_gt", T, JOINTS)

    def mp(a):
        return float(np.mean(np.linalg.norm(a.astype(np.float64) - gt, axis=-1)))
    cpu = None
    if args.cpu_seconds > 0:
        win = xp[:, :RF_FULL].contiguous()
        lifter_forward(sd, win, FW, causal=True)
        n, tc = 0, 0.0
        while tc < args.cpu_seconds:
            t1 = time.perf_counter()
            lifter_forward(sd, win, FW, causal=True)
            tc += time.perf_counter() - t1
            n += 1
        cpu = {"value": round(n / tc, 2), "unit": "poses/s", "cores": torch.get_num_threads(),
               "kind": "port", "sample": f"{n} single-frame causal steps (one 243-frame window "
                                         f"through the torch-CPU restatement each) in {tc:.1f} s"}
    out = {
        "metric": METRIC, "value": round(world * args.steps / dt, 2), "unit": "poses/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (seeded random-walk 2D frames, counter-hash weights)",
        "config": {"workload": "config5 causal streaming TemporalModel 243-frame RF, 17 joints, "
                               "1024 ch, one frame per step (10 GEMV launches), hipGraph of "
                               f"{G} consecutive steps fed from the device frame queue",
                   "frames_per_step": 1, "steps_per_graph": G, "parallelism": f"replicas{world}"},
        "roofline": {"bound": "hbm", "kernel": "stream step (10 stream_gemv launches)",
                     "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(achieved / 8000.0, 4), "traffic": None,
                     "bytes_per_step": step_bytes, "avg_step_us": round(step_s * 1e6, 3)},
        "cpu_baseline": cpu,
        "parity": {"frames": T, f"{args.dtype}_max_coord_delta_mm": float(np.abs(outs - ref).max()) * 1e3,
                   f"{args.dtype}_mpjpe_delta_mm": abs(mp(outs) - mp(ref)) * 1e3},
    }
    if cpu:
        out["speedup_vs_cpu"] = round(out["value"] / cpu["value"], 1)
    print(json.dumps(out), flush=True)


RF_FULL = 243


def train_flop_per_window(T, fw=FW, cin=2 * JOINTS, channels=CHANNELS, jout=JOINTS):
    """Algorithmic FLOP of one training iteration of the dilated TemporalModel on one
    window of T frames: forward convs + weight gradients + input gradients (none for the
    expand conv, whose input is data).  2 x MACs, BN/ReLU/dropout/Adam excluded."""
    L = T - (fw[0] - 1)
    fwd = wg = dg = 2 * L * channels * cin * fw[0]
    wg = fwd
    dg = 0
    dil = fw[0]
    for w in fw[1:]:
        L = L - (w - 1) * dil
        k = 2 * L * channels * channels * w + 2 * L * channels * channels
        fwd += k
        wg += k
        dg += k
        dil *= w
    s = 2 * L * channels * jout * 3
    return fwd + s, wg + s, dg + s


def train_main(args, world, rank, dev):
    """Training throughput: the reference's iteration (run.py:451-487) — TemporalModel
    (dilated, 3,3,3,3,3, 1024 ch, dropout 0.25) in train mode on B windows of 243 frames
    (run.py:666: ChunkedGenerator(batch_size // stride) with stride 1), mpjpe, backward,
    Adam(amsgrad) (run.py:662) — f32 on the native trainer.  N > 1 ranks: data-parallel,
    gradients averaged with one all_reduce per step (RCCL)."""
    from common.models.TemporalModel import TemporalModel
    from vp3d_amd import synth
    from vp3d_amd.train import Adam

    model = TemporalModel(JOINTS, 2, JOINTS, FW, channels=CHANNELS, dropout=0.25)
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()], seed=0)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.cuda().train()
    opt = Adam(model.parameters(), lr=1e-3, amsgrad=True)
    RF = model.receptive_field()
    B = args.batch
    x = synth_windows(B, RF, JOINTS, 1000 + rank, dev)
    tgt = (torch.randn((B, 1, JOINTS, 3), device=dev) * 0.2).contiguous()
    from common.loss import mpjpe
    from vp3d_amd.shard import allreduce_gradients
    params = [p for p in model.parameters()]
    bucket = [None]

    def step():
        y = model(x)
        loss = mpjpe(y, tgt)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        # data parallel: one all_reduce of one flat gradient bucket (68 MB, RCCL)
        bucket[0] = allreduce_gradients(params, bucket[0])
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank != 0:
        return
    fwd, wg, dg = train_flop_per_window(RF)
    flop_step = (fwd + wg + dg) * B
    windows_s = world * B * args.steps / dt
    out = {
        "metric": "training windows/sec (TemporalModel 243-frame RF, 17 joints, 1024ch, f32)",
        "value": round(windows_s, 2), "unit": "windows/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded windows, counter-hash weights)",
        "config": {"workload": "training iteration run.py:451-487: TemporalModel train mode (BN batch stats, "
                               "dropout 0.25) + mpjpe + backward + Adam(amsgrad)",
                   "windows_per_gpu": B, "global_batch": B * world,
                   "parallelism": f"dp{world}" + (" (gradient all_reduce, RCCL)" if world > 1 else "")},
        "flop_per_window": fwd + wg + dg,
        "tflops_effective": round(flop_step * world * args.steps / dt / 1e12, 2),
        "loss_last": float(loss.item()),
    }
    if args.cpu_seconds > 0:
        out["cpu_baseline"] = train_cpu_baseline(sd, RF, args.cpu_seconds)
    print(json.dumps(out), flush=True)


def train_cpu_baseline(sd, RF, seconds):
    """The oracle's training iteration (reference op sequence, torch-CPU autograd + Adam) on
    a bounded sample: batches of 8 windows until ~`seconds` elapse."""
    from oracle.train_ref import TrainLoop
    threads = torch.get_num_threads()
    loop = TrainLoop(sd, FW, lr=1e-3, amsgrad=True)
    rng = np.random.default_rng(0)
    Bc = 8
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        x = (rng.standard_normal((Bc, RF, JOINTS, 2)) * 0.3).astype(np.float32)
        tg = (rng.standard_normal((Bc, 1, JOINTS, 3)) * 0.2).astype(np.float32)
        loop.step(x, tg)
        n += Bc
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 3), "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": f"{n} windows (batches of {Bc}, dropout 0) through the oracle's training iteration "
                      f"(oracle/train_ref.py: torch-CPU autograd + Adam) in {dt:.1f} s"}


def seq_flop_per_pose(kind, W=243, d=128, layers=2, ff=128, heads=4, head=(128, 128, 128), cin=46, jout=51,
                      shared_projection=True):
    """Algorithmic FLOP of one sliding-window pose of CoupledTransformer / CoupledLSTM at the
    run.py defaults, as the native path evaluates it: the per-frame input projection once per
    frame (shared by the W windows that contain it), the last encoder layer for the last
    query only (the model keeps enc_out[:, -1]); softmax/LayerNorm/activations excluded."""
    if kind == "transformer":
        f = 2 * cin * d  # input projection, one new frame per window
        for l in range(layers):
            last = l == layers - 1
            f += 2 * W * d * 3 * d                                   # q, k, v projections
            q = 1 if last else W
            f += 2 * 2 * q * W * d                                   # q k^T and p v
            f += 2 * q * d * d + 2 * 2 * q * d * ff                  # out proj, feed-forward
    else:
        H = d
        f = 2 * cin * 4 * H
        f += W * 2 * (4 * H * H)                                     # layer-0 recurrence
        f += (layers - 1) * W * 2 * (2 * 4 * H * H)                  # upper cells: input + recurrence
    w = d
    for h in head:
        f += 2 * w * h
        w = h
    f += 2 * w * jout
    return f


def seq_main(args, world, rank, dev):
    """Sliding-window evaluation of the trajectory lifters: one step
    = model.sliding_window over one padded sequence of N + 242 frames -> N poses
    (run.py:713), CoupledTransformer / CoupledLSTM at the run.py defaults, f32."""
    from vp3d_amd import synth
    kind = args.seq_model
    torch.manual_seed(0)
    if kind == "transformer":
        from common.models.CamTransformer import CoupledTransformer
        model = CoupledTransformer(JOINTS, 2, JOINTS, 3, 128, 2, 4, 128, [128, 128, 128])
    else:
        from common.models.CamLSTM import CoupledLSTM
        model = CoupledLSTM(JOINTS, 2, JOINTS, 3, 128, 2, [128, 128, 128])
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    model.cuda().eval()
    W = 243
    N = args.batch
    L = N + W - 1
    x2 = synth_windows(1, L, JOINTS, 1000 + rank, dev)
    xc = (torch.randn((1, L, 3, 4), device=dev) * 0.5).contiguous()
    lifter = model.native_lifter(dev)
    with torch.no_grad():
        for _ in range(args.warmup):
            y = lifter.sliding_window(x2, xc, W)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            y = lifter.sliding_window(x2, xc, W)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank != 0:
        return
    flop = seq_flop_per_pose(kind)
    poses_s = world * N * args.steps / dt
    out = {
        "metric": f"3D poses/sec, {'CoupledTransformer' if kind == 'transformer' else 'CoupledLSTM'} sliding window "
                  "(243-frame window, 17 joints, camera-trajectory input)",
        "value": round(poses_s, 2), "unit": "poses/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded sequence, torch-default-init weights)",
        "config": {"workload": f"sliding_window of {kind} over {L} frames (run.py:713)", "poses_per_step": N,
                   "parallelism": f"dp{world} (independent sequences)"},
        "flop_per_pose": flop, "tflops_effective": round(poses_s * flop / 1e12, 3),
    }
    if args.cpu_seconds > 0:
        from oracle.seq_lifter_ref import lstm_forward, sliding_windows, transformer_forward
        threads = torch.get_num_threads()
        n = 0
        x2c, xcc = x2.cpu(), xc.cpu()
        t0 = time.perf_counter()
        pos = 0
        while time.perf_counter() - t0 < args.cpu_seconds and pos + 64 <= N:
            w2, wc = sliding_windows(x2c[:, pos:pos + 64 + W - 1], xcc[:, pos:pos + 64 + W - 1], W)
            if kind == "transformer":
                transformer_forward(sd, w2, wc, 4, 2, 3)
            else:
                lstm_forward(sd, w2, wc, 128, 2, 3)
            n += 64
            pos += 64
        dtc = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n / dtc, 2), "unit": "poses/s", "cores": threads, "kind": "port",
                               "sample": f"{n} sliding windows (batches of 64) through oracle/seq_lifter_ref.py "
                                         f"(torch-CPU, the reference's op sequence) in {dtc:.1f} s"}
    print(json.dumps(out), flush=True)


def sequence_main(args, world, rank, dev):
    """Sequence mode (SURVEY.md §8(d) "also report"): the dilated TemporalModel over one
    long edge-padded sequence, the run.py --evaluate shape (UnchunkedGenerator, B = 1,
    T_out + 242 frames in, T_out poses out); bf16 by default.  FLOP(T_out) =
    2 * (16,933,888 * T_out + 2,591,981,568)."""
    from common.models.TemporalModel import TemporalModel
    from oracle.temporal_ref import lifter_forward
    from vp3d_amd import synth

    model = TemporalModel(JOINTS, 2, JOINTS, FW, channels=CHANNELS)
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()], seed=0)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.eval().cuda().set_compute_dtype(args.dtype)
    RF = model.receptive_field()
    T_out = args.batch
    x = synth_windows(1, T_out + RF - 1, JOINTS, 1000 + rank, dev)
    lifter = model.native_lifter(dev)
    lifter.reserve(1, T_out + RF - 1, args.dtype)
    y = torch.empty((1, T_out, JOINTS, 3), device=dev)
    with torch.no_grad():
        for _ in range(args.warmup):
            lifter.forward(x, args.dtype, out=y)
        torch.cuda.synchronize()
        lifter.profile(True)
        lifter.profile_reset()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            lifter.forward(x, args.dtype, out=y)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        lifter.profile(False)
    prof = lifter.profile_read()
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank != 0:
        return
    value = world * T_out * args.steps / dt
    flop_step = 2 * (16933888 * T_out + 2591981568)
    dom = max(prof, key=lambda r: r["ms_total"])
    dom_ms = dom["ms_total"] / max(dom["launches"], 1)
    names = ["expand"] + [f"block{(i // 2) + 1}_{'k3' if i % 2 == 0 else '1x1'}"
                          for i in range(2 * (len(FW) - 1))] + ["shrink"]
    # parity on the first 256 output frames (a time shard: inputs [0, 256 + RF - 1))
    P = min(256, T_out)
    ref = lifter_forward(sd, x[:, :P + RF - 1].cpu(), FW).numpy()
    got = y[:, :P].cpu().numpy()
    out = {
        "metric": "3D poses/sec, dilated TemporalModel sequence mode (243-frame RF, 17 joints, 1024ch)",
        "value": round(value, 2), "unit": "poses/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded random-walk sequence, counter-hash weights)",
        "config": {"workload": f"TemporalModel (dilated) on one sequence of {T_out + RF - 1} frames -> {T_out} poses "
                               "(run.py --evaluate, UnchunkedGenerator)", "poses_per_step": T_out,
                   "parallelism": f"dp{world} (independent sequences)"},
        "flop_per_step": flop_step, "tflops_effective": round(value / T_out * flop_step / 1e12, 2),
        "roofline": {"bound": "mfma", "kernel": f"conv_gemm ({names[dom['layer']]})",
                     "achieved": round(dom["flop"] / (dom_ms * 1e-3) / 1e12, 2), "peak": PEAK_TFLOPS[args.dtype],
                     "unit": "TFLOP/s", "frac": round(dom["flop"] / (dom_ms * 1e-3) / 1e12 / PEAK_TFLOPS[args.dtype], 4),
                     "traffic": None, "avg_launch_ms": round(dom_ms, 4), "flop_per_launch": dom["flop"]},
        "per_layer_ms": {names[r["layer"]]: round(r["ms_total"] / max(r["launches"], 1), 4) for r in prof},
        "parity": {"frames_checked": P, "max_coord_delta_mm": float(np.abs(got - ref).max()) * 1e3},
    }
    if args.cpu_seconds > 0:
        nthr = torch.get_num_threads()
        Tc = 2048
        xc = x[:, :Tc + RF - 1].cpu()
        n, t_cpu = 0, 0.0
        while t_cpu < args.cpu_seconds:
            t1 = time.perf_counter()
            lifter_forward(sd, xc, FW)
            t_cpu += time.perf_counter() - t1
            n += Tc
        out["cpu_baseline"] = {"value": round(n / t_cpu, 2), "unit": "poses/s", "cores": nthr, "kind": "port",
                               "sample": f"{n} poses as sequences of {Tc + RF - 1} frames through oracle/temporal_ref.py "
                                         f"(torch-CPU, fp32) in {t_cpu:.1f} s"}
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VP3D_BENCH_REHEARSE=1: rehearse the N-rank path on a box with fewer GPUs (ranks share
    # devices round-robin, gloo instead of RCCL); never used for reported numbers
    rehearse = os.environ.get("VP3D_BENCH_REHEARSE") == "1"
    if rehearse:
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        # the CPU baseline is a single-GPU (N = 1) figure: under torchrun every rank gets
        # OMP_NUM_THREADS=1 and the node's cores are shared by N processes
        args.cpu_seconds = 0.0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if args.stream or args.train or args.seq_model or args.sequence:
        fn = (train_main if args.train else seq_main if args.seq_model else
              sequence_main if args.sequence else stream_main)
        fn(args, world, rank, dev)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    from common.models.TemporalModel import TemporalModelOptimized1f
    from vp3d_amd import synth

    jin = 23 if args.traj else JOINTS
    model = TemporalModelOptimized1f(jin, 2, JOINTS, FW, channels=CHANNELS)
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()], seed=0)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.eval().cuda()
    model.set_compute_dtype(args.dtype)
    RF = model.receptive_field()
    B = args.batch

    pipe = None
    if args.traj:
        from vp3d_amd.pipeline import SyntheticTrajectoryBatcher
        pipe = SyntheticTrajectoryBatcher(B, RF, seed=1000 + rank, device=dev)
        x = None
    else:
        x = synth_windows(B, RF, jin, 1000 + rank, dev)
    lifter = model.native_lifter(dev)
    lifter.reserve(B, RF, args.dtype)
    y = torch.empty((B, 1, JOINTS, 3), device=dev)

    last_in = [x]

    def step():
        if pipe is not None:
            # config 3: K.E of every frame + window gather + camera concat + forward,
            # the gather fused into the expand conv's operand loads
            pairs = pipe.next_pairs()
            lifter.forward_windows(pipe.seqs, pairs, RF, pipe.pad, concat_cams=True, dtype=args.dtype,
                                   out=y)
            last_in[0] = pairs
        else:
            lifter.forward(x, args.dtype, out=y)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        # then untimed steps until the device has been busy for ~0.5 s: after a cold
        # start (the trajectory setup leaves the GPU idle for seconds) the step period
        # falls from ~5.8 to ~3.2 ms over the first ~20 steps as the clocks ramp
        # (profiles/r01f_traj_step_ramp.txt), which a 5-step warm-up does not cover
        torch.cuda.synchronize()
        t_settle = time.perf_counter()
        while time.perf_counter() - t_settle < args.settle_seconds:
            step()
            torch.cuda.synchronize()
        # per-layer times from an untimed pass with events around every launch; the timed
        # loop below carries events around the dominant layer only (events on all ten
        # launches cost ~75 us per step)
        lifter.profile(True)
        lifter.profile_layers(None)
        lifter.profile_reset()
        for _ in range(min(args.steps, 10)):
            step()
        layer_prof = lifter.profile_read()
        dom_layer = max(layer_prof, key=lambda r: r["ms_total"])["layer"]
        lifter.profile_layers([dom_layer])
        lifter.profile_reset()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        lifter.profile(False)
        lifter.profile_layers(None)
    prof = lifter.profile_read()

    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    total_poses = world * B * args.steps
    value = total_poses / dt
    # dominant kernel: its HIP-event duration over the timed steps
    dom = prof[dom_layer]
    dom_avg_ms = max(dom["ms_total"] / max(dom["launches"], 1), 1e-9)
    achieved = dom["flop"] / (dom_avg_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    layer_names = ["expand"] + [f"block{(i // 2) + 1}_{'k3' if i % 2 == 0 else '1x1'}"
                                for i in range(2 * (len(FW) - 1))] + ["shrink"]
    per_layer = {layer_names[r["layer"]]: round(r["ms_total"] / max(r["launches"], 1), 4)
                 for r in layer_prof}

    out = None
    if rank == 0:
        # ---- parity on a window subset (oracle = reference op sequence on CPU) ----
        from oracle.temporal_ref import lifter_forward
        # the timed kernels' own output (last timed step, full batch B) on the first
        # P windows, plus the fp32 parity path on the same windows
        P = min(args.parity_windows, B)
        idx = torch.cat([torch.arange(P // 2), torch.arange(B - (P - P // 2), B)]).to(dev)
        xfull = pipe.gather(last_in[0]) if pipe is not None else last_in[0]
        xs = xfull[idx].contiguous()
        y_fast = y[idx].cpu().numpy()
        with torch.no_grad():
            model.set_compute_dtype("fp32")
            y_32 = model(xs).cpu().numpy()
            model.set_compute_dtype(args.dtype)
        ref = lifter_forward(sd, xs.cpu(), FW, strided=True).numpy()
        gt = synth.gt_poses(3, "bench_gt", P, JOINTS).reshape(ref.shape)

        def mp(a):
            return float(np.mean(np.linalg.norm(a.astype(np.float64) - gt, axis=-1)))
        parity = {
            "windows": P,
            "windows_checked": "first and last half of the timed batch (timed kernels' output)",
            "mpjpe_ref_mm": round(mp(ref) * 1e3, 6),
            "fp32_mpjpe_delta_mm": abs(mp(y_32) - mp(ref)) * 1e3,
            "fp32_max_coord_delta_mm": float(np.abs(y_32 - ref).max()) * 1e3,
            f"{args.dtype}_mpjpe_delta_mm": abs(mp(y_fast) - mp(ref)) * 1e3,
            f"{args.dtype}_max_coord_delta_mm": float(np.abs(y_fast - ref).max()) * 1e3,
        }

        # ---- CPU baseline: the oracle on a bounded sample of the same workload ----
        cpu = None
        if args.cpu_seconds > 0:
            nthr = torch.get_num_threads()
            cb = 64
            xc = xs[:1].cpu().expand(cb, -1, -1, -1).contiguous()
            lifter_forward(sd, xc[:8], FW, strided=True)  # warm-up
            n, t_cpu = 0, 0.0
            while t_cpu < args.cpu_seconds:
                t1 = time.perf_counter()
                lifter_forward(sd, xc, FW, strided=True)
                t_cpu += time.perf_counter() - t1
                n += cb
            cpu = {"value": round(n / t_cpu, 2), "unit": "poses/s", "cores": nthr, "kind": "port",
                   "sample": f"{n} windows of 243x17x2 through the torch-CPU restatement "
                             f"(oracle/temporal_ref.py, fp32, batch {cb}) in {t_cpu:.1f} s"}

        traffic = None
        tfile = os.path.join(REPO, "profiles", f"traffic_{args.dtype}_b{B}.json")
        if os.path.exists(tfile):
            with open(tfile) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")

        flop_pose = 358541312 if args.traj else 352569344
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "poses/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (seeded random-walk 2D windows, counter-hash weights)",
            "config": {
                "workload": ("config3 trajectory-conditioned (46ch) " if args.traj else "config2 ")
                            + "TemporalModelOptimized1f 243-frame RF windows, 17 joints, 1024 ch",
                "windows_per_gpu": B,
                "global_batch": B * world,
                "parallelism": f"dp{world} (independent window shards, no collective)",
                "flop_per_pose": flop_pose,
            },
            "tflops_effective": round(value * flop_pose / 1e12, 2),
            "roofline": {
                "bound": "mfma",
                "kernel": f"conv_gemm ({layer_names[dom['layer']]})",
                "achieved": round(achieved, 2),
                "peak": peak,
                "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4),
                "traffic": traffic,
                "avg_launch_ms": round(dom_avg_ms, 4),
                "launches_timed": dom["launches"],
                "flop_per_launch": dom["flop"],
            },
            "per_layer_ms": per_layer,
            "per_layer_note": "untimed pass with HIP events around every launch",
            "cpu_baseline": cpu,
            "parity": parity,
        }
        if cpu:
            out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
