#!/usr/bin/env python3
"""Headline benchmark: 3D poses/s of the 243-frame-RF, 17-joint, 1024-channel
TemporalModelOptimized1f lifter on MI355X (BASELINE.json configs 2 and 4).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch 65536 | --batch B] [--dtype f16x3]

One step = one eval-mode forward of the global batch of 243-frame windows (65,536 by
default: config 4), sharded over the N ranks by vp3d_amd.shard.shard_range, every
rank's shard gathered on device from one seeded window set and resident in HBM before
the timed region (strong scaling; N = 1 is the single-GPU config-2/4 point), in the
split-fp16 path (f16x3: the north-star MPJPE tolerance at 16-bit MFMA rates).
`value` = G*K / max-over-ranks(wall time of K steps).  --batch B instead gives every
rank its own B windows (weak scaling).

At N = 1 the line also carries, each with its own roofline, parity and CPU baseline:
  bf16, fp32    config 2's dtype and the exact parity path on the same windows
  batch_sweep_poses_per_s   B = 1,024 / 8,192 / 65,536 in f16x3 and bf16
  config3       trajectory-conditioned windows (K.E + gather + concat in the step): fp16,
                f16x3, fp32
  config5       causal streaming, fp32 (exact weights, the north-star gate) and fp16 (config 5's
                dtype): the hipGraph-pipelined step and one frame in flight (serve latency
                p50 / p90 / p99)
  sequence      the dilated TemporalModel over one 65,778-frame sequence (run.py --evaluate's
                shape) in f16x3 and fp32 (the gate) and bf16, with ΔMPJPE vs the oracle
Besides the JSON contract fields the line carries
  roofline      dominant kernel (block-1 k3 conv GEMM) FLOP per launch / its average
                HIP-event duration on the launch stream during the timed steps; traffic =
                the committed PMC summary of the same build (null if the build differs)
  cpu_baseline  the oracle (the reference's torch-CPU op sequence) on this host
  parity        MPJPE delta vs the oracle on a window subset, every dtype
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
# MI355X dense peaks (MI355X_MICROARCH.md); f16x3 (split fp16) issues three f16 MFMA products
# per algorithmic multiply-add, so its algorithmic-FLOP ceiling is the f16 peak / 3
PEAK_TFLOPS = {"bf16": 2500.0, "fp16": 2500.0, "fp32": 157.3, "f16x3": 2500.0 / 3}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--global-batch", type=int, default=65536,
                    help="windows per step over all ranks (config 4: sharded with shard_range; strong scaling)")
    ap.add_argument("--batch", type=int, default=None,
                    help="windows per GPU per step instead of --global-batch (weak scaling); the per-step "
                         "unit count of --train / --sequence / --seq-model")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp16", "fp32", "f16x3"],
                    help="default: f16x3 (configs 2/4: split fp16, fp32-level accuracy on the 16-bit MFMAs), "
                         "fp16 (--traj, --stream)")
    ap.add_argument("--sweep", type=lambda v: [int(t) for t in v.split(",") if t], default=[1024, 8192, 65536],
                    help="config-2 batch sweep on one GPU (windows per step)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip every leg (the other dtypes, the sweep, configs 3 and 5) and the CPU baseline")
    ap.add_argument("--no-legs", action="store_true", help="skip the config-3 and config-5 legs of the default line")
    ap.add_argument("--pregathered", action="store_true",
                    help="configs 2/4: time the forward over a window tensor gathered once before the "
                         "timed region (the reference's form: batch built outside the model) instead of "
                         "the batch assembly + forward of the default step")
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
                    help="approximate CPU-baseline duration over its 5 timed runs (0 disables)")
    ap.add_argument("--parity-windows", type=int, default=32)
    ap.add_argument("--settle-seconds", type=float, default=0.5,
                    help="untimed steps after --warmup until the device has run this long")
    args = ap.parse_args()
    if args.batch is None and (args.train or args.seq_model or args.sequence):
        args.batch = 1024 if args.train else (16384 if args.seq_model else 65536)
    return args


def synth_windows(B, T, jin, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    base = (torch.rand((B, 1, jin, 2), generator=g, device=device) - 0.5) * 1.2
    steps = torch.randn((B, T, jin, 2), generator=g, device=device) * 0.003
    return (base + torch.cumsum(steps, dim=1)).contiguous()


def stream_traffic(mode):
    """HBM bytes per pipelined step (graph of 64) of the stream kernel from the committed PMC
    summary (profiles/r03prof_stream_traffic.json: FETCH_SIZE x 2 + WRITE_SIZE per graph
    launch / 64: the weights once per launch plus the hand-off polls), or None."""
    tfile = os.path.join(REPO, "profiles", "r03prof_stream_traffic.json")
    if mode != "pipe" or not os.path.exists(tfile):
        return None
    with open(tfile) as f:
        return json.load(f).get("per_step_in_graph_bytes")


def stream_main(args, world, rank, dev, emit=True):
    """Config 5: causal TemporalModel, one frame in / one pose out per step.  A graph of Q
    steps is ONE persistent launch -- by default the layer-pipelined form (each CU runs one
    layer with its weights in VGPRs as f32: the exact fp32 weights for --dtype fp32, 16-bit
    ones widened for fp16 / bf16; the frames of the graph flow through the layer groups;
    VP3D_STREAM_MODE=persist: every CU runs every layer with its 16-bit weights in LDS,
    =launches: 10 GEMV launches per step)."""
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
    mode = st.mode
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
    step_flop = 2 * n_w  # one multiply-add per weight per step (algorithmic; 33,867,776 FLOP at 1024 ch)
    step_s = ev_ms * 1e-3 / args.steps
    achieved = step_bytes / step_s / 1e9
    # parity: first 64 frames of a stream vs the whole-sequence causal evaluation
    T = 64
    xs = synth_windows(1, T, JOINTS, 7, dev)
    st.check()
    st.reset()
    outs = torch.stack([st.step(xs[0, t]).clone() for t in range(T)]).cpu().numpy()
    st.check()
    # latency of ONE step from an idle stream (eager launch, frame already in the queue)
    lat = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        st.step(xs[0, 0])
        e1.record()
        e1.synchronize()
        lat.append(e0.elapsed_time(e1) * 1e3)
    # real-time serving, ONE frame in flight: host frame in -> host pose out, wall clock
    serve_lat = serve_py = None
    if mode == "pipe":
        frames_h = xs[0].cpu().numpy()
        serve_lat, serve_py = [], []
        with st.serve(idle_ms=200.0) as sv:
            for i in range(32 + 512):
                t0 = time.perf_counter_ns()
                sv.step(frames_h[i % T])
                if i >= 32:  # after the first frames (weights to VGPRs, clocks up)
                    serve_py.append((time.perf_counter_ns() - t0) * 1e-3)
                    serve_lat.append(sv.last_latency_us)
    pad = (RF_FULL - 1) // 2
    xp = torch.cat([xs[:, :1].expand(1, 2 * pad, -1, -1), xs], dim=1).cpu()
    ref = lifter_forward(sd, xp, FW, causal=True).numpy()[0]
    gt = synth.gt_poses(3, "stream_gt", T, JOINTS)

    def mp(a):
        return float(np.mean(np.linalg.norm(a.astype(np.float64) - gt, axis=-1)))
    cpu = getattr(args, "stream_cpu_baseline", None)
    if cpu is None and args.cpu_seconds > 0:
        win = xp[:, :RF_FULL].contiguous()
        cpu = cpu_baseline(cpu_job("lifter", sd, {"x": win}, fw=FW, causal=True), 1, "poses/s",
                           "single-frame causal steps (one 243-frame window through the torch-CPU "
                           "restatement each, B = 1)", target_s=args.cpu_seconds / 5)
    out = {
        "metric": METRIC, "value": round(world * args.steps / dt, 2), "unit": "poses/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (seeded random-walk 2D frames, counter-hash weights)",
        "config": {"workload": "config5 causal streaming TemporalModel 243-frame RF, 17 joints, "
                               "1024 ch, one frame per step, hipGraph of "
                               f"{G} consecutive steps fed from the device frame queue"
                               + {"pipe": " (one persistent launch, one layer per CU with its weights in VGPRs, "
                                          "frames pipelined through the layer groups)",
                                  "persist": " (one persistent launch: every CU runs every layer, weights in LDS)",
                                  "launches": " (10 GEMV launches per step)"}[mode],
                   "frames_per_step": 1, "steps_per_graph": G, "mode": mode, "parallelism": f"replicas{world}"},
        # the bound that applies: with the weights resident on chip (pipe: f32 in VGPRs,
        # persist: 16-bit in LDS) a step is f32 FMA work (v_pk_fma_f32) spread over the CUs and
        # chained through 10 layer hand-offs -- priced here against the f32 vector FMA peak; the
        # weight-streaming (HBM) view is kept beside it for the GEMV form
        "roofline": {"bound": "valu" if mode != "launches" else "hbm",
                     "kernel": {"pipe": "stream_pipe_kernel", "persist": "stream_persist_kernel",
                                "launches": "stream step (10 stream_gemv launches)"}[mode],
                     "achieved": round(step_flop / step_s / 1e12, 3) if mode != "launches" else round(achieved, 1),
                     "peak": 157.3 if mode != "launches" else 8000.0,
                     "unit": "TFLOP/s" if mode != "launches" else "GB/s",
                     "frac": round(step_flop / step_s / 1e12 / 157.3, 4) if mode != "launches"
                     else round(achieved / 8000.0, 4),
                     "traffic": stream_traffic(mode), "flop_per_step": step_flop,
                     "avg_step_us": round(step_s * 1e6, 3),
                     "note": ("achieved = the step's algorithmic FLOP (2 x MACs of the 10 convs) / the pipelined "
                              "step time (frames of a 64-step graph flowing through the layer groups); peak = "
                              "the f32 vector peak (157.3 TF spec, packed v_pk_fma_f32 -- the instruction the "
                              "kernel issues, on f32 weights resident in VGPRs). The per-frame floor is the "
                              "hand-off chain: one frame crosses 10 layer groups (serve_latency_us)."
                              if mode != "launches" else
                              "weights re-read every step: HBM-bound GEMVs"),
                     "hbm_view": {"bytes_per_step": step_bytes, "achieved_GBps": round(achieved, 1),
                                  "frac_of_8TBps": round(achieved / 8000.0, 4)}},
        "cpu_baseline": cpu,
        "single_step_latency_us": round(float(np.median(serve_lat if serve_lat else lat)), 2),
        "single_step_latency_note": ("serve form: one frame in flight, host frame posted to pinned memory -> pose "
                                     "back in host memory, the library's wall clock around post + wait "
                                     "(vp3d_stream_serve_step; resident launch), median of 512; "
                                     "serve_python_latency_us adds the Python/ctypes call" if serve_lat else
                                     "eager launch of one step from an idle stream (HIP events)"),
        "serve_latency_us": ({"median": round(float(np.median(serve_lat)), 2),
                              "p90": round(float(np.percentile(serve_lat, 90)), 2),
                              "p99": round(float(np.percentile(serve_lat, 99)), 2),
                              "frames_per_s_one_in_flight": round(1e6 / float(np.median(serve_lat)), 1)}
                             if serve_lat else None),
        "serve_python_latency_us": round(float(np.median(serve_py)), 2) if serve_py else None,
        "eager_step_latency_us": round(float(np.median(lat)), 2),
        "faults": 0,  # st.check() after the timed graphs and after the parity steps
        "parity": {"frames": T, f"{args.dtype}_max_coord_delta_mm": float(np.abs(outs - ref).max()) * 1e3,
                   f"{args.dtype}_mpjpe_delta_mm": abs(mp(outs) - mp(ref)) * 1e3,
                   "meets_north_star_1e-4mm": bool(abs(mp(outs) - mp(ref)) * 1e3 <= 1e-4),
                   "reference": "oracle/temporal_ref.py on the whole edge-padded sequence, causal "
                                "(generators.py:193-198, TemporalModel.py:126-138)"},
    }
    if cpu:
        out["speedup_vs_cpu"] = round(out["value"] / cpu["value"], 1)
    st.close()
    if emit:
        emit_line(out)
    return out


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
        # the step is a chain of f32 GEMMs (forward, dgrad, wgrad of every conv on the f32 MFMA)
        # plus HBM-bound BN / ReLU / dropout / Adam passes; priced as a whole against the f32
        # MFMA peak (per GPU), the GEMM-only share of the time is in profiles/ (rocprofv3)
        "roofline": {"bound": "mfma", "kernel": "whole training step (all launches)",
                     "achieved": round(flop_step * args.steps / dt / 1e12, 2), "peak": 157.3,
                     "unit": "TFLOP/s", "frac": round(flop_step * args.steps / dt / 1e12 / 157.3, 4),
                     "traffic": None,
                     "note": "algorithmic FLOP of the step (2 x MACs of forward + weight and input gradients, "
                             "BN / dropout / Adam excluded) / the step's wall time, per GPU"},
        "loss_last": float(loss.item()),
    }
    if args.cpu_seconds > 0:
        rng = np.random.default_rng(0)
        xb = (rng.standard_normal((8, RF, JOINTS, 2)) * 0.3).astype(np.float32)
        tb = (rng.standard_normal((8, 1, JOINTS, 3)) * 0.2).astype(np.float32)
        out["cpu_baseline"] = cpu_baseline(cpu_job("train", sd, {"x": xb, "tgt": tb}, fw=FW), 8, "windows/s",
                                           "training iterations on batches of 8 windows (dropout 0) through "
                                           "oracle/train_ref.py (torch-CPU autograd + Adam)",
                                           target_s=args.cpu_seconds / 5)
    emit_line(out)


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
    # parity: the first P poses (a time shard: frames [0, P + W - 1)) vs the oracle's sliding
    # window (oracle/seq_lifter_ref.py: CamTransformer.py:86-89 unfold + the eval forward)
    from oracle.seq_lifter_ref import lstm_forward, sliding_windows, transformer_forward
    P = min(64, N)
    w2, wc = sliding_windows(x2[:, :P + W - 1].cpu(), xc[:, :P + W - 1].cpu(), W)
    with torch.no_grad():
        ref = (transformer_forward(sd, w2, wc, 4, 2, 3) if kind == "transformer"
               else lstm_forward(sd, w2, wc, 128, 2, 3)).reshape(P, JOINTS, 3).numpy()
    got = y[0, :P].cpu().numpy()
    gt = synth.gt_poses(3, "seq_lifter_gt", P, JOINTS).reshape(ref.shape)

    def mp(a):
        return float(np.mean(np.linalg.norm(a.astype(np.float64) - gt, axis=-1)))
    achieved = poses_s / world * flop / 1e12
    out = {
        "metric": f"3D poses/sec, {'CoupledTransformer' if kind == 'transformer' else 'CoupledLSTM'} sliding window "
                  "(243-frame window, 17 joints, camera-trajectory input)",
        "value": round(poses_s, 2), "unit": "poses/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded sequence, torch-default-init weights)",
        "config": {"workload": f"sliding_window of {kind} over {L} frames (run.py:713)", "poses_per_step": N,
                   "parallelism": f"dp{world} (independent sequences)"},
        "flop_per_pose": flop, "tflops_effective": round(poses_s * flop / 1e12, 3),
        # every Linear (projections, attention in/out, feed-forward, LSTM gates, head) runs on the
        # f32 MFMA GEMM or the MFMA attention / LSTM kernels: the step is priced as a whole
        # against the f32 MFMA peak (per GPU), like --train
        "roofline": {"bound": "mfma", "kernel": "whole sliding_window step (all launches)",
                     "achieved": round(achieved, 3), "peak": 157.3, "unit": "TFLOP/s",
                     "frac": round(achieved / 157.3, 4), "traffic": None,
                     "note": "algorithmic FLOP per pose (seq_flop_per_pose: 2 x MACs of every Linear, QK^T and "
                             "PV, the input projection once per frame; softmax / LayerNorm / activations "
                             "excluded) x poses/s per GPU"},
        "faults": 0,
        "parity": {"poses_checked": P, "f32_max_coord_delta_mm": float(np.abs(got - ref).max()) * 1e3,
                   "f32_mpjpe_delta_mm": abs(mp(got) - mp(ref)) * 1e3,
                   "meets_north_star_1e-4mm": bool(abs(mp(got) - mp(ref)) * 1e3 <= 1e-4),
                   "reference": "oracle/seq_lifter_ref.py sliding windows (CamTransformer.py:72-205 / "
                                "CamLSTM.py:33-129, eval mode) on the same frames and weights"},
    }
    if args.cpu_seconds > 0:
        w2, wc = sliding_windows(x2[:, :64 + W - 1].cpu(), xc[:, :64 + W - 1].cpu(), W)
        fn = cpu_job(kind, sd, {"x": w2, "xc": wc})
        out["cpu_baseline"] = cpu_baseline(fn, 64, "poses/s", "64 sliding windows per run through "
                                           "oracle/seq_lifter_ref.py (torch-CPU, the reference's op sequence)",
                                           target_s=args.cpu_seconds / 5)
    emit_line(out)


class SequenceCase:
    """Sequence mode (SURVEY.md §8(d) "also report"): the dilated TemporalModel over one
    long edge-padded sequence, the run.py --evaluate shape (run.py:697-711: UnchunkedGenerator,
    B = 1, T_out + 242 frames in, T_out poses out).  FLOP(T_out) =
    2 * (16,933,888 * T_out + 2,591,981,568)."""

    def __init__(self, T_out, rank, dev):
        from common.models.TemporalModel import TemporalModel
        from vp3d_amd import synth
        model = TemporalModel(JOINTS, 2, JOINTS, FW, channels=CHANNELS)
        self.sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()], seed=0)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in self.sd.items()})
        model.eval().cuda()
        self.RF = model.receptive_field()
        self.T_out = T_out
        self.x = synth_windows(1, T_out + self.RF - 1, JOINTS, 1000 + rank, dev)
        self.lifter = model.native_lifter(dev)
        self.y = torch.empty((1, T_out, JOINTS, 3), device=dev)
        self.flop_step = 2 * (16933888 * T_out + 2591981568)
        self._ref = None

    def run(self, dtype, steps, warmup, settle_s, world):
        self.lifter.reserve(1, self.T_out + self.RF - 1, dtype)
        lifter, x, y = self.lifter, self.x, self.y

        def step():
            lifter.forward(x, dtype, out=y)
        with torch.no_grad():
            r = profiled_run(lifter, step, steps, warmup, settle_s, world)
        lifter.sync_status()  # raises on a device-side fault of any forward of the leg
        return r

    def parity(self, P=256):
        """The first P output frames (a time shard: inputs [0, P + RF - 1)) vs the oracle."""
        from oracle.temporal_ref import lifter_forward
        from vp3d_amd import synth
        P = min(P, self.T_out)
        if self._ref is None:
            ref = lifter_forward(self.sd, self.x[:, :P + self.RF - 1].cpu(), FW).numpy()
            gt = synth.gt_poses(3, "seq_gt", P, JOINTS).reshape(ref.shape)
            self._ref = (ref, gt)
        ref, gt = self._ref
        got = self.y[:, :P].cpu().numpy()

        def mp(a):
            return float(np.mean(np.linalg.norm(a.astype(np.float64) - gt, axis=-1)))
        return {"frames_checked": P, "mpjpe_delta_mm": abs(mp(got) - mp(ref)) * 1e3,
                "max_coord_delta_mm": float(np.abs(got - ref).max()) * 1e3,
                "meets_north_star_1e-4mm": bool(abs(mp(got) - mp(ref)) * 1e3 <= 1e-4)}

    def leg(self, dtype, steps, warmup, settle_s, world=1):
        dt, per_layer, dom = self.run(dtype, steps, warmup, settle_s, world)
        value = world * self.T_out * steps / dt
        r = roofline_of(dom, PEAK_TFLOPS[dtype])
        if dtype == "f16x3":
            r["peak_note"] = "f16 dense MFMA peak / 3: three f16 products per algorithmic multiply-add"
        return dt, {"value": round(value, 2), "unit": "poses/s", "steps": steps,
                    "ms_per_step": round(dt / steps * 1e3, 4),
                    "tflops_effective": round(value / self.T_out * self.flop_step / 1e12, 2),
                    "roofline": r, "per_layer_ms": per_layer, "faults": 0, **self.parity()}

    def cpu_baseline(self, seconds):
        Tc = 2048
        xc = self.x[:, :Tc + self.RF - 1].cpu()
        return cpu_baseline(cpu_job("lifter", self.sd, {"x": xc}, fw=FW), Tc, "poses/s",
                            f"one sequence of {Tc + self.RF - 1} frames -> {Tc} poses per run through "
                            "oracle/temporal_ref.py (torch-CPU, fp32)", target_s=seconds / 5)

    def close(self):
        self.lifter.close()
        self.x = self.y = None


def sequence_main(args, world, rank, dev):
    """--sequence: the dilated TemporalModel over one long sequence as the main line (bf16 by
    default; --dtype f16x3 / fp32 for the north-star gate)."""
    case = SequenceCase(args.batch, rank, dev)
    dt, leg = case.leg(args.dtype, args.steps, args.warmup, args.settle_seconds, world)
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank != 0:
        return
    T_out = case.T_out
    value = world * T_out * args.steps / dt
    out = {
        "metric": "3D poses/sec, dilated TemporalModel sequence mode (243-frame RF, 17 joints, 1024ch)",
        "value": round(value, 2), "unit": "poses/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded random-walk sequence, counter-hash weights)",
        "config": {"workload": f"TemporalModel (dilated) on one sequence of {T_out + case.RF - 1} frames -> {T_out} "
                               "poses (run.py --evaluate, UnchunkedGenerator)", "poses_per_step": T_out,
                   "parallelism": f"dp{world} (independent sequences)"},
        "flop_per_step": case.flop_step, "tflops_effective": round(value / T_out * case.flop_step / 1e12, 2),
        "roofline": leg["roofline"], "per_layer_ms": leg["per_layer_ms"],
        "faults": leg["faults"],
        "parity": {k: leg[k] for k in ("frames_checked", "mpjpe_delta_mm", "max_coord_delta_mm",
                                       "meets_north_star_1e-4mm")},
    }
    if args.cpu_seconds > 0:
        out["cpu_baseline"] = case.cpu_baseline(args.cpu_seconds)
        out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
    case.close()
    emit_line(out)


# keys the driver must see: it keeps only the TAIL of stdout, so the headline's own timing,
# roofline, CPU baseline, fault count and parity go last, after the (long) legs
TAIL_KEYS = ("per_layer_ms", "per_layer_note", "tflops_effective", "roofline", "cpu_baseline", "speedup_vs_cpu",
             "faults", "faults_note", "parity")


def emit_line(out):
    """Print the ONE JSON line of this run, the contract fields first and TAIL_KEYS last."""
    head = {k: v for k, v in out.items() if k not in TAIL_KEYS}
    head.update({k: out[k] for k in TAIL_KEYS if k in out})
    print(json.dumps(head), flush=True)


def host_cpu_info():
    """CPU model and core counts of this host (/proc/cpuinfo)."""
    model, cores, logical = None, set(), 0
    try:
        phys = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    logical += 1
                elif k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    cores.add((phys, v))
    except OSError:
        pass
    return {"cpu_model": model, "host_physical_cores": len(cores) or None, "host_logical_cpus": logical or None}


def cpu_threads():
    """Threads for the CPU baseline: one per physical core of this host, capped by the CPU share
    the job was given (OMP_NUM_THREADS: 16 per GPU on the MI355X boxes)."""
    info = host_cpu_info()
    n = info["host_physical_cores"] or os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return n, info


def cpu_job(kind, sd, arrays, **kwargs):
    """A CPU-baseline job for oracle/cpu_timer.py: the oracle function `kind` on `arrays` with
    the state dict `sd` (numpy or torch values)."""
    return {"kind": kind, "sd": sd, "arrays": arrays, "kwargs": kwargs}


def _timer_child(job, units, cpus, target_s, repeats):
    """Run oracle/cpu_timer.py on `job` in a child process pinned one thread per CPU of `cpus`
    (this process keeps the GPU; the child never touches it).  Returns its JSON record."""
    import shutil
    import subprocess
    import tempfile
    from oracle.cpu_timer import child_env

    def host(v):
        return v.detach().to("cpu").numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
    tmp = tempfile.mkdtemp(prefix="vp3d_cpu_")
    try:
        path = os.path.join(tmp, "job.npz")
        meta = {"kind": job["kind"], "kwargs": job["kwargs"], "units": int(units), "target_s": float(target_s),
                "repeats": int(repeats), "threads": len(cpus)}
        payload = {f"sd:{k}": np.ascontiguousarray(host(v)) for k, v in job["sd"].items()}
        payload.update({k: np.ascontiguousarray(host(v)) for k, v in job["arrays"].items()})
        np.savez(path, meta=np.array(json.dumps(meta)), **payload)
        r = subprocess.run([sys.executable, "-m", "oracle.cpu_timer", path], cwd=REPO, env=child_env(cpus),
                           capture_output=True, text=True, timeout=max(300.0, 6 * target_s * (repeats + 2)))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if r.returncode != 0 or not r.stdout.strip():
        raise RuntimeError(f"cpu baseline child failed (rc {r.returncode}): {r.stderr[-2000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_baseline(job, units_per_run, unit, sample_desc, repeats=5, target_s=2.5, all_cores=False):
    """Median of `repeats` timed runs (after a warm-up and a calibration run) of the oracle on
    the host cores, in a child process whose torch threads are pinned one per distinct physical
    core inside this process's affinity set (OMP_PLACES / OMP_PROC_BIND; oracle/cpu_timer.py).
    One run of `job` processes `units_per_run` units; each timed run repeats it to ~target_s.
    all_cores: also one short timing on every physical core of the affinity set (side figure)."""
    from oracle.cpu_timer import cgroup_cpu_quota, pick_cores
    threads, info = cpu_threads()
    cpus, n_phys = pick_cores(threads)
    res = _timer_child(job, units_per_run, cpus, target_s, repeats)
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    pinned = [t for t in res["thread_cpu_map"] if "," not in t["allowed"] and "-" not in t["allowed"]]
    out = {"value": res["value"], "unit": unit, "cores": len(cpus), "kind": "port",
           "sample": f"{sample_desc}; median of {repeats} runs of {res['reps']} x {units_per_run} after a warm-up "
                     f"and a calibration run ({res['timed_s']:.1f} s timed)",
           "runs": res["runs"], "runs_order": "time order", "spread": res["spread"],
           "pinned_cpus": cpus, "threads_pinned": len(pinned),
           "pinned_threads_ran_on": sorted({t["last_cpu"] for t in pinned}),
           "affinity_cpus": affinity, "affinity_physical_cores": n_phys, "cgroup_cpu_quota": cgroup_cpu_quota(),
           **info,
           "threads_note": "torch threads = physical cores capped by the job's CPU share (OMP_NUM_THREADS), one "
                           "thread pinned per distinct physical core (the least-busy cores of sched_getaffinity "
                           "by a 0.3 s /proc/stat sample, the idler sibling of each; OMP_PLACES + "
                           "OMP_PROC_BIND=close in a child process)"}
    if all_cores and n_phys > len(cpus):
        allc, _ = pick_cores(None)
        r2 = _timer_child(job, units_per_run, allc, max(0.6, target_s / 3), 3)
        out["all_physical_cores"] = {"value": r2["value"], "cores": len(allc), "runs": r2["runs"],
                                     "spread": r2["spread"],
                                     "note": "side figure: one thread per physical core of the whole affinity "
                                             "set, beyond the job's CPU share: under a cgroup quota "
                                             "(cgroup_cpu_quota CPUs) these threads share that quota, and other "
                                             "jobs may share these cores"}
    return out


def timed_steps(step, steps, warmup, settle_s, world, sync=None):
    """W warm-up steps, untimed steps until the device has run `settle_s` (clock ramp),
    then exactly `steps` steps bracketed by barrier + synchronize; returns seconds."""
    sync = sync or torch.cuda.synchronize
    for _ in range(warmup):
        step()
    sync()
    t = time.perf_counter()
    while time.perf_counter() - t < settle_s:
        step()
        sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0


LAYER_NAMES = ["expand"] + [f"block{(i // 2) + 1}_{'k3' if i % 2 == 0 else '1x1'}"
                            for i in range(2 * (len(FW) - 1))] + ["shrink"]


def profiled_run(lifter, step, steps, warmup, settle_s, world):
    """Per-layer times from an untimed pass with events around every launch, then the
    timed steps with events around the dominant layer only (events on all ten launches
    cost ~75 us per step).  Returns (dt, per_layer_ms, dominant-layer record)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    while time.perf_counter() - t < settle_s:
        step()
        torch.cuda.synchronize()
    lifter.profile(True)
    lifter.profile_layers(None)
    lifter.profile_reset()
    for _ in range(min(steps, 10)):
        step()
    layer_prof = lifter.profile_read()
    dom_layer = max(layer_prof, key=lambda r: r["ms_total"])["layer"]
    lifter.profile_layers([dom_layer])
    lifter.profile_reset()
    dt = timed_steps(step, steps, 0, 0.0, world)
    lifter.profile(False)
    lifter.profile_layers(None)
    dom = lifter.profile_read()[dom_layer]
    per_layer = {LAYER_NAMES[r["layer"]]: round(r["ms_total"] / max(r["launches"], 1), 4) for r in layer_prof}
    return dt, per_layer, dom


def roofline_of(dom, peak, traffic=None, traffic_note=None):
    avg_ms = max(dom["ms_total"] / max(dom["launches"], 1), 1e-9)
    achieved = dom["flop"] / (avg_ms * 1e-3) / 1e12
    r = {"bound": "mfma", "kernel": f"conv_gemm ({LAYER_NAMES[dom['layer']]})", "achieved": round(achieved, 2),
         "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
         "avg_launch_ms": round(avg_ms, 4), "launches_timed": dom["launches"], "flop_per_launch": dom["flop"]}
    if traffic_note:
        r["traffic_source"] = traffic_note
    return r


def committed_traffic(dtype, B, traj=False):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary
    (tools/traffic.py over rocprofv3 FETCH_SIZE / WRITE_SIZE passes), only when that summary was
    taken on the library built from these sources (its build_hash); otherwise None, with the
    stale figure and its provenance in the returned note."""
    tfile = os.path.join(REPO, "profiles", f"traffic_{dtype}_b{B}{'_traj' if traj else ''}.json")
    if not os.path.exists(tfile):
        return None, None
    with open(tfile) as f:
        t = json.load(f)
    from vp3d_amd import _native
    cur = _native.load().vp3d_build_hash().decode()
    same = t.get("build_hash") == cur
    note = {"file": os.path.relpath(tfile, REPO), "build_hash": t.get("build_hash"), "current_build": cur,
            "same_build": same, "git_commit": t.get("git_commit")}
    if not same:
        note["stale_hbm_bytes_per_launch"] = t.get("hbm_bytes_per_launch")
    return (t.get("hbm_bytes_per_launch") if same else None), note


class WindowsCase:
    """One TemporalModelOptimized1f workload over 243-frame windows resident in HBM (configs 2-4:
    17 joints; config 3: 23 "joints" = keypoints + the 12 K.E channels).

    G windows of one seeded global set (vp3d_amd.pipeline.SyntheticWindowPool), this rank's
    shard gathered on device inside every step (fused into the expand conv on the 16-bit and
    split-fp16 paths); config 3 also recomputes the per-frame K.E inside the step."""

    def __init__(self, traj, G, rank, world, dev, batch=None, pregathered=False):
        from common.models.TemporalModel import TemporalModelOptimized1f
        from vp3d_amd import synth
        from vp3d_amd.pipeline import SyntheticWindowPool
        from vp3d_amd.shard import window_shard
        self.traj, self.dev = traj, dev
        self.jin = 23 if traj else JOINTS
        model = TemporalModelOptimized1f(self.jin, 2, JOINTS, FW, channels=CHANNELS)
        self.sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()], seed=0)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in self.sd.items()})
        model.eval().cuda()
        self.RF = model.receptive_field()
        self.pad = (self.RF - 1) // 2
        self.pool = SyntheticWindowPool(1000, dev, cameras=traj)
        if batch:
            self.G = batch * world
            s, e = rank * batch, (rank + 1) * batch
            self.pairs = torch.from_numpy(self.pool.global_pairs(self.G)[s:e]).to(dev)
            self.scaling = "weak"
        else:
            self.G = G
            self.pairs, s, e = window_shard(self.pool, G, rank, world, dev)
            self.scaling = "strong"
        self.B = e - s
        self.lifter = model.native_lifter(dev)
        self.x = None
        if not traj and pregathered:
            self.x = self.pool.seqs.gather(self.pairs, self.RF, self.pad, "2d").view(self.B, self.RF, self.jin, 2)
        self.flop_pose = 358541312 if traj else 352569344
        self._ref = None

    def make_step(self, dtype, y, pairs=None, x=None):
        pairs = self.pairs if pairs is None else pairs
        lifter, seqs, RF, pad = self.lifter, self.pool.seqs, self.RF, self.pad
        if self.traj:
            def step():
                # config 3: K.E of every frame, then the window gather + camera concat fused
                # into the expand conv's operand loads, then the stack
                seqs.refresh_cameras()
                lifter.forward_windows(seqs, pairs, RF, pad, concat_cams=True, dtype=dtype, out=y)
        elif x is None:
            def step():
                # configs 2/4: the batch of the step (ChunkedGenerator's window gather with
                # edge clamping, generators.py:102-137) assembled on device from the resident
                # sequences, then the stack (TemporalModel.py:62-76)
                lifter.forward_windows(seqs, pairs, RF, pad, concat_cams=False, dtype=dtype, out=y)
        else:
            def step():
                lifter.forward(x, dtype, out=y)
        return step

    def run(self, dtype, steps, warmup, settle_s, world):
        """Time `steps` steps in `dtype`; returns (seconds, per-layer ms, dominant record, output)."""
        y = torch.empty((self.B, 1, JOINTS, 3), device=self.dev)
        self.lifter.reserve(self.B, self.RF, dtype)
        with torch.no_grad():
            dt, per_layer, dom = profiled_run(self.lifter, self.make_step(dtype, y, x=self.x), steps, warmup,
                                              settle_s, world)
        # a device-side fault of any forward of the leg (split-K timeout, f16x3 range) raises here
        self.lifter.sync_status()
        return dt, per_layer, dom, y

    def parity_ref(self, P):
        """The oracle on P windows from both ends of the shard (rank 0), once per case."""
        if self._ref is None:
            from oracle.temporal_ref import lifter_forward
            from vp3d_amd import synth
            P = min(P, self.B)
            idx = torch.cat([torch.arange(P // 2), torch.arange(self.B - (P - P // 2), self.B)]).to(self.dev)
            xs = self.pool.seqs.gather(self.pairs[idx].contiguous(), self.RF, self.pad, "2d",
                                       concat_cams=self.traj).view(P, self.RF, self.jin, 2)
            ref = lifter_forward(self.sd, xs.cpu(), FW, strided=True).numpy()
            # the same windows in float64: the yardstick for how much of a delta is the
            # reference's own fp32 rounding
            ref64 = lifter_forward(self.sd, xs.cpu(), FW, strided=True, dtype=torch.float64).numpy()
            gt = synth.gt_poses(3, "bench_gt", P, JOINTS).reshape(ref.shape)
            self._ref = (idx, ref, gt, ref64)
        return self._ref

    @staticmethod
    def _mp(a, gt):
        return float(np.mean(np.linalg.norm(a.astype(np.float64) - gt, axis=-1)))

    def parity(self, y, P):
        idx, ref, gt, ref64 = self.parity_ref(P)
        yf = y[idx].cpu().numpy()
        mp = self._mp
        return {"mpjpe_delta_mm": abs(mp(yf, gt) - mp(ref, gt)) * 1e3,
                "max_coord_delta_mm": float(np.abs(yf - ref).max()) * 1e3,
                "mpjpe_delta_vs_fp64_mm": abs(mp(yf, gt) - mp(ref64, gt)) * 1e3,
                "meets_north_star_1e-4mm": bool(abs(mp(yf, gt) - mp(ref, gt)) * 1e3 <= 1e-4)}

    def parity_info(self, P):
        idx, ref, gt, ref64 = self.parity_ref(P)
        mp = self._mp
        return {"windows": int(idx.numel()), "windows_checked": "first and last half of rank 0's shard "
                "(the timed kernels' own output)",
                "mpjpe_ref_mm": round(mp(ref, gt) * 1e3, 6),
                "reference_fp32_vs_fp64_mpjpe_delta_mm": abs(mp(ref, gt) - mp(ref64, gt)) * 1e3,
                "reference_fp32_vs_fp64_max_coord_delta_mm": float(np.abs(ref - ref64).max()) * 1e3,
                "output_rms_m": round(float(np.sqrt(np.mean(ref.astype(np.float64) ** 2))), 6)}

    def cpu_baseline(self, seconds, all_cores=False):
        xc = self.pool.seqs.gather(self.pairs[:64].contiguous(), self.RF, self.pad, "2d",
                                   concat_cams=self.traj).view(-1, self.RF, self.jin, 2).cpu()
        return cpu_baseline(cpu_job("lifter", self.sd, {"x": xc}, fw=FW, strided=True), int(xc.shape[0]),
                            "poses/s", f"windows of 243x{self.jin}x2 through oracle/temporal_ref.py (torch-CPU, fp32, "
                            f"batch {int(xc.shape[0])})", target_s=seconds / 5, all_cores=all_cores)

    def leg(self, dtype, steps, warmup, settle_s, P, G=None):
        """One dtype on this case (rank 0, N = 1): rate, roofline, per-layer times, parity."""
        dt, per_layer, dom, y = self.run(dtype, steps, warmup, settle_s, 1)
        traffic, tnote = committed_traffic(dtype, self.B, self.traj)
        out = {"value": round((G or self.G) * steps / dt, 2), "unit": "poses/s", "steps": steps,
               "ms_per_step": round(dt / steps * 1e3, 4),
               "tflops_effective": round((G or self.G) * steps / dt * self.flop_pose / 1e12, 2),
               "roofline": roofline_of(dom, PEAK_TFLOPS[dtype], traffic, tnote), "per_layer_ms": per_layer,
               "faults": 0, **self.parity(y, P)}
        if dtype == "f16x3":
            out["roofline"]["peak_note"] = ("f16 dense MFMA peak / 3: three f16 products per algorithmic "
                                            "multiply-add (hi.hi + hi.lo + lo.hi)")
        del y
        return out

    def close(self):
        self.lifter.close()
        self.x = None


def windows_main(args, world, rank, dev):
    """Configs 2-4 (default: config 4 at N ranks), or config 3 with --traj.

    Default line: a global batch of --global-batch windows (65,536: config 4) sharded over the
    ranks with vp3d_amd.shard.shard_range (strong scaling; N = 1 is the config-2/4 single-GPU
    point), timed in the accurate split-fp16 path (f16x3: the north-star tolerance at MFMA
    rates).  --batch B: B windows per rank (weak scaling).  At N = 1 the line also carries
    the bf16 (config 2's dtype) and fp32 legs, the batch sweep, config 3 (fp16 / f16x3 / fp32)
    and config 5 (causal streaming) as legs, each with its roofline, parity and CPU baseline."""
    traj = args.traj
    dtype = args.dtype or ("fp16" if traj else "f16x3")
    case = WindowsCase(traj, args.global_batch, rank, world, dev, args.batch, args.pregathered)
    G, B = case.G, case.B
    dt, per_layer, dom, y = case.run(dtype, args.steps, args.warmup, args.settle_seconds, world)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    value = G * args.steps / dt if case.scaling == "strong" else world * B * args.steps / dt
    if rank != 0:
        return
    P = args.parity_windows
    parity = dict(case.parity_info(P), **{f"{dtype}_{k}": v for k, v in case.parity(y, P).items()})
    del y
    traffic, tnote = committed_traffic(dtype, B, traj)
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "poses/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": case.scaling, "vs_baseline": None, "dtype": dtype,
        "dtype_note": ("f16x3 = split fp16: every f32 value carried as f16 hi + lo, three f16 MFMA products per "
                       "multiply-add accumulated in f32 -- the accuracy of the reference's fp32 (parity below) at "
                       "16-bit MFMA rates" if dtype == "f16x3" else None),
        "data": "synthetic (seeded random-walk 2D keypoint tracks gathered into windows on device, "
                "counter-hash weights)",
        "config": {
            "workload": ("config3 trajectory-conditioned (46ch) " if traj else
                         ("config4 global batch sharded over ranks, " if case.scaling == "strong" else "config2 ")
                         ) + "TemporalModelOptimized1f 243-frame RF windows, 17 joints, 1024 ch" +
                        ("; windows pre-gathered before the timed region" if case.x is not None else
                         "; window batch assembled on device from resident sequences inside the step"),
            "global_batch": G, "windows_per_gpu": B,
            "parallelism": f"dp{world} (contiguous shards of one global window set, no collective)"
            if case.scaling == "strong" else f"dp{world} (independent windows per rank, no collective)",
            "flop_per_pose": case.flop_pose},
        "tflops_effective": round(value * case.flop_pose / 1e12, 2),
        "roofline": roofline_of(dom, PEAK_TFLOPS[dtype], traffic, tnote),
        "per_layer_ms": per_layer,
        "per_layer_note": "untimed pass with HIP events around every launch",
        "faults": 0,
        "faults_note": "vp3d_sync_status after every timed leg: a device-side fault (split-K timeout, f16x3 "
                       "range) raises instead of reporting",
        "parity": parity,
    }
    if dtype == "f16x3":
        out["roofline"]["peak_note"] = ("f16 dense MFMA peak / 3: three f16 products per algorithmic "
                                        "multiply-add (hi.hi + hi.lo + lo.hi)")
    if world > 1 or args.no_extras:
        emit_line(out)
        return
    legs = ["bf16", "fp32"] if not traj else ["f16x3", "fp32"]
    for dl in legs:
        if dl == dtype:
            continue
        ks = max(3, args.steps // 4) if dl == "fp32" else max(5, args.steps // 2)
        out[dl] = case.leg(dl, ks, 1, 0.3, P)
        parity[f"{dl}_mpjpe_delta_mm"] = out[dl]["mpjpe_delta_mm"]
        parity[f"{dl}_max_coord_delta_mm"] = out[dl]["max_coord_delta_mm"]
    if not traj:
        # ---- config-2 batch sweep (1 GPU), the timed dtype and bf16 ----
        sweep = {}
        for sdt in dict.fromkeys([dtype, "bf16"]):
            row = {}
            for Bs in args.sweep:
                if Bs == B and sdt == dtype:
                    row[str(Bs)] = round(value, 2)
                    continue
                if Bs == B and sdt in out:
                    row[str(Bs)] = out[sdt]["value"]
                    continue
                ps = torch.from_numpy(case.pool.global_pairs(Bs)).to(dev)
                ysw = torch.empty((Bs, 1, JOINTS, 3), device=dev)
                xsw = case.pool.seqs.gather(ps, case.RF, case.pad, "2d").view(Bs, case.RF, case.jin, 2) \
                    if args.pregathered else None
                case.lifter.reserve(Bs, case.RF, sdt)
                ks = max(5, args.steps // 2)
                with torch.no_grad():
                    dts = timed_steps(case.make_step(sdt, ysw, ps, xsw), ks, 3, 0.2, 1)
                case.lifter.sync_status()
                row[str(Bs)] = round(Bs * ks / dts, 2)
                del ysw, xsw
            sweep[sdt] = row
        out["batch_sweep_poses_per_s"] = sweep
    # ---- CPU baseline: the oracle (reference op sequence) on 64 windows of the same set ----
    if args.cpu_seconds > 0:
        cpu = case.cpu_baseline(args.cpu_seconds, all_cores=True)
        out["cpu_baseline"] = cpu
        out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        for dl in legs:
            if dl in out:
                out[dl]["speedup_vs_cpu"] = round(out[dl]["value"] / cpu["value"], 1)
    case.close()
    del case
    if not traj and not args.no_legs:
        # ---- config 3 at the same global batch: fp16 (fast), f16x3 and fp32 (the gate) ----
        c3 = WindowsCase(True, args.global_batch, 0, 1, dev)
        leg3 = {"workload": "config3 trajectory-conditioned (46ch: K.E of every frame + window gather + camera "
                            "concat inside the step) TemporalModelOptimized1f, 243-frame RF windows of the dolly "
                            "sequences (K.E translations to ~22 m)", "global_batch": c3.G,
                "flop_per_pose": c3.flop_pose, "parity_info": c3.parity_info(P)}
        for dl, ks in (("fp16", max(5, args.steps // 2)), ("f16x3", max(5, args.steps // 2)),
                       ("fp32", max(3, args.steps // 4))):
            leg3[dl] = c3.leg(dl, ks, 1, 0.3, P)
        if args.cpu_seconds > 0:
            leg3["cpu_baseline"] = c3.cpu_baseline(args.cpu_seconds)
            for dl in ("fp16", "f16x3", "fp32"):
                leg3[dl]["speedup_vs_cpu"] = round(leg3[dl]["value"] / leg3["cpu_baseline"]["value"], 1)
        out["config3"] = leg3
        c3.close()
        del c3
        # ---- sequence mode (run.py --evaluate's path): f16x3 and fp32 at the gate, bf16 ----
        sq = SequenceCase(65536, 0, dev)
        legs_s = {"workload": f"TemporalModel (dilated) on one sequence of {65536 + sq.RF - 1} frames -> 65,536 "
                              "poses per step (run.py:697-711, UnchunkedGenerator edge padding)",
                  "flop_per_step": sq.flop_step}
        for dl, ks in (("f16x3", max(5, args.steps // 2)), ("fp32", max(3, args.steps // 4)),
                       ("bf16", max(5, args.steps // 2))):
            legs_s[dl] = sq.leg(dl, ks, 1, 0.3)[1]
        if args.cpu_seconds > 0:
            legs_s["cpu_baseline"] = sq.cpu_baseline(args.cpu_seconds)
            for dl in ("f16x3", "fp32", "bf16"):
                legs_s[dl]["speedup_vs_cpu"] = round(legs_s[dl]["value"] / legs_s["cpu_baseline"]["value"], 1)
        out["sequence"] = legs_s
        sq.close()
        del sq
        # ---- config 5: causal streaming, hipGraph of 64 steps + serve latency: fp32 (exact
        # weights resident, the north-star gate) and fp16 (config 5's named dtype) ----
        c5 = {}
        for d5 in ("fp32", "fp16"):
            a5 = argparse.Namespace(**vars(args))
            a5.dtype, a5.steps, a5.warmup = d5, 64 * 40, 64 * 4
            if "fp32" in c5:
                a5.stream_cpu_baseline = c5["fp32"].get("cpu_baseline")
            c5[d5] = stream_main(a5, 1, 0, dev, emit=False)
        out["config5"] = c5
    emit_line(out)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` (N > 1) started without a launcher: start N ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as a CHILD process and
    return its exit code.  This process never touches the GPU (device_count() does not
    initialise it on this image); it refuses when fewer than N GPUs are visible, unless the
    run is a rehearsal (VP3D_BENCH_REHEARSE=1: ranks share the GPUs; VP3D_BENCH_DRY=1: no GPU)."""
    import subprocess
    rehearse = os.environ.get("VP3D_BENCH_REHEARSE") == "1" or os.environ.get("VP3D_BENCH_DRY") == "1"
    if not rehearse:
        ndev = torch.cuda.device_count()
        if ndev < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {ndev} (VP3D_BENCH_REHEARSE=1 shares "
                  "them for a rehearsal)", file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench.py: launching {n} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def dry_main(args, world, rank):
    """VP3D_BENCH_DRY=1 (CPU tests only, never a reported number): the rank plumbing of the
    default line -- the launcher, gloo rendezvous, this rank's shard_range of the global batch,
    barrier-bracketed timing of K steps, MAX over ranks, ONE line from rank 0 -- with a CPU
    stand-in step instead of the GPU forward."""
    from vp3d_amd.shard import shard_range
    if world > 1:
        dist.init_process_group("gloo")
    s, e = shard_range(args.global_batch, rank, world)
    a = np.ones((64, 64), np.float32)

    def step():
        a.dot(a)
    dt = timed_steps(step, args.steps, args.warmup, 0.0, world, sync=lambda: None)
    t = torch.tensor([dt], dtype=torch.float64)
    sizes = torch.tensor([e - s], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(sizes, op=dist.ReduceOp.SUM)
    dt = float(t.item())
    if rank == 0:
        emit_line({"metric": METRIC, "value": round(args.global_batch * args.steps / dt, 2), "unit": "poses/s",
                   "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                   "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
                   "vs_baseline": None, "dtype": "none", "dry_run": True,
                   "data": "DRY RUN (VP3D_BENCH_DRY=1): CPU stand-in step, rank plumbing only -- not a measurement",
                   "config": {"workload": "dry rehearsal of the config-4 rank plumbing", "global_batch": args.global_batch,
                              "windows_per_gpu": e - s, "windows_all_ranks": int(sizes.item()),
                              "parallelism": f"dp{world} (contiguous shards, no collective)"}})
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # not under a launcher: start the N ranks ourselves (before any GPU call)
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to label a {world}-rank run as "
              f"{args.gpus} GPUs", file=sys.stderr, flush=True)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("VP3D_BENCH_DRY") == "1":
        dry_main(args, world, rank)
        return
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
        if args.dtype is None:
            args.dtype = "fp16" if args.stream else "bf16"
        fn = (train_main if args.train else seq_main if args.seq_model else
              sequence_main if args.sequence else stream_main)
        fn(args, world, rank, dev)
    else:
        windows_main(args, world, rank, dev)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
