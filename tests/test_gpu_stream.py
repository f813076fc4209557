"""Causal streaming step (config 5) vs the whole-sequence causal evaluation.

Reference semantics: UnchunkedGenerator pads a causal sequence with 2*pad copies
of frame 0 in front (generators.py:193-198), and TemporalModel(causal=True) maps
it to one pose per frame; pose k of the stream must equal frame k of that.
Tolerances: fp32 stream (exact f32 weights, f32 FMAs: only the order of the sums
differs from the reference) within 2e-5 m per coordinate and |dMPJPE| <= 1e-7 m (the
north-star 1e-4 mm); fp16 weights within 0.3 mm, bf16 within 3 mm (measured 0.14 /
0.90 mm, round 2)."""
import numpy as np
import pytest
import torch

from helpers import make_model
from oracle.temporal_ref import lifter_forward
from vp3d_amd import synth
from vp3d_amd.stream import CausalStream

pytestmark = pytest.mark.gpu


def _ref(sd, x, fw):
    pad = (int(np.prod(fw)) - 1) // 2
    xp = np.concatenate([np.repeat(x[:, :1], 2 * pad, axis=1), x], axis=1)
    return lifter_forward(sd, xp, list(fw), causal=True).numpy()[0]


def _dmpjpe(out, ref, gt):
    """|MPJPE(out, gt) - MPJPE(ref, gt)| in metres (loss.py:11-17 on both)."""
    m = lambda p: float(np.linalg.norm(p.astype(np.float64) - gt, axis=-1).mean())
    return abs(m(out) - m(ref))


@pytest.mark.parametrize("dtype,tol", [("fp32", 2e-5), ("fp16", 3e-4), ("bf16", 3e-3)])
def test_stream_matches_sequence(dtype, tol):
    fw = (3, 3, 3, 3, 3)
    m, sd = make_model(False, fw, causal=True)
    T = 200
    x = synth.normalized_windows(11, "stream", 1, T)
    ref = _ref(sd, x, fw)  # (T, 17, 3)
    m.cuda()
    st = CausalStream(m.native_lifter(), dtype)
    xs = torch.from_numpy(x[0]).cuda()
    out = torch.stack([st.step(xs[t]).clone() for t in range(T)]).cpu().numpy()
    st.check()
    assert st.mode == "pipe"
    err = np.abs(out - ref).max()
    gt = np.random.default_rng(3).normal(0.0, 0.2, ref.shape)
    dm = _dmpjpe(out, ref, gt)
    print(f"stream {dtype} ({st.mode}): max|d|={err:.3e} m, dMPJPE={dm * 1e3:.3e} mm")
    assert err <= tol
    if dtype == "fp32":
        assert dm <= 1e-7
    assert st.frames_seen() == T
    st.reset()
    first = st.step(xs[0]).cpu().numpy()
    np.testing.assert_allclose(first, out[0], atol=1e-7)


@pytest.mark.parametrize("dtype", ["fp16", "fp32"])
@pytest.mark.parametrize("fw,channels", [((3, 3, 3, 3, 3), 1024), ((3, 5, 3), 256), ((3, 3, 3), 256)])
def test_stream_forms_match_sequence(fw, channels, dtype, monkeypatch):
    """Every form of the step agrees with the whole-sequence reference:
    VP3D_STREAM_MODE=launches (per-layer GEMVs), =persist (every CU runs every layer,
    16-bit weights in LDS; fp32 has no such form and falls back to launches) and =pipe
    (one layer per CU, weights in VGPRs, frames pipelined through the layer groups; a
    width-5 block is outside it and falls back to persist, or launches for fp32).  fp32
    under the north-star gates: 2e-5 m per coordinate, |dMPJPE| <= 1e-7 m."""
    m, sd = make_model(False, fw, causal=True, channels=channels)
    T = 120
    x = synth.normalized_windows(13, "stream_forms", 1, T)
    ref = _ref(sd, x, fw)
    gt = np.random.default_rng(4).normal(0.0, 0.2, ref.shape)
    m.cuda()
    xs = torch.from_numpy(x[0]).cuda()
    outs = {}
    no_persist = "launches" if dtype == "fp32" else "persist"
    for mode in ("launches", "persist", "pipe"):
        monkeypatch.setenv("VP3D_STREAM_MODE", mode)
        st = CausalStream(m.native_lifter(), dtype)
        want = mode
        if mode == "persist" and dtype == "fp32":
            want = "launches"
        if mode == "pipe" and 5 in fw:
            want = no_persist
        assert st.mode == want, (mode, st.mode)
        assert st.persistent == (want != "launches")
        outs[mode] = torch.stack([st.step(xs[t]).clone() for t in range(T)]).cpu().numpy()
        st.check()
        err = np.abs(outs[mode] - ref).max()
        dm = _dmpjpe(outs[mode], ref, gt)
        print(f"stream {dtype} {mode} fw={fw}: max|d|={err:.3e} m, dMPJPE={dm * 1e3:.3e} mm")
        if dtype == "fp32":
            assert err <= 2e-5 and dm <= 1e-7
        else:
            assert err <= 3e-4
    monkeypatch.delenv("VP3D_STREAM_MODE", raising=False)
    st = CausalStream(m.native_lifter(), dtype)
    assert st.mode == (no_persist if 5 in fw else "pipe")


@pytest.mark.parametrize("fw,channels,T,graphs,dtype", [((3, 3, 3), 256, 80, (1, 8), "fp16"),
                                                         ((3, 3, 3, 3, 3), 1024, 192, (64,), "fp16"),
                                                         ((3, 3, 3, 3, 3), 1024, 192, (64,), "fp32")])
def test_stream_graph_replay_matches_eager(fw, channels, T, graphs, dtype):
    """Graphs of G steps fed from the device frame queue reproduce the eager per-step
    results bit for bit -- in the pipelined form a graph of 64 steps is one launch with up
    to 10 frames in flight through the layer groups, an eager step is a launch of one."""
    m, sd = make_model(False, fw, causal=True, channels=channels)
    x = torch.from_numpy(synth.normalized_windows(12, "graph", 1, T)[0]).cuda().reshape(T, -1)
    m.cuda()
    eager = CausalStream(m.native_lifter(), dtype)
    assert eager.mode == "pipe"
    want = torch.stack([eager.step(x[t]).clone().reshape(-1) for t in range(T)])
    eager.check()
    for G in graphs:
        g = CausalStream(m.native_lifter(), dtype)
        Q = g.queue_len
        assert T % G == 0 and Q % G == 0
        s = torch.cuda.Stream()
        fq, pr = g.io_tensors()
        g.capture(s, steps=G)
        got = []
        with torch.cuda.stream(s):
            for t0 in range(0, T, G):
                for t in range(t0, t0 + G):
                    fq[t % Q].copy_(x[t])
                g.replay(s)
                for t in range(t0, t0 + G):
                    got.append(pr[t % Q].clone())
        torch.cuda.synchronize()
        g.check()
        assert torch.equal(torch.stack(got), want), G
        assert g.frames_seen() == T


def test_stream_rejects_noncausal():
    m, _ = make_model(False, (3, 3), causal=False, channels=64)
    m.cuda()
    with pytest.raises(RuntimeError):
        CausalStream(m.native_lifter(), "fp16")


@pytest.mark.parametrize("mode", ["pipe", "persist"])
def test_stream_timeout_is_sticky(mode, monkeypatch):
    """Fault injection: VP3D_STREAM_SPIN_TICKS=0 makes the first unanswered poll of a
    persistent step time out.  The timeout word is sticky: check() raises, later step()s
    and graph replays are refused by the host (no synchronisation needed) and the device
    launches become no-ops, so the stream position never drifts; reset() clears it."""
    monkeypatch.setenv("VP3D_STREAM_MODE", mode)
    monkeypatch.setenv("VP3D_STREAM_SPIN_TICKS", "0")
    m, _ = make_model(False, (3, 3, 3), causal=True, channels=256)
    m.cuda()
    st = CausalStream(m.native_lifter(), "fp16")
    assert st.mode == mode
    xs = torch.from_numpy(synth.normalized_windows(17, "stream_fault", 1, 8)[0]).cuda()
    failed_at = None
    for t in range(8):
        try:
            st.step(xs[t])
        except RuntimeError:
            failed_at = t
            break
        torch.cuda.synchronize()
    assert failed_at is not None, "no step timed out with a zero spin budget"
    with pytest.raises(RuntimeError, match="timed out"):
        st.check()
    with pytest.raises(RuntimeError, match="timed out"):
        st.step(xs[0])
    seen = st.frames_seen()
    assert 0 <= seen < failed_at
    st.reset()
    st.check()
    assert st.frames_seen() == 0


@pytest.mark.parametrize("dtype", ["fp16", "fp32"])
def test_stream_serve_one_frame_in_flight(dtype):
    """Serving (vp3d_stream_serve_*): the pipelined launch stays resident and takes frames
    posted from host memory one at a time.  Poses equal the whole-sequence causal
    reference (the dtype's gate) and the batch form's within 1e-6 m (the serve form sums the
    shrink as per-workgroup partials, VP3D_STREAM_FOLD); frames may be posted ahead; the
    stream continues seamlessly in the batch form after serving; an idle launch ends itself
    and further posts are refused."""
    import time
    fw = (3, 3, 3, 3, 3)
    m, sd = make_model(False, fw, causal=True)
    T = 96
    x = synth.normalized_windows(19, "stream_serve", 1, T)
    ref = _ref(sd, x, fw)
    m.cuda()
    st = CausalStream(m.native_lifter(), dtype)
    assert st.mode == "pipe"
    with st.serve(idle_ms=500.0) as sv:
        served = [sv.step(x[0, t]) for t in range(48)]
        ts = [sv.post(x[0, t]) for t in range(48, 64)]  # 16 frames in flight at once
        assert ts == list(range(48, 64))
        served += [sv.wait(t) for t in ts]
    assert st.frames_seen() == 64
    xs = torch.from_numpy(x[0]).cuda()
    rest = [st.step(xs[t]).cpu().numpy() for t in range(64, T)]  # batch form continues
    out = np.concatenate([np.stack(served), np.stack(rest)])
    err = np.abs(out - ref).max()
    dm = _dmpjpe(out, ref, np.random.default_rng(6).normal(0.0, 0.2, ref.shape))
    print(f"serve {dtype}: max|d|={err:.3e} m, dMPJPE={dm * 1e3:.3e} mm")
    if dtype == "fp32":
        assert err <= 2e-5 and dm <= 1e-7
    else:
        assert err <= 3e-4
    st.reset()
    batch = torch.stack([st.step(xs[t]).clone() for t in range(64)]).cpu().numpy()
    # the serve form folds the shrink into the last 1x1 (partial sums per workgroup, added on
    # the host): the batch form's shrink sums the same products in another order
    np.testing.assert_allclose(np.stack(served), batch, rtol=0, atol=1e-6)
    # an idle launch ends itself; the next post is refused until serving restarts
    with st.serve(idle_ms=5.0) as sv:
        sv.step(x[0, 64])
        time.sleep(0.05)
        with pytest.raises(RuntimeError, match="ended"):
            sv.post(x[0, 65])
    assert st.frames_seen() == 65


def test_stream_serve_restarts_at_the_idle_limit():
    """A frame posted right at the idle limit: the launch's expand workgroups (4 at 1024
    channels) agree on one end frame (the claim word of stream_pipe.hip), so whichever way
    each race goes the stream position never skips a frame and the expand histories stay in
    step.  Frames are posted with delays around idle_ms; every time the launch has ended
    the session is restarted at the device's position and the frame re-posted.  The poses
    of all frames must equal the batch form's (within 1e-6 m: the serve form's folded shrink
    sums the same products in another order) -- no frame skipped or repeated."""
    import time
    fw = (3, 3, 3, 3, 3)
    m, sd = make_model(False, fw, causal=True)
    T = 64
    x = synth.normalized_windows(23, "stream_serve_edge", 1, T)
    m.cuda()
    st = CausalStream(m.native_lifter(), "fp16")
    rng = np.random.default_rng(5)
    idle_ms = 0.1
    poses = {}
    restarts = 0
    t = 0
    while t < T:
        with st.serve(idle_ms=idle_ms) as sv:
            assert st.frames_seen() == t
            while t < T:
                deadline = time.perf_counter() + rng.uniform(0.06e-3, 0.14e-3)
                while time.perf_counter() < deadline:
                    pass
                try:
                    i = sv.post(x[0, t])
                    assert i == t
                    poses[t] = sv.wait(t)
                except RuntimeError as e:
                    assert "ended" in str(e), e
                    break
                t += 1
        restarts += 1
        t = st.frames_seen()
        assert sorted(poses) == list(range(t)), (t, sorted(poses)[-3:])  # no frame skipped or repeated
    print(f"serve at the idle edge: {restarts} sessions for {T} frames")
    assert restarts > 1
    st.reset()
    xs = torch.from_numpy(x[0]).cuda()
    batch = torch.stack([st.step(xs[k]).clone() for k in range(T)]).cpu().numpy()
    np.testing.assert_allclose(np.stack([poses[k] for k in range(T)]), batch, rtol=0, atol=1e-6)


def test_stream_serve_fold_matches_unfolded(monkeypatch):
    """VP3D_STREAM_FOLD: the serve form's shrink as partial sums of the last block's 1x1
    workgroups (added on the host) against the shrink role's all-gather (VP3D_STREAM_FOLD=0,
    bit for bit the batch form): the same poses within 1e-6 m, fp32 weights."""
    fw = (3, 3, 3, 3, 3)
    m, sd = make_model(False, fw, causal=True)
    T = 32
    x = synth.normalized_windows(29, "stream_fold", 1, T)
    m.cuda()
    out = {}
    for fold in ("1", "0"):
        monkeypatch.setenv("VP3D_STREAM_FOLD", fold)
        st = CausalStream(m.native_lifter(), "fp32")
        got = []
        with st.serve(idle_ms=500.0) as sv:
            for t in range(T):
                try:
                    got.append(sv.step(x[0, t]))
                except RuntimeError as e:
                    raise RuntimeError(f"fold={fold} frame {t}: {e}") from e
        out[fold] = np.stack(got)
        st.check()
        st.close()
    xs = torch.from_numpy(x[0]).cuda()
    st = CausalStream(m.native_lifter(), "fp32")
    batch = torch.stack([st.step(xs[t]).clone() for t in range(T)]).cpu().numpy()
    np.testing.assert_array_equal(out["0"], batch)
    d = float(np.abs(out["1"] - out["0"]).max())
    print(f"serve fold vs all-gather shrink: max|d|={d:.3e} m")
    assert d <= 1e-6


def test_stream_serve_after_weight_reload_uses_new_shrink():
    """the folded serve form applies the shrink's affine on the host.  After the
    stream was created, a parameter change re-uploads the handle's weights in place
    (TemporalModel.native_lifter -> vp3d_load_weights); serving must then use the NEW shrink
    bias like the batch form does (serve_begin re-reads it), not the one seen at creation."""
    fw = (3, 3, 3, 3, 3)
    m, sd = make_model(False, fw, causal=True)
    T = 24
    x = synth.normalized_windows(31, "stream_reload", 1, T)
    m.cuda()
    st = CausalStream(m.native_lifter(), "fp32")
    with torch.no_grad():
        m.shrink.bias.add_(0.05)
    assert m.native_lifter() is st.lifter  # the same handle, weights re-uploaded in place
    with st.serve(idle_ms=500.0) as sv:
        served = np.stack([sv.step(x[0, t]) for t in range(T)])
    st.check()
    st.reset()
    xs = torch.from_numpy(x[0]).cuda()
    batch = torch.stack([st.step(xs[t]).clone() for t in range(T)]).cpu().numpy()
    np.testing.assert_allclose(served, batch, rtol=0, atol=1e-6)
    ref = _ref({k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}, x, fw)
    assert np.abs(batch - ref).max() <= 2e-5
