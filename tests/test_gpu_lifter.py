"""GPU parity of the native lifter (libvp3d.so) against the CPU oracle.

Tolerances (stated per the north star, SURVEY.md §7 "Hard parts"):
  fp32  : |MPJPE(native, GT) - MPJPE(oracle, GT)| <= 1e-7 m (= 1e-4 mm) and every
          coordinate within 1e-5 m of the oracle (the reference's own fp32
          deviation from exact arithmetic is ~2e-7 m on these weights).
  f16x3 : the split-fp16 path (every f32 operand as hi + lo f16 halves, three 16-bit MFMA
          products per conv) is held to the fp32 gates above.
  bf16 / fp16 : measured separately; gates about 3x the largest error measured on
          MI355X over these cases (bf16 operands carry 8 mantissa bits, fp16 11).
"""
import numpy as np
import pytest
import torch

from helpers import H16_TOL, make_model, mpjpe_np
from oracle.temporal_ref import lifter_forward
from vp3d_amd import synth

pytestmark = pytest.mark.gpu

FP32_COORD_TOL = 1e-5
FP32_MPJPE_TOL = 1e-7


def _run(strided, B, T, fw=(3, 3, 3, 3, 3), causal=False, channels=1024, jin=17, jout=17,
         dense=False, dtype="fp32", seed=0):
    model, sd = make_model(strided, fw, causal, channels, jin=jin, jout=jout, dense=dense, seed=seed)
    x = synth.normalized_windows(seed + 1, f"x{B}_{T}", B, T, n_joints=jin)
    ref = lifter_forward(sd, x, list(fw), causal=causal, strided=strided, dense=dense).numpy()
    model.cuda().set_compute_dtype(dtype)
    with torch.no_grad():
        y = model(torch.from_numpy(x).cuda())
    torch.cuda.synchronize()
    y = y.cpu().numpy()
    assert y.shape == ref.shape, (y.shape, ref.shape)
    gt = synth.gt_poses(seed + 3, "gt", B * y.shape[1], jout).reshape(y.shape)
    return y, ref, gt


def _check(y, ref, gt, dtype):
    err = np.abs(y - ref).max()
    d_mpjpe = abs(mpjpe_np(y, gt) - mpjpe_np(ref, gt))
    print(f"{dtype}: max|d|={err:.3e} m  dMPJPE={d_mpjpe * 1e3:.3e} mm")
    assert np.isfinite(y).all()
    if dtype in ("fp32", "f16x3"):
        assert err <= FP32_COORD_TOL, err
        assert d_mpjpe <= FP32_MPJPE_TOL, d_mpjpe
    else:
        assert err <= H16_TOL[dtype][0], err
        assert d_mpjpe <= H16_TOL[dtype][1], d_mpjpe


@pytest.mark.parametrize("dtype", ["fp32", "f16x3"])
@pytest.mark.parametrize("causal", [False, True])
def test_opt1f_243_fp32(causal, dtype):
    y, ref, gt = _run(True, 64, 243, causal=causal, dtype=dtype)
    _check(y, ref, gt, dtype)


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_opt1f_243_h16(dtype):
    y, ref, gt = _run(True, 64, 243, dtype=dtype)
    _check(y, ref, gt, dtype)


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "f16x3"])
def test_opt1f_243_h16_large_batch(dtype):
    # B = 2050 windows: the block-1/2 layers (M = 55,350 / 18,450 rows, the last
    # 256-row tile partial) run on the 256x256 whole-line kernel (q64) and the expand
    # conv on the fused expand kernel -- the kernels the headline bench times
    y, ref, gt = _run(True, 2050, 243, dtype=dtype)
    _check(y, ref, gt, dtype)


_CONFIG4 = {}


def _config4_ref():
    if not _CONFIG4:
        model, sd = make_model(True, (3, 3, 3, 3, 3), False, 1024, seed=0)
        xs = synth.normalized_windows(1, "x64_243", 64, 243)
        _CONFIG4.update(model=model, xs=xs,
                        ref=lifter_forward(sd, xs, [3, 3, 3, 3, 3], strided=True).numpy())
    return _CONFIG4["model"], _CONFIG4["xs"], _CONFIG4["ref"]


@pytest.mark.parametrize("dtype", ["bf16", "fp32", "f16x3"])
def test_config4_b65536(dtype):
    """Config 4's whole global batch on one GPU: B = 65,536 windows (243 frames, 1024 ch),
    the shape the headline bench times.  The block-1 outputs are 3.6 GB in bf16 (past 2^31
    bytes: the q64 kernel's per-tile output resource) and 7.2 GB in fp32; the expand output
    10.9 / 21.7 GB.  The input is the 64 oracle windows tiled 1,024 times (windows are
    independent in the strided model), so the first, middle and last tiles -- the last
    256-row tiles of every layer -- are checked against the oracle, and every window
    against the tolerance."""
    model, xs, ref = _config4_ref()
    reps = 65536 // 64
    x = torch.from_numpy(xs).cuda().repeat(reps, 1, 1, 1)
    model.cuda().set_compute_dtype(dtype)
    with torch.no_grad():
        y = model(x)
    torch.cuda.synchronize()
    del x
    assert y.shape == (65536, 1, 17, 3)
    y = y.cpu().numpy().reshape((reps,) + ref.shape)
    gt = synth.gt_poses(3, "gt", 64 * ref.shape[1], 17).reshape(ref.shape)
    for r in (0, 1, reps // 2, reps - 2, reps - 1):
        _check(y[r], ref, gt, dtype)
    tol = FP32_COORD_TOL if dtype in ("fp32", "f16x3") else H16_TOL[dtype][0]
    assert np.abs(y - ref[None]).max() <= tol
    if dtype in ("fp32", "f16x3"):
        # tiles of identical windows: the same rows of every tile give the same bits
        assert np.array_equal(y[0], y[reps - 1])


@pytest.mark.parametrize("gemm,opt1f", [("big", True), ("8p", True), ("8p", False), ("q64", True), ("q64", False),
                                        ("h16", True), ("h16", False)])
def test_gemm_kernel_override(gemm, opt1f, monkeypatch):
    """Every 256x256 kernel on the shapes the default dispatch gives another one:
    VP3D_GEMM=big / 8p / q64 put the strided block convs (B = 2050) on the LDS-ring /
    ping-pong / quadrant-phase kernel (a4 is the default there), VP3D_GEMM=8p / q64 the dilated convs of a long sequence on those kernels;
    VP3D_GEMM=h16 (measurement override) every large layer on the 128x128 kernel."""
    monkeypatch.setenv("VP3D_GEMM", gemm)
    if opt1f:
        y, ref, gt = _run(True, 2050, 243, dtype="bf16")
    else:
        y, ref, gt = _run(False, 1, 20242, dtype="bf16")
    _check(y, ref, gt, "bf16")


@pytest.mark.parametrize("dtype,walk", [("bf16", None), ("fp16", None), ("bf16", "0"), ("bf16", "2"),
                                        ("f16x3", None), ("f16x3", "2")])
def test_gemm_a4_bit_identical_to_q64(dtype, walk, monkeypatch):
    """The one-wave-per-SIMD AGPR kernel (conv_gemm_a4.hip, the default for the strided k3
    and 1x1 + residual convs with >= 384 tiles) sums every output in q64's K order (two
    16x16x32 MFMAs per 64-deep K-tile, K-tiles in order), so both give the same bits.
    B = 4100: blocks 1 and 2 (110,700 / 36,900 rows) run on it with a ragged last row tile.
    walk: VP3D_A4_WALK -- default the 1x1 + residual layers walk their tiles (one workgroup
    per CU), "0" every layer one tile per workgroup, "2" every layer walks.  f16x3: the split
    fp16 mode (three f16 MFMAs per product, q64's order) against q64's, then the fp32 gates."""
    if walk is not None:
        monkeypatch.setenv("VP3D_A4_WALK", walk)
    # whole tiles only: a split-K last round (below) sums those tiles in two chains
    monkeypatch.setenv("VP3D_A4_SPLIT", "0")
    model, sd = make_model(True, (3, 3, 3, 3, 3), False, 1024)
    x = synth.normalized_windows(1, "x4100_243", 4100, 243)
    model.cuda().set_compute_dtype(dtype)
    xd = torch.from_numpy(x).cuda()
    ys = {}
    for gemm in ("q64", "a4"):
        monkeypatch.setenv("VP3D_GEMM", gemm)
        with torch.no_grad():
            ys[gemm] = model(xd).cpu().numpy()
    assert np.isfinite(ys["a4"]).all()
    assert np.array_equal(ys["a4"], ys["q64"]), np.abs(ys["a4"] - ys["q64"]).max()
    # the oracle on the first and last 64 windows
    sel = np.r_[0:64, 4036:4100]
    ref = lifter_forward(sd, x[sel], [3, 3, 3, 3, 3], causal=False, strided=True, dense=False).numpy()
    gt = synth.gt_poses(3, "gt", 128, 17).reshape(ref.shape)
    _check(ys["a4"][sel], ref, gt, dtype)


@pytest.mark.parametrize("dtype,B", [("bf16", 8192), ("f16x3", 8192), ("f16x3", 1024)])
def test_a4_half_n_tail_bit_identical(dtype, B, monkeypatch):
    """B = 8,192: every block conv leaves 128 tiles past its whole rounds (block 4: 128 tiles in
    all); the k3 convs run them as 256 half-N tiles of 256 x 128 (conv_gemm_a4 HN, a second
    launch) -- the same bits as q64's whole tiles and as a4's own whole tiles (VP3D_A4_HN=0,
    no split-K).  B = 1,024, f16x3: blocks 3 and 4 (48 / 16 tiles) run as quarter-N tiles of
    256 x 64."""
    model, sd = make_model(True, (3, 3, 3, 3, 3), False, 1024)
    x = synth.normalized_windows(1, f"x{B}_243", B, 243)
    model.cuda().set_compute_dtype(dtype)
    xd = torch.from_numpy(x).cuda()
    ys = {}
    for name, env in (("hn", {}), ("whole", {"VP3D_A4_HN": "0", "VP3D_A4_SPLIT": "0"}), ("q64", {"VP3D_GEMM": "q64"})):
        for k in ("VP3D_A4_HN", "VP3D_A4_SPLIT", "VP3D_GEMM"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with torch.no_grad():
            ys[name] = model(xd).cpu().numpy()
    assert np.isfinite(ys["hn"]).all()
    assert np.array_equal(ys["hn"], ys["whole"]), np.abs(ys["hn"] - ys["whole"]).max()
    assert np.array_equal(ys["hn"], ys["q64"]), np.abs(ys["hn"] - ys["q64"]).max()
    sel = np.r_[0:32, B - 32:B]
    ref = lifter_forward(sd, x[sel], [3, 3, 3, 3, 3], causal=False, strided=True, dense=False).numpy()
    gt = synth.gt_poses(3, "gt", 64, 17).reshape(ref.shape)
    _check(ys["hn"][sel], ref, gt, dtype)


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "f16x3"])
def test_dilated_seq_a4_bit_identical_to_q64(dtype, monkeypatch):
    """VP3D_GEMM=a4 puts the dilated k3 convs of a long sequence (taps d rows apart: the tile's
    k offset steps d rows at every tap) on conv_gemm_a4; q64 sums in the same order.  40,000
    frames: every block layer has >= 384 tiles of 256 x 256 (both kernels' threshold), 2 rounds
    + 112 tiles -- f16x3 runs those tails as half-N tiles (the k3 and the 1x1 + residual
    layers, the residual rows offset by the dilation's crop)."""
    monkeypatch.setenv("VP3D_A4_SPLIT", "0")  # whole tiles only (a split-K last round sums in two chains)
    model, sd = make_model(False, (3, 3, 3, 3, 3), False, 1024)
    x = synth.normalized_windows(1, "x1_40000", 1, 40000)
    model.cuda().set_compute_dtype(dtype)
    xd = torch.from_numpy(x).cuda()
    ys = {}
    for gemm in ("q64", "a4"):
        monkeypatch.setenv("VP3D_GEMM", gemm)
        with torch.no_grad():
            ys[gemm] = model(xd).cpu().numpy()
    assert np.isfinite(ys["a4"]).all()
    assert np.array_equal(ys["a4"], ys["q64"]), np.abs(ys["a4"] - ys["q64"]).max()


def test_dilated_seq_quarter_n_tail_bit_identical(monkeypatch):
    """Sequence mode at the bench's length (65,778 frames in, 65,536 poses): every block layer
    is 4 rounds + 4 tiles, which f16x3 runs (VP3D_A4_TAIL=hn) as 16 quarter-N tiles of 256 x 64
    (k3 and 1x1 + residual, dilated taps) -- the same bits as q64.  The default since round 6
    splits that tail's K range over every CU (test_dilated_seq_split_tail)."""
    model, sd = make_model(False, (3, 3, 3, 3, 3), False, 1024)
    x = synth.normalized_windows(1, "x1_65778", 1, 65778)
    model.cuda().set_compute_dtype("f16x3")
    xd = torch.from_numpy(x).cuda()
    monkeypatch.setenv("VP3D_A4_TAIL", "hn")
    ys = {}
    for gemm in ("q64", "a4"):
        monkeypatch.setenv("VP3D_GEMM", gemm)
        with torch.no_grad():
            ys[gemm] = model(xd).cpu().numpy()
    assert np.isfinite(ys["a4"]).all()
    assert np.array_equal(ys["a4"], ys["q64"]), np.abs(ys["a4"] - ys["q64"]).max()


@pytest.mark.parametrize("dtype", ["f16x3", "bf16"])
def test_dilated_seq_split_tail(dtype, monkeypatch):
    """The default f16x3 sequence-mode tail (conv_gemm_tail.hip): the 4 tiles past the 4 whole
    rounds of every block layer as (N / 64) x S K-slices over every CU plus a reduction launch.
    Against the quarter-N tiles (one full-K chain per output, VP3D_A4_TAIL=hn): every pose
    within 5e-6 m (S partial chains instead of one: f32 rounding of the partial sums only; the
    tails are the last 242 frames' outputs of every layer, which reach every pose through the
    receptive field), deterministic run to run, and against the oracle under the fp32 gates on
    the first and last output frames (the last ones are computed from the tail rows).  bf16
    (whole tiles in a fifth round otherwise): deterministic, and the bf16 gates vs the oracle."""
    model, sd = make_model(False, (3, 3, 3, 3, 3), False, 1024)
    x = synth.normalized_windows(1, "x1_65778", 1, 65778)
    model.cuda().set_compute_dtype(dtype)
    xd = torch.from_numpy(x).cuda()
    ys = {}
    for name, tail in (("hn", "hn"), ("split", None), ("split2", None)):
        if tail:
            monkeypatch.setenv("VP3D_A4_TAIL", tail)
        else:
            monkeypatch.delenv("VP3D_A4_TAIL", raising=False)
        with torch.no_grad():
            ys[name] = model(xd).cpu().numpy()
    model.native_lifter(torch.device("cuda")).sync_status()
    assert np.isfinite(ys["split"]).all()
    assert np.array_equal(ys["split"], ys["split2"])  # deterministic
    assert not np.array_equal(ys["split"], ys["hn"])  # the split path ran
    if dtype == "f16x3":
        d = np.abs(ys["split"] - ys["hn"]).max()
        assert d <= 5e-6, d  # (measured 1.07e-6 m: the same order as f16x3's own max error vs fp32)
    P = 64
    for lo in (0, 65536 - P):
        ref = lifter_forward(sd, x[:, lo:lo + P + 242], (3, 3, 3, 3, 3)).numpy()
        got = ys["split"][:, lo:lo + P]
        if dtype == "f16x3":
            assert np.abs(got - ref).max() <= 1e-5, (lo, np.abs(got - ref).max())
        else:
            # bf16: the coordinate gate, and the split tail's MPJPE delta against the whole tiles'
            # (a 64-frame delta of bf16 is noisy: both are printed)
            gt = synth.gt_poses(3, "gt", P, 17).reshape(ref.shape)
            hn = ys["hn"][:, lo:lo + P]
            d_s = abs(mpjpe_np(got, gt) - mpjpe_np(ref, gt)) * 1e3
            d_h = abs(mpjpe_np(hn, gt) - mpjpe_np(ref, gt)) * 1e3
            e_s, e_h = np.abs(got - ref).max(), np.abs(hn - ref).max()
            print(f"bf16 frames {lo}..: split max|d| {e_s:.3e} m dMPJPE {d_s:.4f} mm; whole tiles {e_h:.3e} m {d_h:.4f} mm")
            assert e_s <= H16_TOL[dtype][0], e_s


def test_dilated_long_seq_bf16():
    # one long sequence: every block layer has >= 384 output tiles, so the dilated
    # taps (row offsets 0, d, 2d) and the residual slice run on the LDS-ring kernel
    y, ref, gt = _run(False, 1, 20242, dtype="bf16")
    _check(y, ref, gt, "bf16")


@pytest.mark.parametrize("dtype", ["fp32", "f16x3"])
@pytest.mark.parametrize("causal", [False, True])
def test_dilated_seq_243_fp32(causal, dtype):
    y, ref, gt = _run(False, 1, 600, causal=causal, dtype=dtype)
    _check(y, ref, gt, dtype)


@pytest.mark.parametrize("dtype", ["fp32", "f16x3"])
def test_dilated_batch_ragged_fp32(dtype):
    # B=3 sequences, lengths give M not a multiple of the 128-row tile
    y, ref, gt = _run(False, 3, 300, fw=(3, 3, 3), channels=256, dtype=dtype)
    _check(y, ref, gt, dtype)


def test_dilated_27_bf16():
    y, ref, gt = _run(False, 2, 500, fw=(3, 3, 3), dtype="bf16")
    _check(y, ref, gt, "bf16")


@pytest.mark.parametrize("dtype", ["fp32", "f16x3"])
def test_dense_ablation_fp32(dtype):
    y, ref, gt = _run(False, 1, 120, fw=(3, 3, 3), channels=128, dense=True, dtype=dtype)
    _check(y, ref, gt, dtype)


@pytest.mark.parametrize("dtype", ["fp32", "f16x3"])
def test_small_channels_odd_joints(dtype):
    # trajectory-conditioned shape: 23 input "joints" (17 kp + 6 camera pairs), C=64
    y, ref, gt = _run(True, 5, 27, fw=(3, 3, 3), channels=64, jin=23, dtype=dtype)
    _check(y, ref, gt, dtype)


@pytest.mark.parametrize("dtype", ["fp32", "f16x3"])
def test_width5_blocks(dtype):
    y, ref, gt = _run(False, 2, 200, fw=(3, 5, 3), channels=128, dtype=dtype)
    _check(y, ref, gt, dtype)


def test_f16x3_unsupported_channels():
    """The split path needs channels % 64 == 0 (<= 1024): other widths raise, never a
    silent fallback."""
    m, _ = make_model(True, fw=(3, 3), channels=96)
    m.cuda().set_compute_dtype("f16x3")
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, 9, 17, 2, device="cuda"))


def test_weights_reload_and_equivalence():
    """Optimized1f and TemporalModel share weights (TemporalModel.py:147-149):
    the 1f output on every RF window equals the dilated sequence output."""
    m1, sd = make_model(True)
    md, _ = make_model(False)
    md.load_state_dict(m1.state_dict())
    T = 243 + 15
    x = torch.from_numpy(synth.normalized_windows(7, "eq", 1, T)).cuda()
    m1.cuda()
    md.cuda()
    with torch.no_grad():
        yd = md(x)  # (1, 16, 17, 3)
        win = x.unfold(1, 243, 1).permute(0, 1, 4, 2, 3)[0]  # (16, 243, 17, 2)
        y1 = m1(win.contiguous())  # (16, 1, 17, 3)
    assert (yd[0] - y1[:, 0]).abs().max().item() < 1e-5


def test_cpu_eval_raises():
    m, _ = make_model(True, fw=(3, 3), channels=64)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 9, 17, 2))


def test_shape_asserts_and_short_input():
    m, _ = make_model(False, fw=(3, 3), channels=64)
    m.cuda()
    with pytest.raises(AssertionError):
        m(torch.zeros(1, 20, 16, 2, device="cuda"))
    with pytest.raises(AssertionError):
        m(torch.zeros(20, 16, 2, device="cuda"))
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 5, 17, 2, device="cuda"))


@pytest.mark.parametrize("B", [8192, 300])
def test_x3_expand_three_per_cu_bit_identical(B, monkeypatch):
    """The f16x3 expand of the gathered config-4 shape runs three workgroups per CU (one
    resident weight chunk, 2 row blocks per wave) since round 6; the two-per-CU form
    (VP3D_X3_EXPAND_RING=2: 2-chunk ring, 3 row blocks) computes every output the same way, so
    the forwards are the same bits (B = 300: one partial round split into channel ranges)."""
    from vp3d_amd.pipeline import SyntheticWindowPool
    model, sd = make_model(True, (3, 3, 3, 3, 3), False, 1024)
    model = model.cuda()
    lifter = model.native_lifter(torch.device("cuda"))
    pool = SyntheticWindowPool(3, device="cuda", n_seq=8, seq_len=1024)
    pairs = torch.from_numpy(pool.global_pairs(B)).cuda()
    ys = {}
    for name, env in (("ring1", None), ("ring2", "2")):
        if env:
            monkeypatch.setenv("VP3D_X3_EXPAND_RING", env)
        else:
            monkeypatch.delenv("VP3D_X3_EXPAND_RING", raising=False)
        with torch.no_grad():
            ys[name] = lifter.forward_windows(pool.seqs, pairs, 243, 121, dtype="f16x3").cpu().numpy()
    lifter.sync_status()
    assert np.isfinite(ys["ring1"]).all()
    assert np.array_equal(ys["ring1"], ys["ring2"]), np.abs(ys["ring1"] - ys["ring2"]).max()


def test_x3_split_shrink(monkeypatch):
    """Since round 6 the f16x3 forward runs its shrink (N = 51) in split fp16 too, over the split
    rows of the last block (conv_gemm_tail.hip: 64 columns, a fixed 2 K-slices per output, rows
    in chunks of 131,072 that fit the split workspace).  One 140,242-frame sequence (two row
    chunks): within 5e-6 m of the exact-f32 shrink (VP3D_X3_SHRINK=f32, f32 rows from the last
    block) and under the fp32 gates vs the oracle on the first and last frames."""
    model, sd = make_model(False, (3, 3, 3, 3, 3), False, 1024)
    x = synth.normalized_windows(1, "x1_140242", 1, 140242)
    model.cuda().set_compute_dtype("f16x3")
    xd = torch.from_numpy(x).cuda()
    ys = {}
    for name, env in (("split", None), ("f32", "f32")):
        if env:
            monkeypatch.setenv("VP3D_X3_SHRINK", env)
        else:
            monkeypatch.delenv("VP3D_X3_SHRINK", raising=False)
        with torch.no_grad():
            ys[name] = model(xd).cpu().numpy()
    model.sync_status()
    assert np.isfinite(ys["split"]).all()
    d = np.abs(ys["split"] - ys["f32"]).max()
    assert d <= 5e-6, d  # (measured 2.0e-6 m over 140,000 poses: the f16x3 products' own error)
    P = 64
    for lo in (0, 140000 - P):
        ref = lifter_forward(sd, x[:, lo:lo + P + 242], (3, 3, 3, 3, 3)).numpy()
        got = ys["split"][:, lo:lo + P]
        assert np.abs(got - ref).max() <= 1e-5, (lo, np.abs(got - ref).max())


@pytest.mark.parametrize("dtype", ["fp32", "f16x3"])
def test_f32_narrow_shrink_bit_identical(dtype, monkeypatch):
    """The exact-f32 narrow GEMM that runs the shrink (N = 51) keeps conv_gemm_f32's MFMA k
    order: the same bits as the tile kernel (VP3D_F32_NARROW=0), on a ragged batch (the narrow
    kernel takes M < 32,768 rows).  f16x3: with its exact-f32 shrink (VP3D_X3_SHRINK=f32; the
    default is the split-fp16 shrink, test_x3_split_shrink)."""
    if dtype == "f16x3":
        monkeypatch.setenv("VP3D_X3_SHRINK", "f32")
    model, _ = make_model(True, seed=0)
    model = model.cuda()
    model.set_compute_dtype(dtype)
    x = torch.from_numpy(synth.normalized_windows(11, "narrow", 1000, 243)).cuda()
    with torch.no_grad():
        y_new = model(x).cpu().numpy()
        monkeypatch.setenv("VP3D_F32_NARROW", "0")
        y_old = model(x).cpu().numpy()
    assert np.array_equal(y_new, y_old)


@pytest.mark.parametrize("dtype", ["bf16", "f16x3"])
def test_a4_split_k_last_round(dtype, monkeypatch):
    """Config 4's per-GPU share at N = 8 (8,192 windows): every block leaves 128 tiles past the
    last whole round of 256 CUs, which conv_gemm_a4 can run as 2 half-K units each (the owner
    adds the helper's f32 partial sums before its epilogue; block 4's 128 tiles in all) --
    VP3D_A4_SPLIT=2: on every layer it fits, walked 1x1 layers and bf16 included.  Against
    the whole-tile run (VP3D_A4_SPLIT=0): f16x3 within 1e-6 m (only the partial sums' rounding
    differs), bf16 within its coordinate gate; both against the oracle on the first and last
    64 windows under their dtype's gates."""
    monkeypatch.setenv("VP3D_A4_SPLIT", "2")  # every layer it fits (default: none -- half-N tails)
    model, sd = make_model(True, (3, 3, 3, 3, 3), False, 1024)
    B = 8192
    x = synth.normalized_windows(5, "x8192_243", B, 243)
    model.cuda().set_compute_dtype(dtype)
    xd = torch.from_numpy(x).cuda()
    with torch.no_grad():
        y = model(xd).cpu().numpy()
        y2 = model(xd).cpu().numpy()
        monkeypatch.setenv("VP3D_A4_SPLIT", "0")
        y_whole = model(xd).cpu().numpy()
    assert np.isfinite(y).all()
    assert np.array_equal(y, y2)  # deterministic: the owner adds the partials in unit order
    d = float(np.abs(y - y_whole).max())
    print(f"{dtype}: split vs whole-tile max|d| {d:.3e} m")
    assert d <= (1e-6 if dtype == "f16x3" else H16_TOL[dtype][0]), d
    sel = np.r_[0:64, B - 64:B]
    ref = lifter_forward(sd, x[sel], [3, 3, 3, 3, 3], causal=False, strided=True, dense=False).numpy()
    gt = synth.gt_poses(3, "gt", 128, 17).reshape(ref.shape)
    _check(y[sel], ref, gt, dtype)


def test_a4_split_k_timeout_raises(monkeypatch):
    """Fault injection for the split-K owner's bounded wait (conv_gemm_a4.hip owner_wait):
    VP3D_A4_SPLIT_DROP=1 makes every helper unit skip its count, so each owner tile of the
    partial last round (VP3D_A4_SPLIT=2: every conv at 8,192 windows) gives up after its bound
    (VP3D_A4_SPLIT_SPIN_TICKS, 1 ms here).  The fault must surface, not pass as poses:
    the next forward on the handle is refused and sync_status raises RuntimeError; after
    sync_status cleared it (tile flags re-zeroed) the handle reproduces the good poses bit
    for bit."""
    # split-K wherever it fits (the default runs these tails as half-N tiles, no split)
    monkeypatch.setenv("VP3D_A4_SPLIT", "2")
    model, _ = make_model(True, (3, 3, 3, 3, 3), False, 1024)
    B = 8192
    x = torch.from_numpy(synth.normalized_windows(5, "x8192_243", B, 243)).cuda()
    model.cuda().set_compute_dtype("f16x3")
    lifter = model.native_lifter()
    with torch.no_grad():
        good = model(x).cpu().numpy()
        lifter.sync_status()  # no fault on the split path
        monkeypatch.setenv("VP3D_A4_SPLIT_DROP", "1")
        monkeypatch.setenv("VP3D_A4_SPLIT_SPIN_TICKS", "100000")
        model(x)
        torch.cuda.synchronize()
        monkeypatch.delenv("VP3D_A4_SPLIT_DROP")
        monkeypatch.delenv("VP3D_A4_SPLIT_SPIN_TICKS")
        with pytest.raises(RuntimeError, match="split-K"):
            model(x)  # refused at entry: the fault of the last forward is pending
        with pytest.raises(RuntimeError, match="split-K"):
            lifter.sync_status()
        lifter.sync_status()  # cleared
        again = model(x).cpu().numpy()
        lifter.sync_status()
    assert np.array_equal(again, good)


@pytest.mark.parametrize("where,B", [("input", 64), ("block0_k", 64), ("block1_1x1", 64), ("block1_1x1", 2048)])
def test_f16x3_range_fault_raises(where, B):
    """f16x3 carries activations as f16 halves (|x| <= 65,504).  A value past that range --
    in the input rows (x 1e6) or in a hidden layer's output (its BN gamma x 1e6) -- is
    flagged where it is split (gemm::x3_range_flag: the expand's input and epilogue, the q64
    and a4 epilogues) into the handle's fault word: the next forward is refused naming
    f16x3, sync_status raises it once, and the handle works again afterwards.  B = 64
    windows runs the hidden layers on q64, B = 2,048 on the one-wave-per-SIMD a4 kernel."""
    model, _ = make_model(True, (3, 3, 3, 3, 3), False, 1024)
    x = torch.from_numpy(synth.normalized_windows(5, "x64_243", B, 243)).cuda()
    model.cuda().set_compute_dtype("f16x3")
    lifter = model.native_lifter()
    with torch.no_grad():
        good = model(x).cpu().numpy()
        lifter.sync_status()
        if where == "input":
            model(x * 1e6)
        else:
            bn = model.layers_bn[0 if where == "block0_k" else 3]
            g0 = bn.weight.detach().clone()
            bn.weight.mul_(1e6)
            model(x)
            torch.cuda.synchronize()
            bn.weight.copy_(g0)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="f16x3"):
            model(x)
        with pytest.raises(RuntimeError, match="non-finite"):
            lifter.sync_status()
        lifter.sync_status()
        again = model(x).cpu().numpy()
        model.native_lifter().sync_status()
    assert np.array_equal(again, good)


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "f16x3"])
@pytest.mark.parametrize("B", [8192, 300])
def test_expand_split_round_bit_identical(dtype, B, monkeypatch):
    """expand_gemm runs a partial last round of row blocks (or all of them, for small M) as
    channel-range workgroups (B = 8,192: 32 / 64 row blocks past 5 / 10 whole rounds of 512
    slots -> 8 workgroups each; B = 300: under one round).  Each output element keeps its own
    K order, so the stack's output is bit-identical to whole row blocks (VP3D_EXPAND_SPLIT=0)."""
    model, _ = make_model(True, (3, 3, 3, 3, 3), False, 1024)
    x = torch.from_numpy(synth.normalized_windows(9, f"xs{B}", B, 243)).cuda()
    model.cuda().set_compute_dtype(dtype)
    with torch.no_grad():
        y = model(x).cpu().numpy()
        monkeypatch.setenv("VP3D_EXPAND_SPLIT", "0")
        y_whole = model(x).cpu().numpy()
    assert np.isfinite(y).all()
    assert np.array_equal(y, y_whole)
