"""GPU parity of the native training step (vp3d_train_forward / vp3d_train_backward /
vp3d_adam_step through the drop-in TemporalModel in train mode).

References:
  * tests/golden/train_*.npz — the reference's own two training iterations
    (run.py:451-487 + Adam(amsgrad) run.py:662, dropout 0), made by make_golden.py;
  * oracle/train_ref.py — the same iteration on torch-CPU, fed the dropout masks the
    native trainer drew (vp3d_train_dropout_mask) for the dropout cases.

Tolerances (f32 on both sides; the native convs accumulate in another order and the
BN statistics in f64):
  output y           |dy| <= 1e-5 m absolute
  loss               relative 1e-5
  gradients          per tensor ||g - g64|| <= max(1e-4, 4 ||g32 - g64|| / ||g64||) ||g64||
                     (g32 / g64: the oracle's fp32 / fp64 gradients) and every element within
                     2e-3 * max|g64|.  An activation whose BN output lies within rounding of 0
                     can take the other side of the ReLU in two f32 implementations, and with
                     few rows per channel (the last blocks of a 32-window batch) one such
                     element moves a whole channel's BatchNorm gradients by ~1e-3; the dropout
                     cases therefore feed the trainer's ReLU decisions (vp3d_train_relu_mask)
                     to the fp64 / fp32 oracle as well as its dropout masks.
  running stats      relative 1e-5, absolute 1e-6 (batch means near 0)
  weights after Adam Adam's first steps move each weight by about +-lr * sign(g), so a
                     gradient element within rounding of 0 may flip its step: all weights
                     within 2*lr + 1e-6 and >= 99.9 % within 1e-5.  Step it >= 1 starts
                     from the reference's own weights of step it-1 (teacher forcing), so
                     each step is compared on identical inputs.
  Adam kernel alone  exp_avg / exp_avg_sq / max_exp_avg_sq bit-exact against
                     torch.optim.Adam (CPU); parameters within 1 ulp of the update: the f32
                     sqrt is correctly rounded, torch-CPU's vectorised sqrt is not (errors
                     up to ~0.55 ulp measured), so ~1 % of the updates differ by 1 ulp.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle.train_ref import TrainLoop, lifter_train_forward, mpjpe as mpjpe_ref
from vp3d_amd import synth
from vp3d_amd.lifter import weight_order

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["train_dilated_c64", "train_opt1f_c64", "train_causal_c64", "train_dense_c32"]
GRAD_REL = 2e-4


def _load(name):
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    return g, meta, {k[2:]: g[k] for k in g.files if k.startswith("w/")}


def _model(meta, state, dropout=0.0, channels=None, jin=17):
    from common.models.TemporalModel import TemporalModel, TemporalModelOptimized1f
    c = channels or meta["channels"]
    if meta["strided"]:
        m = TemporalModelOptimized1f(jin, 2, 17, meta["fw"], causal=meta["causal"], channels=c, dropout=dropout)
    else:
        m = TemporalModel(jin, 2, 17, meta["fw"], causal=meta["causal"], channels=c, dropout=dropout,
                          dense=meta["dense"])
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in state.items()})
    return m.cuda().train()


def _oracle(state, x, tgt, meta, p=0.0, masks=None, dtype=torch.float32, relu_masks=None):
    """Oracle train-mode forward + mpjpe + backward in `dtype`: (y, loss, grads, running stats)."""
    params = {k: torch.tensor(np.array(v), dtype=dtype) for k, v in state.items()
              if not k.endswith("num_batches_tracked")}
    for k, t in params.items():
        if "running" not in k:
            t.requires_grad_(True)
    y = lifter_train_forward(params, torch.from_numpy(np.asarray(x)).to(dtype), meta["fw"], causal=meta["causal"],
                             strided=meta["strided"], dense=meta["dense"], p=p, masks=masks,
                             relu_masks=relu_masks)
    loss = mpjpe_ref(y, torch.from_numpy(np.asarray(tgt)).to(dtype))
    loss.backward()
    grads = {k: t.grad.numpy() for k, t in params.items() if t.requires_grad}
    stats = {k: t.detach().numpy() for k, t in params.items() if "running" in k}
    return y.detach().numpy(), float(loss), grads, stats


def _grad_close(got, g32, g64, what):
    got, g32, g64 = (np.asarray(a, dtype=np.float64) for a in (got, g32, g64))
    nrm = max(np.linalg.norm(g64), 1e-30)
    rel = np.linalg.norm(got - g64) / nrm
    ref_rel = np.linalg.norm(g32 - g64) / nrm
    err = np.abs(got - g64).max()
    print(f"{what}: rel {rel:.2e} (oracle fp32 {ref_rel:.2e}), max|d|/max|g| {err / np.abs(g64).max():.2e}")
    assert rel <= max(1e-4, 4 * ref_rel), f"{what}: relative error {rel:.3e} (oracle fp32 {ref_rel:.3e})"
    assert err <= 2e-3 * np.abs(g64).max() + 1e-30, f"{what}: max|d| {err:.3e}"


def _weights_close(got, want, lr, what):
    d = np.abs(np.asarray(got, np.float64) - np.asarray(want, np.float64))
    assert d.max() <= 2 * lr + 1e-6, f"{what}: {d.max():.3e}"
    assert (d <= 1e-5).mean() >= 0.999, f"{what}: {(d > 1e-5).mean():.4%} of weights off by > 1e-5"


@pytest.mark.parametrize("name", CASES)
def test_train_steps_match_reference(name):
    """Two reference iterations: forward, mpjpe, backward, Adam(amsgrad) — the drop-in
    model in train mode with the native Adam (teacher-forced weights from step 1 on)."""
    from vp3d_amd.train import Adam
    g, meta, state = _load(name)
    m = _model(meta, state)
    opt = Adam(m.parameters(), lr=meta["lr"], amsgrad=meta["amsgrad"])
    for it in range(meta["steps"]):
        if it > 0:
            prev = {k[len(f"s{it - 1}/after/"):]: g[k] for k in g.files if k.startswith(f"s{it - 1}/after/")}
            m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in prev.items()})
            state = prev
        x = torch.from_numpy(g[f"s{it}/x"]).cuda()
        tgt = torch.from_numpy(g[f"s{it}/target"]).cuda()
        y = m(x)
        loss = torch.mean(torch.norm(y - tgt, dim=-1))  # common/loss.py:11-17
        opt.zero_grad()
        loss.backward()
        np.testing.assert_allclose(y.detach().cpu().numpy(), g[f"s{it}/y"], atol=1e-5, rtol=0)
        np.testing.assert_allclose(loss.item(), float(g[f"s{it}/loss"]), rtol=1e-5)
        _, _, g64, _ = _oracle(state, g[f"s{it}/x"], g[f"s{it}/target"], meta, dtype=torch.float64)
        for k, prm in m.named_parameters():
            _grad_close(prm.grad.cpu().numpy(), g[f"s{it}/grad/{k}"], g64[k], f"step {it} grad {k}")
        opt.step()
        for k, v in m.state_dict().items():
            if k.endswith("num_batches_tracked"):
                assert int(v) == it + 1
            elif "running" in k:
                np.testing.assert_allclose(v.cpu().numpy(), g[f"s{it}/after/{k}"], rtol=1e-5, atol=1e-6,
                                           err_msg=k)
            else:
                _weights_close(v.cpu().numpy(), g[f"s{it}/after/{k}"], meta["lr"], f"step {it} {k}")


def test_train_step_with_stock_torch_adam():
    """The autograd node feeds any torch optimiser (here torch.optim.Adam on the device)."""
    g, meta, state = _load("train_dilated_c64")
    m = _model(meta, state)
    opt = torch.optim.Adam(m.parameters(), lr=meta["lr"], amsgrad=True)
    x = torch.from_numpy(g["s0/x"]).cuda()
    tgt = torch.from_numpy(g["s0/target"]).cuda()
    loss = torch.mean(torch.norm(m(x) - tgt, dim=-1))
    opt.zero_grad()
    loss.backward()
    opt.step()
    for k, v in m.state_dict().items():
        if "running" not in k and not k.endswith("num_batches_tracked"):
            _weights_close(v.cpu().numpy(), g[f"s0/after/{k}"], meta["lr"], k)


def _masks(m, B, T, kind="dropout"):
    tr = m.native_trainer(torch.device("cuda", torch.cuda.current_device()))
    n_layers = 1 + 2 * (len(m.filter_widths) - 1)
    get = tr.dropout_mask if kind == "dropout" else tr.relu_mask
    return [get(l, m.channels).cpu().numpy() for l in range(n_layers)]


@pytest.mark.parametrize("strided,fw,B,T,channels", [
    (False, (3, 3, 3), 4, 35, 64),
    (True, (3, 3, 3), 16, 27, 64),
    (False, (3, 3, 3, 3, 3), 4, 243, 1024),
    (True, (3, 3, 3, 3, 3), 32, 243, 1024),
])
def test_train_dropout_parity_with_oracle(strided, fw, B, T, channels):
    """Dropout p = 0.25: the oracle fed the masks the trainer drew gives the same output,
    loss and gradients; about 75 % of the activations are kept."""
    p = 0.25
    torch.manual_seed(1234)  # the module draws its dropout seed from torch's generator
    meta = dict(strided=strided, fw=list(fw), causal=False, dense=False, channels=channels)
    from helpers import make_model
    _, sd = make_model(strided, fw, channels=channels, seed=5)
    m = _model(meta, sd, dropout=p)
    x = synth.normalized_windows(6, "drop", B, T)
    y = m(torch.from_numpy(x).cuda())
    tgt = synth.normal(7, "drop/target", tuple(y.shape), std=0.2).astype(np.float32)
    loss = torch.mean(torch.norm(y - torch.from_numpy(tgt).cuda(), dim=-1))
    loss.backward()
    masks = _masks(m, B, T)
    # kept fraction over every element of every layer: binomial, 4 sigma (the smallest
    # case has ~15k elements, sigma 0.35 %; a per-layer mean of means was 1.7 sigma at 1 %)
    n = sum(mk.size for mk in masks)
    keep = sum(float(mk.sum()) for mk in masks) / n
    assert abs(keep - 0.75) < max(0.005, 4 * np.sqrt(0.75 * 0.25 / n)), (keep, n)

    rm = _masks(m, B, T, "relu")
    y32, l32, g32, st32 = _oracle(sd, x, tgt, meta, p=p, masks=masks)
    _, _, g64, _ = _oracle(sd, x, tgt, meta, p=p, masks=masks, dtype=torch.float64, relu_masks=rm)
    # the fp32 yardstick with the same ReLU decisions
    _, _, g32, _ = _oracle(sd, x, tgt, meta, p=p, masks=masks, relu_masks=rm)
    np.testing.assert_allclose(y.detach().cpu().numpy(), y32, atol=1e-5, rtol=0)
    np.testing.assert_allclose(loss.item(), l32, rtol=1e-5)
    for k, prm in m.named_parameters():
        _grad_close(prm.grad.cpu().numpy(), g32[k], g64[k], k)
    for k, v in m.state_dict().items():
        if "running" in k:
            np.testing.assert_allclose(v.cpu().numpy(), st32[k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_train_dense_1024_large_wgrad():
    """--dense at the full size (3,3,3,3,3, 1024 channels, 243 frames): the last k-conv has
    163 taps, so one weight-gradient partial is 1024 x 166,912 floats (683 MB), larger than
    the 256 MB split budget; the partial buffer is sized from the largest layer."""
    meta = dict(strided=False, fw=[3, 3, 3, 3, 3], causal=False, dense=True, channels=1024)
    from helpers import make_model
    _, sd = make_model(False, (3, 3, 3, 3, 3), channels=1024, seed=9, dense=True)
    m = _model(meta, sd)
    B, T = 4, 243
    x = synth.normalized_windows(6, "dense1024", B, T)
    y = m(torch.from_numpy(x).cuda())
    tgt = synth.normal(7, "dense1024/target", tuple(y.shape), std=0.2).astype(np.float32)
    loss = torch.mean(torch.norm(y - torch.from_numpy(tgt).cuda(), dim=-1))
    loss.backward()
    torch.cuda.synchronize()
    rm = _masks(m, B, T, "relu")
    y64, l64, g64, _ = _oracle(sd, x, tgt, meta, dtype=torch.float64, relu_masks=rm)
    y32, l32, g32, _ = _oracle(sd, x, tgt, meta, relu_masks=rm)
    # the last blocks normalise over B rows per channel (one output frame per window), so
    # BatchNorm amplifies rounding: compare with the fp64 oracle, within 4x the fp32
    # oracle's own deviation from it (measured at B = 2: 3.3e-5 m vs fp32-oracle, 1e-5 gate)
    yd = np.abs(y.detach().cpu().numpy().astype(np.float64) - y64).max()
    y_ref_err = np.abs(y32.astype(np.float64) - y64).max()
    print(f"dense 1024 train forward: max|y - y64| {yd:.3e}, oracle fp32 {y_ref_err:.3e}")
    assert yd <= max(1e-5, 4 * y_ref_err), (yd, y_ref_err)
    assert abs(loss.item() - l64) <= max(1e-5 * abs(l64), 4 * abs(l32 - l64)), (loss.item(), l32, l64)
    for k, prm in m.named_parameters():
        _grad_close(prm.grad.cpu().numpy(), g32[k], g64[k], k)


def test_adam_kernel_bitexact_vs_torch():
    """vp3d_adam_step == torch.optim.Adam(amsgrad=True) (CPU, single-tensor path), 3 steps,
    tensors of assorted sizes (block tails, several tensors per launch)."""
    from vp3d_amd.train import Adam
    rng = np.random.default_rng(0)
    shapes = [(1024, 64, 3), (51, 1024, 1), (1024,), (7,), (3000,)]
    init = [rng.standard_normal(s).astype(np.float32) * 0.05 for s in shapes]
    cpu = [torch.tensor(a, requires_grad=True) for a in init]
    gpu = [torch.nn.Parameter(torch.tensor(a).cuda()) for a in init]
    o_cpu = torch.optim.Adam(cpu, lr=1e-3, amsgrad=True)
    o_gpu = Adam(gpu, lr=1e-3, amsgrad=True)
    n_diff = n_all = 0
    for it in range(3):
        for c, gp, s in zip(cpu, gpu, shapes):
            gr = (rng.standard_normal(s) * 10.0 ** rng.integers(-6, 1)).astype(np.float32)
            c.grad = torch.tensor(gr)
            gp.grad = torch.tensor(gr).cuda()
        o_cpu.step()
        o_gpu.step()
        sc, sg = o_cpu.state_dict()["state"], o_gpu.state_dict()["state"]
        for i in sc:
            for key in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
                np.testing.assert_array_equal(sg[i][key].cpu().numpy(), sc[i][key].numpy(), err_msg=key)
        for c, gp in zip(cpu, gpu):
            a, b = gp.detach().cpu().numpy(), c.detach().numpy()
            # 1 ulp of the update term (|update| <~ 4 lr) or of the parameter, whichever is larger:
            # the cases are the update terms whose sqrt torch-CPU rounds the other way
            tol = np.spacing(np.maximum(np.abs(b), np.float32(4e-3)))
            d = np.abs(a.astype(np.float64) - b.astype(np.float64))
            assert (d <= tol).all(), float((d / tol).max())
            n_diff += int((d > 0).sum())
            n_all += d.size
            c.data.copy_(torch.from_numpy(a))  # continue from identical parameters
    assert n_diff / n_all < 0.03, n_diff / n_all
    for i in sc:
        assert float(sg[i]["step"]) == float(sc[i]["step"]) == 3.0


def test_native_writes_bump_versions():
    """Adam and the running-stat update write through raw pointers; the version counters
    move so (a) the eval lifter re-folds after a step, (b) a step between a forward and
    its backward is caught by autograd's saved-tensor check."""
    from vp3d_amd.train import Adam
    g, meta, state = _load("train_dilated_c64")
    m = _model(meta, state)
    opt = Adam(m.parameters(), lr=meta["lr"], amsgrad=True)
    x = torch.from_numpy(g["s0/x"]).cuda()
    tgt = torch.from_numpy(g["s0/target"]).cuda()
    loss = torch.mean(torch.norm(m(x) - tgt, dim=-1))
    opt.zero_grad()
    loss.backward()
    m.eval()
    with torch.no_grad():
        y_before = m(x).clone()
    opt.step()
    with torch.no_grad():
        y_after = m(x)
    assert not torch.equal(y_before, y_after)  # the lifter saw the updated weights
    # the eval output equals a fresh model built from the stepped state
    fresh = _model(meta, {k: v.cpu().numpy() for k, v in m.state_dict().items()}).eval()
    with torch.no_grad():
        torch.testing.assert_close(fresh(x), y_after, rtol=0, atol=0)
    m.train()
    loss = torch.mean(torch.norm(m(x) - tgt, dim=-1))
    opt.zero_grad()
    loss.backward(retain_graph=True)
    opt.step()
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        loss.backward()


def test_train_errors():
    g, meta, state = _load("train_opt1f_c64")
    m = _model(meta, state)
    with pytest.raises(RuntimeError):
        m.cpu()(torch.from_numpy(g["s0/x"]))
    m.cuda()
    x = torch.from_numpy(g["s0/x"]).cuda()
    y1 = m(x)
    m(x)  # a second forward replaces the trainer's saved activations
    with pytest.raises(RuntimeError, match="another train-mode forward"):
        y1.sum().backward()
    with pytest.raises(AssertionError):  # Optimized1f trains on receptive-field windows only
        m(torch.cat([x, x[:, :3]], dim=1))
