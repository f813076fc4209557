"""Training step of the temporal lifter on the MI355X kernels.

The reference trains `TemporalModel` in train mode inside run.py's loop
(run.py:451-487): forward with BatchNorm batch statistics and dropout, mpjpe,
``loss.backward()``, ``optimizer.step()`` with ``optim.Adam(..., amsgrad=True)``
(run.py:662), BN momentum decayed per epoch (run.py:553-556).

* `NativeTrainer` owns a ``vp3d_trainer`` (include/vp3d.h): the f32 train-mode
  forward and the backward of every layer run in libvp3d.so; the parameters stay in
  the module's own tensors and are passed by device pointer on every call.
* `TrainStep` is the autograd node the drop-in `TemporalModelBase.forward` uses in
  train mode, so a reference training loop (`loss.backward()`, any torch optimiser)
  runs unchanged.
* `Adam` is a drop-in for ``torch.optim.Adam`` (same arguments, same state keys, so
  checkpoints interchange) whose step is one native launch over up to 64 tensors.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

import torch
from torch.autograd.graph import increment_version

from . import _native as N


def _ptrs(tensors: Sequence) -> ctypes.Array:
    return (ctypes.c_void_p * len(tensors))(*[0 if t is None else t.data_ptr() for t in tensors])


class NativeTrainer:
    """One vp3d_trainer on one HIP device (geometry of one lifter configuration)."""

    def __init__(self, num_joints_in: int, in_features: int, num_joints_out: int,
                 filter_widths: Sequence[int], causal: bool, channels: int, dense: bool,
                 variant: int, device, bn_eps: float = 1e-5):
        self._lib = N.load()
        self.cfg = N.make_cfg(num_joints_in, in_features, num_joints_out, filter_widths, causal,
                              channels, dense, variant, bn_eps)
        self.n_params = self._lib.vp3d_weight_count(ctypes.byref(self.cfg))
        if self.n_params < 0:
            raise AssertionError("invalid lifter configuration")
        self.device = torch.device(device)
        self.num_joints_out = num_joints_out
        self.generation = 0
        self._h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_trainer_create(ctypes.byref(self.cfg), ctypes.byref(self._h)),
                    "vp3d_trainer_create")
        # a scratch handle-free helper for output lengths
        self._out_frames = None

    def forward(self, x: torch.Tensor, params: Sequence[torch.Tensor], p: float, momentum: float,
                seed: int, T_out: int) -> torch.Tensor:
        """Train-mode forward.  params: the state_dict tensors in order (running stats are
        updated in place).  Returns y (B, T_out, J_out, 3)."""
        assert len(params) == self.n_params, (len(params), self.n_params)
        B, T = int(x.shape[0]), int(x.shape[1])
        y = torch.empty((B, T_out, self.num_joints_out, 3), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_train_forward(self._h, _ptrs(params), len(params), x.data_ptr(), B, T,
                                                 float(p), float(momentum), int(seed) & (2 ** 64 - 1),
                                                 y.data_ptr(), N.stream_ptr(self.device)),
                    "vp3d_train_forward")
        # the running statistics were written through raw pointers: bump their version
        # counters so caches keyed on them (the eval lifter's folded weights) see the change
        increment_version([t for t in params if not t.requires_grad])
        self.generation += 1
        return y

    def backward(self, params: Sequence[torch.Tensor], dy: torch.Tensor,
                 trainable: Sequence[bool]) -> List[torch.Tensor | None]:
        grads = [torch.empty_like(t) if tr else None for t, tr in zip(params, trainable)]
        dy = dy.contiguous().float()
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_train_backward(self._h, _ptrs(params), len(params), dy.data_ptr(),
                                                  _ptrs(grads), N.stream_ptr(self.device)),
                    "vp3d_train_backward")
        return grads

    def layer_rows(self, layer: int) -> int:
        return int(self._lib.vp3d_train_layer_rows(self._h, layer))

    def dropout_mask(self, layer: int, channels: int) -> torch.Tensor:
        """Keep mask (uint8, rows x channels) of conv layer `layer` in the latest forward."""
        rows = self.layer_rows(layer)
        if rows < 0:
            raise RuntimeError("no train-mode forward yet")
        out = torch.empty((rows, channels), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_train_dropout_mask(self._h, layer, out.numel(), out.data_ptr(),
                                                      N.stream_ptr(self.device)), "vp3d_train_dropout_mask")
        return out

    def relu_mask(self, layer: int, channels: int) -> torch.Tensor:
        """ReLU mask (uint8, rows x channels: BN output > 0) of conv layer `layer` in the latest
        forward (test hook)."""
        rows = self.layer_rows(layer)
        if rows < 0:
            raise RuntimeError("no train-mode forward yet")
        out = torch.empty((rows, channels), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_train_relu_mask(self._h, layer, out.numel(), out.data_ptr(),
                                                   N.stream_ptr(self.device)), "vp3d_train_relu_mask")
        return out

    def close(self) -> None:
        if self._h:
            self._lib.vp3d_trainer_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TrainStep(torch.autograd.Function):
    """y = lifter(x) in train mode; the backward yields every parameter's gradient."""

    @staticmethod
    def forward(ctx, trainer: NativeTrainer, p: float, momentum: float, seed: int, T_out: int,
                trainable: tuple, x: torch.Tensor, *state: torch.Tensor):
        y = trainer.forward(x, state, p, momentum, seed, T_out)
        ctx.trainer = trainer
        ctx.generation = trainer.generation
        ctx.trainable = trainable
        # x and the parameters must be the ones the backward sees (the trainer keeps the
        # activations); the native Adam bumps the version counters of what it writes, so an
        # optimiser step between this forward and its backward fails torch's saved-tensor check
        # (the running statistics, which every train-mode forward rewrites, are held by
        # reference only: a second forward is reported by the generation check below)
        ctx.save_for_backward(x, *[t for t, tr in zip(state, trainable) if tr])
        ctx.state = state
        return y

    @staticmethod
    def backward(ctx, dy):
        trainer = ctx.trainer
        if trainer.generation != ctx.generation:
            raise RuntimeError("vp3d: another train-mode forward of this model ran before this backward; "
                               "the native trainer keeps the activations of the latest forward only")
        ctx.saved_tensors  # version check of x and the trained parameters
        grads = trainer.backward(ctx.state, dy, ctx.trainable)
        return (None, None, None, None, None, None, None, *grads)


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (run.py:662: ``optim.Adam(params, lr=lr, amsgrad=True)``) with the
    update of all tensors of a step in one native launch per 64 tensors (vp3d_adam_step).

    Same constructor arguments and per-parameter state (``step``, ``exp_avg``,
    ``exp_avg_sq``, ``max_exp_avg_sq``) as torch's, so ``state_dict`` /
    ``load_state_dict`` interchange with ``torch.optim.Adam`` checkpoints
    (run.py:563-569).  Parameters must be float32 HIP tensors."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      amsgrad=amsgrad, maximize=False, foreach=None, capturable=False,
                                      differentiable=False, fused=None))
        self._lib = N.load()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            amsgrad = group["amsgrad"]
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients")
                if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous():
                    raise RuntimeError("vp3d Adam: parameters must be contiguous float32 HIP tensors")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    if amsgrad:
                        st["max_exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(p)
            for step, plist in by_step.items():
                for i in range(0, len(plist), 64):
                    chunk = plist[i:i + 64]
                    dev = chunk[0].device
                    sts = [self.state[p] for p in chunk]
                    grads = [p.grad.contiguous() for p in chunk]
                    numel = (ctypes.c_int64 * len(chunk))(*[p.numel() for p in chunk])
                    vmax = _ptrs([s["max_exp_avg_sq"] for s in sts]) if amsgrad else None
                    with torch.cuda.device(dev):
                        N.check(self._lib.vp3d_adam_step(
                            len(chunk), _ptrs(chunk), _ptrs(grads), _ptrs([s["exp_avg"] for s in sts]),
                            _ptrs([s["exp_avg_sq"] for s in sts]), vmax, numel, float(group["lr"]),
                            float(beta1), float(beta2), float(group["eps"]), float(group["weight_decay"]),
                            step, 1 if amsgrad else 0, N.stream_ptr(dev)), "vp3d_adam_step")
                    # written through raw pointers: make the in-place update visible to
                    # autograd's saved-tensor checks and to the eval lifter's weight cache
                    increment_version(chunk)
        return loss
