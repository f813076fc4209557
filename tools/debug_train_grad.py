"""Debug helper: native train step (1f 243, dropout 0.25) vs fp64 oracle fed the same
masks, for several dropout seeds; prints per-tensor relative errors and the worst channels
of expand_bn.weight's gradient."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dynamic-camera-augmented-videopose3d_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_train import _model, _masks, _oracle  # noqa: E402
from helpers import make_model  # noqa: E402
from vp3d_amd import synth  # noqa: E402

strided, fw, B, T, C = True, (3, 3, 3, 3, 3), 32, 243, 1024
meta = dict(strided=strided, fw=list(fw), causal=False, dense=False, channels=C)
_, sd = make_model(strided, fw, channels=C, seed=5)
x = synth.normalized_windows(6, "drop", B, T)
for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    torch.manual_seed(seed)
    m = _model(meta, sd, dropout=0.25)
    y = m(torch.from_numpy(x).cuda())
    tgt = synth.normal(7, "drop/target", tuple(y.shape), std=0.2).astype(np.float32)
    loss = torch.mean(torch.norm(y - torch.from_numpy(tgt).cuda(), dim=-1))
    loss.backward()
    masks = _masks(m, B, T)
    rm = _masks(m, B, T, "relu") if os.environ.get("RELU_MASKS", "1") == "1" else None
    _, _, g64, _ = _oracle(sd, x, tgt, meta, p=0.25, masks=masks, dtype=torch.float64, relu_masks=rm)
    worst = []
    for k, prm in m.named_parameters():
        got = prm.grad.cpu().numpy().astype(np.float64)
        rel = np.linalg.norm(got - g64[k]) / np.linalg.norm(g64[k])
        worst.append((rel, k))
    worst.sort(reverse=True)
    print(f"seed {seed}: worst", [(f"{r:.2e}", k) for r, k in worst[:4]], flush=True)
    k = "expand_bn.weight"
    got = m.expand_bn.weight.grad.cpu().numpy().astype(np.float64)
    d = np.abs(got - g64[k])
    idx = np.argsort(-d)[:5]
    print("   expand_bn.weight worst channels", [(int(i), f"{got[i]:.4e}", f"{g64[k][i]:.4e}") for i in idx], flush=True)
    m.zero_grad()
