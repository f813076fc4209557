#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid) so that the
per-layer launches of the lifter can be matched to bench.py's HIP-event timings.

    python tools/prof_summary.py gpurun_out/TAG/prof/run_kernel_trace.csv [--batch 8192]

Each conv layer of the 243-RF Optimized1f lifter launches one conv_gemm kernel
with a distinct grid (M = B * T_out rows, 128x128 tiles), so the grid size
identifies the layer.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"conv_gemm_(h16|f32)[^(]*", name)
    if m:
        return m.group(0)[:80]
    return name[:80]


def layer_table(B, fw=(3, 3, 3, 3, 3), C=1024, jout=17):
    rows = []
    L = 243 // 3
    rows.append(("expand", B * L, C))
    for i in range(1, len(fw)):
        L = L // 3
        rows.append((f"block{i}_k3", B * L, C))
        rows.append((f"block{i}_1x1", B * L, C))
    rows.append(("shrink", B * L, jout * 3))
    out = {}
    for name, M, N in rows:
        g = ((M + 127) // 128) * ((N + 127) // 128) * 256
        out.setdefault(g, []).append(name)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--batch", type=int, default=8192)
    a = ap.parse_args()
    agg = defaultdict(list)
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
                continue
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            agg[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]))].append(d)
    lt = layer_table(a.batch)
    print("| kernel | grid (work-items) | layer(s) | calls | avg us | min us | max us |")
    print("|---|---|---|---|---|---|---|")
    for (k, g), ds in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if sum(ds) < 20:
            continue
        ds_sorted = sorted(ds)
        print(f"| {k} | {g} | {'/'.join(lt.get(g, ['-']))} | {len(ds)} | "
              f"{sum(ds) / len(ds):.1f} | {ds_sorted[0]:.1f} | {ds_sorted[-1]:.1f} |")


if __name__ == "__main__":
    main()
