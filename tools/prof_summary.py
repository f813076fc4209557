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
    m = re.search(r"(conv_gemm_(h16|f32|q64|q4w|8p)|expand_gemm_h16)[^(]*", name)
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


def per_layer(trace, B):
    """Per-layer durations by dispatch order: a forward of batch B starts at its expand
    dispatch (fused expand kernel, grid = ceil(B*81/256)*256 threads) and is followed by
    the 9 conv-GEMM dispatches of blocks 1-4 (each with its split-K tail launches, if any) and
    the shrink (a conv-GEMM, or the f16x3 shrink's split + reduce launches)."""
    layers = ["expand", "block1_k3", "block1_1x1", "block2_k3", "block2_1x1", "block3_k3",
              "block3_1x1", "block4_k3", "block4_1x1", "shrink"]
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
                continue
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows.sort()
    # the expand grid of the largest forward in the trace (the bench's batch; the 16-bit
    # expand's grid depends on its row-block form, so it is not derived from B)
    eg = max((r[2] for r in rows if "expand_gemm" in r[1]), default=0)
    starts = "expand_gemm"
    if eg == 0:  # the fp32 path: the expand is the largest conv_gemm_f32 launch
        eg = max((r[2] for r in rows if "conv_gemm_f32" in r[1]), default=0)
        starts = "conv_gemm_f32"
    # a layer starts at a conv_gemm dispatch, or at a split-K tail dispatch of ONE 64-column
    # block (the f16x3 shrink since round 6: tail_split_kernel + shrink_reduce_x3_kernel); the
    # other split-tail and reduce dispatches belong to the layer before them (its tail)
    def opens(r):
        return "conv_gemm" in r[1] or ("tail_split_kernel" in r[1] and r[2] == 256)

    def joins(r):
        return "tail_split_kernel" in r[1] or "reduce" in r[1]
    agg = defaultdict(list)
    names = {}
    i = 0
    while i < len(rows):
        if starts in rows[i][1] and rows[i][2] == eg:
            seq = [[rows[i][3], short(rows[i][1])]]
            j = i + 1
            while j < len(rows):
                r = rows[j]
                if opens(r):
                    if len(seq) == len(layers):
                        break
                    seq.append([r[3], short(r[1]) if "conv_gemm" in r[1] else "tail_split_kernel + shrink_reduce (f16x3 shrink)"])
                elif joins(r) and len(seq) > 1:
                    seq[-1][0] += r[3]
                    if "+ tail" not in seq[-1][1] and "shrink" not in seq[-1][1]:
                        seq[-1][1] += " + tail"
                elif starts in r[1] and r[2] == eg:
                    break
                j += 1
            if len(seq) == len(layers):
                for name, (d, k) in zip(layers, seq):
                    agg[name].append(d)
                    names[name] = k
            i = j
        else:
            i += 1
    print()
    print(f"Per layer (forwards of B = {B}, by dispatch order):")
    print()
    print("| layer | kernel | calls | avg us | min us | max us |")
    print("|---|---|---|---|---|---|")
    for name in layers:
        ds = sorted(agg.get(name, []))
        if ds:
            print(f"| {name} | {names[name]} | {len(ds)} | {sum(ds) / len(ds):.1f} | {ds[0]:.1f} | {ds[-1]:.1f} |")


if __name__ == "__main__":
    main()
    import sys
    if len(sys.argv) > 1:
        B = 8192
        if "--batch" in sys.argv:
            B = int(sys.argv[sys.argv.index("--batch") + 1])
        per_layer(sys.argv[1], B)
