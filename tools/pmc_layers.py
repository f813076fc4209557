#!/usr/bin/env python3
"""Per-layer PMC counters of the lifter forward (one rocprofv3 --pmc pass).

    python tools/pmc_layers.py gpurun_out/TAG/pmc_bf16_busy [--batch 65536] [--out profiles/x.md]

Orders the dispatches by Dispatch_Id, splits them into forwards of the bench batch (as
tools/traffic.py: the largest expand dispatch starts a forward, the next 9 GEMM dispatches
are blocks 1-4 and the shrink) and prints, per layer, the mean of every counter over the
forwards plus the derived fractions (MI355X_MICROARCH.md, PMC rows):
  * sclk_mhz = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration
  * mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the share of
    SIMD cycles the matrix cores were busy (16 cycles per 16x16x32 16-bit MFMA)
  * wait_inst = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES: issue stalls per wave cycle
  * busy = SQ_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8)
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

LAYERS = ["expand", "block1_k3", "block1_1x1", "block2_k3", "block2_1x1", "block3_k3",
          "block3_1x1", "block4_k3", "block4_1x1", "shrink"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--out")
    a = ap.parse_args()
    disp = defaultdict(dict)  # dispatch id -> {counter: value, "_name", "_grid", "_ns"}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                d = disp[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = float(r["Counter_Value"])
                d["_name"] = r["Kernel_Name"]
                d["_grid"] = int(r["Grid_Size"])
                d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    ids = sorted(disp)
    eg = max((disp[i]["_grid"] for i in ids if "expand_gemm" in disp[i]["_name"]), default=0)
    acc = defaultdict(lambda: defaultdict(list))
    i = 0
    while i < len(ids):
        d = disp[ids[i]]
        if "expand_gemm" not in d["_name"] or d["_grid"] != eg:
            i += 1
            continue
        seq = [d]
        j = i + 1
        while j < len(ids) and len(seq) < len(LAYERS):
            nm = disp[ids[j]]["_name"]
            # (the f16x3 shrink since round 6: its split launch stands for the layer; config 4 at
            # 65,536 windows has no other split-K tails)
            if "conv_gemm" in nm or ("tail_split_kernel" in nm and len(seq) == len(LAYERS) - 1):
                seq.append(disp[ids[j]])
            j += 1
        if len(seq) == len(LAYERS):
            for name, e in zip(LAYERS, seq):
                for k, v in e.items():
                    if not k.startswith("_") or k == "_ns":
                        acc[name][k].append(v)
        i = j
    counters = sorted({k for v in acc.values() for k in v if not k.startswith("_")})
    lines = [f"Per-layer PMC means over {min((len(v['_ns']) for v in acc.values()), default=0)} forwards "
             f"of B = {a.batch} ({a.dir})", "",
             "| layer | ms | " + " | ".join(counters) + " | sclk MHz | mfma_busy | wait_inst | busy |",
             "|---|---|" + "---|" * (len(counters) + 4)]
    for name in LAYERS:
        if name not in acc:
            continue
        m = {k: sum(v) / len(v) for k, v in acc[name].items()}
        ms = m["_ns"] / 1e6
        gui = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        sclk = gui / (m["_ns"] * 1e-3) if gui and m["_ns"] else 0.0
        mb = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui * 1024) if gui else 0.0
        wi = m.get("SQ_WAIT_INST_ANY", 0.0) / m["SQ_WAVE_CYCLES"] if m.get("SQ_WAVE_CYCLES") else 0.0
        bz = m.get("SQ_BUSY_CYCLES", 0.0) / gui if gui else 0.0
        lines.append(f"| {name} | {ms:.3f} | " + " | ".join(f"{m[c]:.4g}" for c in counters) +
                     f" | {sclk:.0f} | {mb:.3f} | {wi:.3f} | {bz:.3f} |")
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
