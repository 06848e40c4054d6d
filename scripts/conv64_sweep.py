"""The f64 conv engine on RMVPE's U-Net conv shapes (30 s clip: 3008 x 128 mel image): the planner's choice
against forced (tile, split-K, compact) plans, timed alone with events; every forced plan is checked against
the planner's output.  Writes a JSON table for calibrating plan64's time model.

    python scripts/conv64_sweep.py [out.json] [--quick]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rvc-maker_amd")]
from rvc_amd import ops  # noqa: E402

TILES = ["16x512", "16x256", "32x256", "32x128", "64x128", "64x64", "128x128", "128x64", "16x256/32", "32x128/32",
         "64x128/32", "64x64/32", "128x64/32", "128x16", "128x16/32", "16x256/36", "32x128/36", "32x256/36"]
# (Ci, Co, H, W): one 3x3 conv per U-Net level (every level's convs are 1.77 GFLOP), the encoder's first conv
SHAPES = [(16, 16, 3008, 128), (32, 32, 1504, 64), (64, 64, 752, 32), (128, 128, 376, 16), (256, 256, 188, 8),
          (512, 512, 94, 4), (256, 512, 94, 4), (1, 16, 3008, 128)]
# --direct: the convs the f64 RMVPE still runs direct on a 30 s clip after filtfilt / t_pad (mel image 3232 x 128;
# levels >= 2 of >= 64 channels go Winograd): encoder, decoder (concat input) and the 512-channel middle
SHAPES_DIRECT = [(1, 16, 3232, 128), (16, 16, 3232, 128), (32, 16, 3232, 128), (16, 32, 1616, 64), (32, 32, 1616, 64),
                 (64, 32, 1616, 64), (32, 64, 808, 32), (512, 512, 101, 4), (256, 512, 101, 4), (512, 256, 101, 4)]


def run(x, w, b, Ci, Co, H, W, out, reps):
    wrap = W + 2
    L = (H + 2) * wrap
    toff = [dy * wrap + dx for dy in range(3) for dx in range(3)]
    kw = dict(bias=b, pad=wrap + 1, Lin=L, Lout=L, out=out, toff=toff, wrap=wrap, out_act=ops.ACT_RELU, B=1)
    plan = ops.conv64(x, w, Ci, Co, 9, plan=True, **kw)
    ops.conv64(x, w, Ci, Co, 9, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.conv64(x, w, Ci, Co, 9, **kw)
    e1.record()
    torch.cuda.synchronize()
    return plan, e0.elapsed_time(e1) / reps * 1e3


def main():
    path = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "gpurun_out/conv64_sweep.json"
    quick = "--quick" in sys.argv
    planner_only = "--planner-only" in sys.argv
    torch.manual_seed(0)
    rows = []
    for Ci, Co, H, W in (SHAPES_DIRECT if "--direct" in sys.argv else SHAPES):
        L = (H + 2) * (W + 2)
        x = torch.zeros(Ci, H + 2, W + 2, dtype=torch.float64, device="cuda")
        x[:, 1:-1, 1:-1] = torch.randn(Ci, H, W, dtype=torch.float64, device="cuda")
        w = (torch.randn(Ci * 9, Co, dtype=torch.float64, device="cuda") / (3 * Ci ** 0.5)).contiguous()
        b = torch.randn(Co, dtype=torch.float64, device="cuda")
        out = torch.empty(Co, H + 2, W + 2, dtype=torch.float64, device="cuda")
        gflop = 2 * Ci * Co * 9 * H * W / 1e9
        ops.conv64_set_plan()
        plan, us = run(x, w, b, Ci, Co, H, W, out, 20)
        ref = out.clone()
        # torch's own f64 conv as the check of the planner's plan (interior; the border must be 0)
        tw = w.t().reshape(Co, Ci, 3, 3).contiguous()
        tr = torch.relu(torch.nn.functional.conv2d(x[None, :, 1:-1, 1:-1], tw, b, padding=1))[0]
        err = (ref[:, 1:-1, 1:-1] - tr).abs().max().item() / max(tr.abs().max().item(), 1e-30)
        border = max(ref[:, 0].abs().max().item(), ref[:, -1].abs().max().item(), ref[:, :, 0].abs().max().item(),
                     ref[:, :, -1].abs().max().item())
        print(f"Ci {Ci:3d} Co {Co:3d} {H}x{W}: planner {TILES[plan[0]]} ks {plan[1]} cmp {plan[2]} "
              f"({plan[3]} blocks) {us:7.1f} us {gflop / us * 1e3:5.1f} TF  rel err {err:.1e} border {border:.0e}",
              flush=True)
        row = {"Ci": Ci, "Co": Co, "H": H, "W": W, "planner": list(plan), "us": us, "err": err, "border": border,
               "forced": []}
        best = (us, plan)
        if planner_only:
            rows.append(row)
            continue
        kss = [1, 2, 4, 8, 16, 32] if quick else [1, 2, 3, 4, 6, 8, 12, 16, 21, 24, 32]
        for t in range(len(TILES)):
            for cmp in (0, 1):
                for ks in kss:
                    try:
                        ops.conv64_set_plan(t, ks, cmp)
                        out.fill_(float("nan"))
                        p, u = run(x, w, b, Ci, Co, H, W, out, 10)
                    except (RuntimeError, ValueError):
                        continue
                    d = (out - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
                    row["forced"].append({"plan": list(p), "us": u, "diff": d})
                    if d > 1e-12 or d != d:
                        print(f"   MISMATCH {TILES[p[0]]} ks {p[1]} cmp {p[2]}: {d:.2e}", flush=True)
                    if u < best[0]:
                        best = (u, p)
        ops.conv64_set_plan()
        print(f"   best forced {TILES[best[1][0]]} ks {best[1][1]} cmp {best[1][2]} ({best[1][3]} blocks) "
              f"{best[0]:7.1f} us {gflop / best[0] * 1e3:5.1f} TF", flush=True)
        rows.append(row)
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump(rows, f)


if __name__ == "__main__":
    main()
