"""Per-launch accuracy of the conv engines against an f64 evaluation of the same f32 operands: the split-bf16
engine at 6 and 8 passes, the split-fp16 form, and the f32-MFMA engine, next to torch-CPU f32 (what the
reference executes).  RMVPE-like shapes (K = 3 taps over 16..512 channels, K = 1 GEMMs).

    python scripts/conv_prec.py
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gen", action="store_true")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    from rvc_amd import ops
    torch.manual_seed(0)
    dev = "cuda"
    shapes = [(16, 16, 3, 1, 65536), (64, 64, 3, 1, 16384), (256, 256, 3, 1, 2048), (512, 512, 3, 1, 1024),
              (512, 384, 1, 1, 4096), (1536, 384, 1, 1, 3232)]
    if args.gen:  # GeneratorNSF ResBlock convs (synthesizers.py:149-159, residuals.py:22-44), 48k v2 stage widths
        shapes = [(128, 128, k, d, 65536) for k, d in ((3, 1), (3, 3), (7, 1), (7, 5), (11, 1), (11, 5))] + \
                 [(256, 256, k, d, 16384) for k, d in ((3, 1), (3, 5), (7, 3), (11, 1), (11, 5))]
    lines = []
    for Co, Ci, K, dil, L in shapes:
        if args.gen:  # the generator's activations: a ResBlock input after leaky ReLU (0.1), heavy-tailed
            x = torch.randn(Ci, L) * torch.exp(torch.randn(Ci, 1))
            x = torch.where(x >= 0, x, 0.1 * x)
        else:
            x = torch.randn(Ci, L) * 3 + 1  # ReLU'd-like, non-zero mean: sums with cancellation
            x = torch.relu(x)
        w = torch.randn(Co, Ci, K) / (Ci * K) ** 0.5
        pad = dil * (K - 1) // 2
        ref = torch.nn.functional.conv1d(x.double()[None], w.double(), padding=pad, dilation=dil)[0]
        scale = torch.nn.functional.conv1d(x.double().abs()[None], w.double().abs(), padding=pad, dilation=dil)[0]
        cpu = torch.nn.functional.conv1d(x[None], w, padding=pad, dilation=dil)[0].double()
        cw = ops.Conv(w, None, device=dev)
        xd = x.to(dev)
        row = [f"Co {Co:4d} Ci {Ci:4d} K {K:2d} d {dil} L {L:6d}:"]

        def err(y):
            e = (y.double().cpu() - ref) / scale
            return f"{float(e.pow(2).mean().sqrt()):.2e}/{float(e.abs().max()):.2e}"
        row.append(f"torch-cpu f32 {err(cpu)}")
        for name in ("fp32x6", "fp32sa", "f16x3"):
            with ops.precision(name):
                y = cw(xd, pad=pad, dil=dil)
            row.append(f"{name} {err(y)}")
        if args.gen:
            cell = ops.AmaxSlots(1, dev)
            cell.words[0] = int(np.float32(x.abs().max().item()).view(np.int32))
            with ops.precision("f16x3"):
                y = cw(xd, pad=pad, dil=dil, amax_in=cell[0])
            row.append(f"f16x3-amax {err(y)}")
        y = ops.conv1d(xd, cw.w, Ci, Co, K, pad=pad, dil=dil, wx=None)
        row.append(f"f32-mfma {err(y)}")
        torch.cuda.synchronize()
        lines.append("  ".join(row))
        print(lines[-1], flush=True)
    lines.append("(relative error rms/max, normalised by sum |x||w| per output)")
    print(lines[-1])
    if args.out:
        with open(args.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
