"""Per-launch accuracy of the conv engines against an f64 evaluation of the same f32 operands: the split-bf16
engine at 6 and 8 passes, the split-fp16 form, and the f32-MFMA engine, next to torch-CPU f32 (what the
reference executes).  RMVPE-like shapes (K = 3 taps over 16..512 channels, K = 1 GEMMs).

    python scripts/conv_prec.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))


def main():
    from rvc_amd import ops
    torch.manual_seed(0)
    dev = "cuda"
    shapes = [(16, 16, 3, 65536), (64, 64, 3, 16384), (256, 256, 3, 2048), (512, 512, 3, 1024), (512, 384, 1, 4096),
              (1536, 384, 1, 3232)]
    for Co, Ci, K, L in shapes:
        x = torch.randn(Ci, L) * 3 + 1  # ReLU'd-like, non-zero mean: sums with cancellation
        x = torch.relu(x)
        w = torch.randn(Co, Ci, K) / (Ci * K) ** 0.5
        ref = torch.nn.functional.conv1d(x.double()[None], w.double(), padding=K // 2)[0]
        scale = torch.nn.functional.conv1d(x.double().abs()[None], w.double().abs(), padding=K // 2)[0]
        cpu = torch.nn.functional.conv1d(x[None], w, padding=K // 2)[0].double()
        cw = ops.Conv(w, None, device=dev)
        xd = x.to(dev)
        row = [f"Co {Co:4d} Ci {Ci:4d} K {K} L {L:6d}:"]

        def err(y):
            e = (y.double().cpu() - ref) / scale
            return f"{float(e.pow(2).mean().sqrt()):.2e}/{float(e.abs().max()):.2e}"
        row.append(f"torch-cpu f32 {err(cpu)}")
        for name in ("fp32x6", "fp32sa", "f16x3"):
            with ops.precision(name):
                y = cw(xd, pad=K // 2)
            row.append(f"{name} {err(y)}")
        y = ops.conv1d(xd, cw.w, Ci, Co, K, pad=K // 2, wx=None)
        row.append(f"f32-mfma {err(y)}")
        torch.cuda.synchronize()
        print("  ".join(row), flush=True)
    print("(relative error rms/max, normalised by sum |x||w| per output)")


if __name__ == "__main__":
    main()
