"""The f64 RMVPE on the device: conv64 units against torch f64 on the host, then the whole salience of the
headline clip (BASELINE configs[1], tests/test_gpu_configs.py seeds) against the exact (f64) oracle, and the
RMVPE time per 30 s clip in the f64 form and the round-3 f32 form (fp32sa).

    python scripts/rmvpe64_check.py [--skip-oracle]
"""
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rvc-maker_amd"), os.path.join(ROOT, "tests")]
from rvc_amd import ops, synthetic  # noqa: E402

DEV = "cuda"


def conv_units():
    g = torch.Generator().manual_seed(0)
    worst = 0.0
    for (Ci, Co, H, W, B, res, sc) in [(1, 16, 64, 128, 1, False, False), (16, 16, 96, 128, 1, True, False),
                                       (16, 32, 48, 64, 2, True, False), (64, 64, 24, 32, 1, False, False),
                                       (256, 512, 6, 4, 1, True, False), (512, 512, 6, 4, 2, True, False),
                                       (32, 16, 40, 64, 1, False, True), (300, 128, 5, 9, 1, False, True)]:
        k = 1 if sc else 3
        x = torch.randn(B, Ci, H, W, generator=g, dtype=torch.float64)
        w = torch.randn(Co, Ci, k, k, generator=g, dtype=torch.float64) / (Ci * k * k) ** 0.5
        b = torch.randn(Co, generator=g, dtype=torch.float64)
        r = torch.randn(B, Co, H, W, generator=g, dtype=torch.float64) if res else None
        want = F.relu(F.conv2d(x, w, b, padding=k // 2))
        if res:
            want = want + r
        xb = torch.zeros(B, Ci, H + 2, W + 2, dtype=torch.float64)
        xb[:, :, 1:-1, 1:-1] = x
        rb = None
        if res:
            rb = torch.zeros(B, Co, H + 2, W + 2, dtype=torch.float64)
            rb[:, :, 1:-1, 1:-1] = r
            rb = rb.to(DEV)
        wrap, L = W + 2, (H + 2) * (W + 2)
        toff = [dy * wrap + dx for dy in range(k) for dx in range(k)]
        out = torch.full((B, Co, H + 2, W + 2), float("nan"), dtype=torch.float64, device=DEV)
        wkm = ops.pack_km(w.reshape(Co, Ci, k * k)).to(DEV)
        xd = xb.to(DEV)
        ops.conv64(xd if B > 1 else xd[0], wkm, Ci, Co, k * k, bias=b.to(DEV), pad=(wrap + 1) if k == 3 else 0,
                   Lin=L, Lout=L, out=out if B > 1 else out[0], res=(rb if B > 1 else rb[0]) if res else None,
                   out_act=ops.ACT_RELU, toff=toff, wrap=wrap, B=B,
                   x_bstride=xd.stride(0) if B > 1 else 0, y_bstride=out.stride(0) if B > 1 else 0,
                   res_bstride=rb.stride(0) if res and B > 1 else 0)
        got = out.cpu()
        assert torch.all(got[:, :, 0] == 0) and torch.all(got[:, :, -1] == 0) and torch.all(got[..., 0] == 0) \
            and torch.all(got[..., -1] == 0), "border"
        err = (got[:, :, 1:-1, 1:-1] - want).abs().max().item() / max(1.0, want.abs().max().item())
        worst = max(worst, err)
        print(f"conv64 Ci={Ci} Co={Co} {H}x{W} B={B} k={k}: rel err {err:.2e}", flush=True)
    # K = 1 GEMM with f32 output and sigmoid (the classifier)
    x = torch.randn(512, 777, generator=g, dtype=torch.float64)
    w = torch.randn(360, 512, 1, generator=g, dtype=torch.float64) / 20
    b = torch.randn(360, generator=g, dtype=torch.float64)
    cv = ops.Conv64(w, b, DEV)
    got = cv(x.to(DEV), out_act=ops.ACT_SIGMOID, out_f32=True).cpu().double()
    want = torch.sigmoid(w[:, :, 0] @ x + b[:, None]).float().double()
    err = (got - want).abs().max().item()
    print(f"conv64 GEMM 360x512x777 sigmoid f32 out: max err {err:.2e} (0 = the rounding of the f64 result)")
    worst = max(worst, err)
    assert worst < 1e-12, worst


def headline(skip_oracle):
    import f0check
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    seed = 201
    sd = synthetic.rmvpe_state_dict(seed + 2)
    audio = synthetic.synthetic_audio(30.0, seed=1000)
    res = {}
    for prec in ("f64", "fp32sa"):
        rm = RMVPEAMD(sd, DEV, precision=prec)
        vc = VC(48000, Config(DEV), rmvpe=rm)
        xp, _ = vc.filt(torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)).to(DEV), vc.t_pad)
        for _ in range(2):
            rm.f0_device(xp)
        torch.cuda.synchronize()
        t = time.time()
        n = 10
        for _ in range(n):
            rm.f0_device(xp)
        torch.cuda.synchronize()
        dt = (time.time() - t) / n
        rm.check_error()
        print(f"RMVPE {prec}: {dt * 1e3:.2f} ms per 30 s clip", flush=True)
        res[prec] = f0check.device_salience(vc, audio)[0]
    if skip_oracle:
        return
    s64 = f0check.oracle_salience(sd, audio, torch.float64)
    m = f0check.margins(s64)
    for prec, s in res.items():
        nd = f0check.decision_noise(s, s64)
        fl = f0check.flips(s, s64)
        print(f"{prec}: salience err max {np.abs(s - s64).max():.3e}; decision noise max {nd.max():.3e} "
              f"rms {np.sqrt(np.mean(nd ** 2)):.3e}; flips {fl.tolist()} margins {m[fl].tolist()}; "
              f"at 326/721/918/977 {nd[[326, 721, 918, 977]]}", flush=True)


if __name__ == "__main__":
    conv_units()
    headline("--skip-oracle" in sys.argv)
