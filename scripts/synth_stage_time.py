"""Per-stage device time of one 30 s clip through SynthesizerAMD (48k v2, synthetic weights): the TextEncoder, the
flow^-1 and the generator, each alone on an idle GPU (HIP events, median of --reps), under the module switches named on
the command line (``synth.TE_AMAX=0`` style, toggled in-process between variants) -- the stage-level view of an
end-to-end A/B, without the clip stream's concurrency.

    python scripts/synth_stage_time.py [--frames 3000] [--reps 10] base TE_AMAX=0 ATTN_F16=0 ...
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=3000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("variants", nargs="*", default=["base"])
    a = ap.parse_args()
    from rvc_amd import synth, synthetic
    ck = synthetic.make_synth_ckpt(48000, "v2", seed=7)
    m = synth.SynthesizerAMD(ck, "cuda")
    T = a.frames
    g = torch.Generator().manual_seed(0)
    phone = torch.randn(1, 768, T, generator=g).cuda()
    pitch = torch.randint(1, 255, (1, T), generator=g).cuda()
    nsff0 = (torch.rand(1, T, generator=g) * 300 + 80).cuda()
    gc = m.speaker_cond(0)
    defaults = {k: getattr(synth, k) for k in ("TE_AMAX", "FLOW_AMAX", "ATTN_F16", "FUSED_NOISE", "AMAX", "AMAX_UPS")}
    out = {}

    def timed(fn):
        ts = []
        for _ in range(a.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts = sorted(ts[2:])
        return ts[len(ts) // 2]

    for v in a.variants:
        for k, val in defaults.items():
            setattr(synth, k, val)
        if v != "base":
            for kv in v.split(","):
                k, val = kv.split("=")
                setattr(synth, k, val != "0")
        stats = m.text_encoder(phone, pitch, T, 1)
        z_p = torch.randn(1, m.inter, T, device="cuda")
        z = m.flow_reverse(z_p, gc, T, 1)
        noise = torch.randn(1, T * m.upp, device="cuda")
        r = {
            "text_encoder_ms": timed(lambda: m.text_encoder(phone, pitch, T, 1)),
            "flow_ms": timed(lambda: m.flow_reverse(z_p, gc, T, 1)),
            "generator_ms": timed(lambda: m.generator(z, nsff0, gc[4 * 6 * m.hidden:], T, noise, 1)),
        }
        del stats
        out[v] = r
        print(f"{v:28s} " + "  ".join(f"{k} {x:7.3f}" for k, x in r.items()), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
