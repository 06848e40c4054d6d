"""Determinism of the generator with the fused noise source pass (synth.FUSED_NOISE) on a dirty allocator: the 48k v2
generator on one 30 s clip, run repeatedly after the caching allocator's free blocks were filled with garbage (NaN,
1e30, random), fused and unfused; prints the max |difference| of every run against the first unfused run.

    python scripts/fused_noise_check.py [--frames 3000] [--reps 3]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

import torch  # noqa: E402


def dirty(value, gib=8):
    """Fill ~gib GiB of fresh allocations with value and free them (they stay in the caching allocator)."""
    bufs = []
    for _ in range(gib * 4):
        t = torch.empty(64 << 20, device="cuda")
        if value == "rand":
            t.uniform_(-1e3, 1e3)
        else:
            t.fill_(float(value))
        bufs.append(t)
    torch.cuda.synchronize()
    del bufs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=3000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from rvc_amd import synth, synthetic
    ck = synthetic.make_synth_ckpt(48000, "v2", seed=7)
    m = synth.SynthesizerAMD(ck, "cuda")
    T = a.frames
    g = torch.Generator().manual_seed(0)
    z = torch.randn(1, m.inter, T, generator=g).cuda()
    nsff0 = (torch.rand(1, T, generator=g) * 300 + 80).cuda()
    gc = m.speaker_cond(0)
    noise = torch.randn(1, T * m.upp, generator=g).cuda()
    gdec = gc[4 * 6 * m.hidden:]
    outs = {}
    for fused in (False, True):
        synth.FUSED_NOISE = fused
        for r in range(a.reps):
            dirty(("nan", "1e30", "rand")[r % 3])
            o = m.generator(z, nsff0, gdec, T, noise, 1).clone()
            torch.cuda.synchronize()
            outs[(fused, r)] = o
    ref = outs[(False, 0)]
    for k, o in outs.items():
        d = (o - ref).abs().max().item()
        print(f"fused={k[0]} rep={k[1]}: max |o - unfused rep 0| = {d:.3e}  finite={bool(torch.isfinite(o).all())}",
              flush=True)


if __name__ == "__main__":
    main()
