"""Per-shape timing of the conv engine inside one bench step (HIP events around each launch).

    python scripts/conv_profile.py [--seconds 30] [--top 30]

Groups every ops.conv1d launch of one VC.pipeline step by its shape and prints calls, total ms,
average us, algorithmic GFLOP and TFLOP/s per shape -- the table that says which conv shapes the
roofline fraction is lost on.
"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--top", type=int, default=60)
    args = ap.parse_args()
    from rvc_amd import ops, synthetic
    dev = "cuda:0"
    vc, hub, net_g = bench.build_models(dev)
    audio = torch.from_numpy(synthetic.synthetic_audio(args.seconds, seed=1000)).to(dev)
    vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33)
    torch.cuda.synchronize()
    orig = ops.conv1d
    rec = []

    def wrapped(x, w, Ci, Co, K, **kw):
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        out = orig(x, w, Ci, Co, K, **kw)
        e1.record(s)
        B = kw.get("B") or (1 if x.dim() == 2 else x.shape[0])
        Lin = kw.get("Lin") or x.shape[-1]
        key = (B, Ci, Co, K, kw.get("stride", 1), kw.get("dil", 1), kw.get("groups", 1), Lin,
               kw.get("nphase", 1), "2d" if kw.get("wrap") else "", "res" if kw.get("res") is not None else "",
               "acc" if kw.get("accumulate") else "", "x6" if ops.LAST_CONV_ENGINE == 1 else "f32")
        rec.append((key, e0, e1, ops.LAST_CONV_FLOPS))
        return out

    orig_rb = ops.resblock_pair

    def wrapped_rb(x, y, c1, c2, dil, slope, accumulate=False):
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        out = orig_rb(x, y, c1, c2, dil, slope, accumulate=accumulate)
        e1.record(s)
        C, L = x.shape
        key = (1, C, C, c1.K, 1, dil, 1, L, 1, "", "pair", "acc" if accumulate else "", "rb")
        rec.append((key, e0, e1, 2 * 2.0 * C * C * c1.K * L))
        return out

    ops.conv1d = wrapped
    ops.resblock_pair = wrapped_rb
    vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33)
    torch.cuda.synchronize()
    ops.conv1d = orig
    ops.resblock_pair = orig_rb
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for key, e0, e1, fl in rec:
        a = agg[key]
        a[0] += 1
        a[1] += e0.elapsed_time(e1)
        a[2] += fl
    tot_ms = sum(a[1] for a in agg.values())
    tot_fl = sum(a[2] for a in agg.values())
    print(f"{len(rec)} launches, {tot_ms:.2f} ms, {tot_fl / 1e9:.1f} GFLOP, {tot_fl / tot_ms / 1e9:.1f} TFLOP/s")
    print(f"{'B':>3} {'Ci':>5} {'Co':>5} {'K':>3} {'s':>2} {'d':>2} {'g':>3} {'Lin':>8} {'ph':>2} {'flags':>14} "
          f"{'calls':>5} {'ms':>8} {'us/call':>8} {'GFLOP':>8} {'TF/s':>6} {'%time':>6}")
    for key, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: args.top]:
        B, Ci, Co, K, s, d, g, Lin, ph, f2d, fres, facc, eng = key
        flags = ",".join(x for x in (eng, f2d, fres, facc) if x)
        print(f"{B:>3} {Ci:>5} {Co:>5} {K:>3} {s:>2} {d:>2} {g:>3} {Lin:>8} {ph:>2} {flags:>14} {n:>5} {ms:>8.3f} "
              f"{ms / n * 1e3:>8.1f} {fl / 1e9:>8.2f} {fl / ms / 1e9:>6.1f} {100 * ms / tot_ms:>6.1f}")


if __name__ == "__main__":
    main()
