"""Which stage of the clip stream's synthesizer departs from the per-call pipeline (the fused noise pass's exposure,
scripts/stream_diff.py): the stream and the per-call form of the same clips with the synthesizer's stage inputs and
outputs stashed as stream-ordered clones -- feats / coarse / pitchf on entry, z and g after the prior and flow^-1, y
after each upsampling stage (ups + noise), the waveform -- and compared per clip.

    python scripts/stream_stage_diff.py [--clips 2] [--seconds 30]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=30.0)
    a = ap.parse_args()
    from rvc_amd import synthetic, ops
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    dev = "cuda"
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(71), dev)
    rm = RMVPEAMD(synthetic.rmvpe_state_dict(72), dev)
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(48000, "v2", seed=73), dev)
    vc = VC(48000, Config(dev), rmvpe=rm)
    xs = [torch.from_numpy(synthetic.synthetic_audio(a.seconds, seed=900 + i)).to(dev) for i in range(a.clips)]

    log = []  # (name, clone) in issue order of one pass

    def stash(name, t):
        log.append((name, t.detach().clone()))

    prior0, gen0 = vc.prior_device, vc.generate_device

    def prior(model, net_g, sid, a0, pitch, pitchf, version, protect, seg, feats=None, *args, **kw):
        stash("a0", a0)
        stash("pitch", pitch)
        stash("pitchf", pitchf)
        if feats is not None:
            stash("feats", feats)
        prep = prior0(model, net_g, sid, a0, pitch, pitchf, version, protect, seg, feats, *args, **kw)
        stash("z", prep["z"])
        stash("gc", prep["gc"])
        return prep

    def gen(net_g, prep, seg, seed):
        o = gen0(net_g, prep, seg, seed)
        stash("wave", o)
        return o

    vc.prior_device, vc.generate_device = prior, gen
    # the upsampling stages' outputs: wrap every ups conv (its call returns y before the noise term when unfused, the
    # final y when fused) and every noise conv
    for i, up in enumerate(net_g.ups):
        def wrap(conv, name):
            f0 = conv.__call__

            class W:
                def __getattr__(self, k):
                    return getattr(conv, k)

                def __call__(self, *args, **kw):
                    stash(name + ".x", args[0])
                    if kw.get("src") is not None:
                        stash(name + ".har", kw["src"][1])
                    y = f0(*args, **kw)
                    stash(name, y)
                    return y
            return W()
        net_g.ups[i] = wrap(up, f"ups{i}")

    def run_stream():
        log.clear()
        vc.seed = 21
        outs = vc.pipeline_device_stream(hub, net_g, 0, xs, 0, "v2", 0.33)
        torch.cuda.synchronize()
        vc.seed = 0
        return list(log), outs

    def run_percall():
        log.clear()
        for k, x in enumerate(xs):
            vc.seed = 21 + k
            vc.pipeline_device(hub, net_g, 0, x, 0, "v2", 0.33)
        torch.cuda.synchronize()
        vc.seed = 0
        return list(log)

    first, _ = run_stream()
    ref = run_percall()
    later, _ = run_stream()
    n = len(ref) // a.clips

    def cmp(tag, run):
        for k in range(a.clips):
            row = []
            for (name, r), (name2, s) in zip(ref[k * n:(k + 1) * n], run[k * n:(k + 1) * n]):
                assert name == name2, (name, name2)
                if r.shape != s.shape:
                    row.append(f"{name}:shape")
                    continue
                d = (r.double() - s.double()).abs().max().item() if r.numel() else 0.0
                row.append(f"{name}:{d:.1e}" if d else f"{name}:0")
            print(f"{tag} clip {k}: " + " ".join(row), flush=True)

    cmp("first stream", first)
    cmp("stream after per-call", later)
    # the first differing stage output: where its differences lie (channels x positions), and whether they equal the
    # source conv's term (the pass missing or applied twice somewhere) -- the noise conv run alone on the stashed har
    for tag, run in (("first stream", first), ("stream after per-call", later)):
        for k in range(a.clips):
            for (name, r), (_, s) in zip(ref[k * n:(k + 1) * n], run[k * n:(k + 1) * n]):
                if not name.startswith("ups") or "." in name or r.shape != s.shape or torch.equal(r, s):
                    continue
                d = (s - r).reshape(r.shape[-2], r.shape[-1]) if r.dim() >= 2 else (s - r).reshape(1, -1)
                rows = torch.nonzero(d.abs().amax(1)).flatten()
                cols = torch.nonzero(d.abs().amax(0)).flatten()
                print(f"{tag} clip {k} {name}: {int((d != 0).sum())} of {d.numel()} differ; channels {rows.numel()} "
                      f"({int(rows[0])}..{int(rows[-1])}), positions {cols.numel()} ({int(cols[0])}..{int(cols[-1])})",
                      flush=True)
                i = int(name[3:])
                nc, st, pad = net_g.noise[i]
                har = dict(ref[k * n:(k + 1) * n]).get(name + ".har")
                if har is None:
                    break
                B = 1
                term = nc(har.view(B, 1, -1), Lout=d.shape[-1], stride=st, pad=pad).reshape(d.shape)
                torch.cuda.synchronize()
                for sgn, lab in ((1.0, "missing"), (-1.0, "doubled")):
                    m = (d != 0)
                    e = (d + sgn * term)[m].abs().max().item() if m.any() else 0.0
                    print(f"   if the source term were {lab} at the differing points: residual {e:.2e} "
                          f"(|term| there {term[m].abs().max().item():.2e}, |d| {d.abs().max().item():.2e})", flush=True)
                cb = torch.nonzero((d != 0).any(0)).flatten() // 256
                print(f"   256-position blocks touched: {sorted(set(cb.tolist()))[:40]}", flush=True)
                break
    _ = ops


if __name__ == "__main__":
    main()
