"""Where the clip stream's output departs from the per-call pipeline (tests/test_gpu_batch.py's stream tests): the
synthetic models of that module, N x 30 s clips through VC.pipeline_device_stream and through pipeline_device clip by
clip, repeated; per clip the number of differing samples, the first / last differing index and the max |difference|,
the device error flag after each pass, and the f0 of both forms (VC.f0_device on the filtered input) compared.

    python scripts/stream_diff.py [--clips 2] [--seconds 30] [--reps 3]
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--empty-cache", action="store_true", help="release the caching allocator's blocks after the "
                    "per-call references")
    a = ap.parse_args()
    from rvc_amd import synthetic
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
    vc.seed = 21
    first = [o.clone() for o in vc.pipeline_device_stream(hub, net_g, 0, xs, 0, "v2", 0.33)]  # a stream before anything
    torch.cuda.synchronize()
    refs = []
    for k, x in enumerate(xs):
        vc.seed = 21 + k
        refs.append(vc.pipeline_device(hub, net_g, 0, x, 0, "v2", 0.33).clone())
    torch.cuda.synchronize()
    if a.empty_cache:
        torch.cuda.empty_cache()
    vc.seed = 0
    for rep in range(a.reps):
        vc.seed = 21
        outs = vc.pipeline_device_stream(hub, net_g, 0, xs, 0, "v2", 0.33)
        torch.cuda.synchronize()
        err = None
        try:
            vc.check_errors()
        except Exception as e:  # noqa: BLE001
            err = str(e)[:80]
        vc.seed = 0
        for k in range(a.clips):
            d = (outs[k] - refs[k]).abs()
            nz = torch.nonzero(d).flatten()
            if nz.numel():
                print(f"rep {rep} clip {k}: {nz.numel()} of {d.numel()} samples differ, first {int(nz[0])} last "
                      f"{int(nz[-1])}, max {d.max().item():.3e}; error flag: {err}", flush=True)
            else:
                print(f"rep {rep} clip {k}: identical; error flag: {err}", flush=True)
    # per-call repeatability, the first stream against it, and both against the unfused-noise synthesizer
    from rvc_amd import synth
    for k, x in enumerate(xs):
        vc.seed = 21 + k
        o = vc.pipeline_device(hub, net_g, 0, x, 0, "v2", 0.33)
        torch.cuda.synchronize()
        print(f"per-call again clip {k}: max diff {(o - refs[k]).abs().max().item():.3e}; the process's first stream: "
              f"{(first[k] - refs[k]).abs().max().item():.3e}", flush=True)
    fused = synth.FUSED_NOISE
    synth.FUSED_NOISE = not fused
    for k, x in enumerate(xs):
        vc.seed = 21 + k
        o = vc.pipeline_device(hub, net_g, 0, x, 0, "v2", 0.33)
        torch.cuda.synchronize()
        print(f"clip {k} with FUSED_NOISE={not fused}: vs per-call {(o - refs[k]).abs().max().item():.3e}, vs first "
              f"stream {(o - first[k]).abs().max().item():.3e}, vs last stream {(o - outs[k]).abs().max().item():.3e}",
              flush=True)
    synth.FUSED_NOISE = fused
    vc.seed = 0


if __name__ == "__main__":
    main()
