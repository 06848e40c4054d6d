"""CPU-baseline calibration (build container only: needs /root/reference).

Times the reference's own ``VC.pipeline`` (main/inference/convert.py:388-458, CPU, fp32, imported through
the golden-vector harness of tests/golden/make_golden.py) and the torch-CPU oracle (oracle/pipeline.py)
on the same synthetic clip with the same weights and thread count, and writes the ratio to
profiles/cpu_calibration.json.  bench.py's ``cpu_baseline`` (the oracle timed on the GPU box's host) reports
it beside its own number, so the box-side oracle time can be read as a reference-path time.

    python scripts/cpu_calibrate.py [seconds] [threads]
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    from rvc_amd import melbasis, synthetic
    from oracle import contentvec as ocv
    from oracle import pipeline as opl
    from oracle import rmvpe as orm
    from oracle import synth as osy
    import make_golden as mg
    out_path = os.path.join(REPO, "profiles", "cpu_calibration.json")
    mg.setup_harness()
    torch.set_num_threads(threads)
    seed, sr = 1234, 48000
    ck = synthetic.make_synth_ckpt(sr, "v2", seed=seed)
    audio = synthetic.synthetic_audio(seconds, seed=1000)
    # reference: VC.pipeline with its own loaders (the per-call rmvpe.pt reload timed separately)
    import main.inference.convert as conv
    from main.library.architectures import fairseq
    from main.library.predictors.RMVPE import RMVPE
    net_g = mg.build_ref_synth(ck)
    cpath = os.path.join("assets", "models", "embedders", "contentvec_synth.pt")
    torch.save(synthetic.make_contentvec_ckpt(seed + 1), cpath)
    hub = fairseq.load_model(cpath)[0][0].float().eval()
    rpath = os.path.join("assets", "models", "predictors", "rmvpe.pt")
    torch.save(synthetic.rmvpe_state_dict(seed + 2), rpath)
    vc = conv.VC(sr, conv.config)
    t0 = time.perf_counter()
    RMVPE(rpath, is_half=False, device="cpu")
    reload_s = time.perf_counter() - t0
    kw = dict(model=hub, net_g=net_g, sid=0, pitch=0, f0_method="rmvpe", file_index="", index_rate=0.0,
              pitch_guidance=1, filter_radius=3, volume_envelope=1, version="v2", protect=0.33, hop_length=64,
              f0_autotune=False, f0_autotune_strength=1, suffix=".pth", embed_suffix=".pt", f0_file=None,
              f0_onnx=False, pbar=mg.Pbar())
    torch.manual_seed(0)
    vc.pipeline(audio=audio[:16000].copy(), **kw)  # warm (allocator, thread pool)
    t0 = time.perf_counter()
    ref_out = vc.pipeline(audio=audio.copy(), **kw)
    ref_s = time.perf_counter() - t0 - reload_s
    # oracle: same clip, same weights, same threads
    Ws, Wc = osy.load_weights(ck["weight"]), ocv.load_weights(synthetic.make_contentvec_ckpt(seed + 1))
    Wr = orm.load_weights(synthetic.rmvpe_state_dict(seed + 2))
    mb = torch.from_numpy(melbasis.mel_filterbank())
    g = torch.Generator().manual_seed(0)
    noise = lambda s, k, sh: torch.randn(*sh, generator=g)  # noqa: E731
    opl.pipeline(Wc, Ws, Wr, mb, ck["config"], 0, audio[:16000], 0.0, "v2", 0.33, noise)
    t0 = time.perf_counter()
    orc_out = opl.pipeline(Wc, Ws, Wr, mb, ck["config"], 0, audio, 0.0, "v2", 0.33, noise)
    orc_s = time.perf_counter() - t0
    res = {"seconds": seconds, "threads": threads, "host_cpus": os.cpu_count(), "reference_s": round(ref_s, 3),
           "reference_rmvpe_reload_s": round(reload_s, 3), "oracle_s": round(orc_s, 3),
           "oracle_over_reference_time": round(orc_s / ref_s, 4), "output_samples": [len(ref_out), len(orc_out)],
           "reference_xrt": round(len(ref_out) / sr / ref_s, 4), "oracle_xrt": round(len(orc_out) / sr / orc_s, 4),
           "note": "reference VC.pipeline timed without its per-call rmvpe.pt reload (reported separately); "
                   "both on the same synthetic 48k v2 weights and clip, fp32, torch CPU"}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    assert np.isfinite(ref_out).all() and len(ref_out) == len(orc_out)


if __name__ == "__main__":
    main()
