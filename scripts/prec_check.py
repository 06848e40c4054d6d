"""Waveform error of VC.pipeline at each conv-engine precision vs the reference golden (48k v2)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
from rvc_amd import ops, synthetic  # noqa: E402
from rvc_amd.contentvec import ContentVecAMD  # noqa: E402
from rvc_amd.pipeline import VC, Config  # noqa: E402
from rvc_amd.rmvpe import RMVPEAMD  # noqa: E402
from rvc_amd.synth import SynthesizerAMD  # noqa: E402

DEV = "cuda"
for name in sys.argv[1:] or ["pipeline_48k_v2"]:
    g = dict(np.load(os.path.join(REPO, "tests", "golden", name + ".npz")))
    sr, version, seed = int(g["sr"]), str(g["version"]), int(g["seed"])
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, version, seed=seed), DEV)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(seed + 1), DEV)
    vc = VC(sr, Config(DEV), rmvpe=RMVPEAMD(synthetic.rmvpe_state_dict(seed + 2), DEV))
    vc.noise_fn = lambda s, k, sh: torch.from_numpy(g[f"{'z' if k == 'z' else 'sine'}_noise_{s}"]).to(DEV)
    ref = g["out"].astype(np.float64)
    for prec in ("fp32", "fp32x6", "f16x3", "bf16x3", "bf16"):
        with ops.precision(prec):
            out = vc.pipeline_device(hub, net_g, 0, g["audio"], float(g["pitch"]), version, float(g["protect"]))
        o = out.cpu().numpy().astype(np.float64)
        err = float(np.sqrt(np.mean((o - ref) ** 2)))
        print(f"{name} {prec:7s} rms err {err:.3e}  rel {err / np.sqrt(np.mean(ref ** 2)):.3e}", flush=True)
