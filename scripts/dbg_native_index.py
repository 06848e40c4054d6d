"""Debug: rvc_vc_convert with an IVF index vs VC.pipeline_device (tests/test_gpu_native.py) across variants."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
sys.path.insert(0, REPO)

from rvc_amd import melbasis, synthetic  # noqa: E402
from rvc_amd.contentvec import ContentVecAMD  # noqa: E402
from rvc_amd.faiss_index import IVFFlatIndex  # noqa: E402
from rvc_amd.native import NativeVC  # noqa: E402
from rvc_amd.pipeline import VC, Config  # noqa: E402
from rvc_amd.retrieval import IVFFlatDevice  # noqa: E402
from rvc_amd.rmvpe import RMVPEAMD  # noqa: E402
from rvc_amd.synth import SynthesizerAMD, fold_weight_norm  # noqa: E402

DEV = "cuda"


def rms(a, b):
    return float((a.double() - b.double()).pow(2).mean().sqrt())


def main():
    hub_ck, rm_sd, cpt = synthetic.make_contentvec_ckpt(71), synthetic.rmvpe_state_dict(72), \
        synthetic.make_synth_ckpt(48000, "v2", seed=73)
    hub, net_g = ContentVecAMD(hub_ck, DEV), SynthesizerAMD(cpt, DEV)
    vc = VC(48000, Config(DEV), rmvpe=RMVPEAMD(rm_sd, DEV))
    feats = hub.features_cf(torch.from_numpy(synthetic.synthetic_audio(8.0, seed=74)).to(DEV)).t().cpu().numpy()
    hw = dict(hub_ck["model"])
    p = "encoder.pos_conv.0.weight"
    hw[p] = torch._weight_norm(hw.pop(p + "_v").float(), hw.pop(p + "_g").float(), 2)
    nat = NativeVC(hub_ck, rm_sd, cpt, DEV, synth_weights=fold_weight_norm(cpt["weight"]), hub_weights=hw,
                   window=torch.hann_window(1024), mel_basis=melbasis.mel_filterbank(16000, 1024, 128, 30, 8000))
    audio = torch.from_numpy(synthetic.synthetic_audio(5.1, seed=75)).float().to(DEV)
    plain_py = vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33)
    plain_nat = nat.convert(audio, 0, 0.0, 0.33, "v2", seed=0)
    torch.cuda.synchronize()
    print("plain: native vs python", rms(plain_nat, plain_py), torch.equal(plain_nat, plain_py), flush=True)
    for nprobe in (1, 3):
        rng = np.random.default_rng(2)
        idx = IVFFlatIndex.build(feats[rng.choice(len(feats), 24, replace=False)], feats, nprobe=nprobe)
        nat.load_index(idx)
        dix = IVFFlatDevice(idx, DEV)
        for rate in (0.66, 1.0):
            ref = vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33, dix, rate)
            got = nat.convert(audio, 0, 0.0, 0.33, "v2", seed=0, index_rate=rate)
            got2 = nat.convert(audio, 0, 0.0, 0.33, "v2", seed=0, index_rate=rate)
            ref2 = vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33, dix, rate)
            torch.cuda.synchronize()
            print(f"nprobe {nprobe} rate {rate}: native vs python {rms(got, ref):.3e} equal {torch.equal(got, ref)}; "
                  f"native repeat {torch.equal(got, got2)}; python repeat {torch.equal(ref, ref2)}; "
                  f"vs plain: nat {rms(got, plain_nat):.3e} py {rms(ref, plain_py):.3e}", flush=True)
    # the retrieval alone on python features, both arithmetics
    fe = hub.features_cf(torch.nn.functional.pad(audio[None, None], (16000, 16000), mode="reflect")[0, 0])
    D1, I1 = dix.search_cf(fe)
    D2, I2 = dix.search_cf(fe, arithmetic="exact")
    print("faiss vs exact neighbour lists equal:", bool((I1 == I2).all()), float((I1 != I2).float().mean()))


if __name__ == "__main__":
    main()
