"""One 30 s clip (48k v2, RMVPE) through the model-level ABI (rvc_vc_convert, NativeVC) vs the Python host
(VC.pipeline_device) on the same GPU: ms per clip and xRT; outputs compared bit for bit."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rvc-maker_amd"))
import torch

from rvc_amd import melbasis, synthetic
from rvc_amd.contentvec import ContentVecAMD
from rvc_amd.native import NativeVC
from rvc_amd.pipeline import VC, Config
from rvc_amd.rmvpe import RMVPEAMD
from rvc_amd.synth import SynthesizerAMD, fold_weight_norm

dev = "cuda"
hub_ck, rm_sd, cpt = synthetic.make_contentvec_ckpt(1), synthetic.rmvpe_state_dict(2), synthetic.make_synth_ckpt(48000, "v2", 3)
hub, net_g = ContentVecAMD(hub_ck, dev), SynthesizerAMD(cpt, dev)
vc = VC(48000, Config(dev), rmvpe=RMVPEAMD(rm_sd, dev))
hw = dict(hub_ck["model"])
p = "encoder.pos_conv.0.weight"
hw[p] = torch._weight_norm(hw.pop(p + "_v").float(), hw.pop(p + "_g").float(), 2)
nat = NativeVC(hub_ck, rm_sd, cpt, dev, synth_weights=fold_weight_norm(cpt["weight"]), hub_weights=hw,
               window=torch.hann_window(1024), mel_basis=melbasis.mel_filterbank(16000, 1024, 128, 30, 8000))
audio = torch.from_numpy(synthetic.synthetic_audio(30.0, seed=4)).float().to(dev)


def timed(fn, n=6):
    for _ in range(2):
        out = fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        out = fn()
    torch.cuda.synchronize()
    return out, (time.perf_counter() - t) / n * 1e3


a, ta = timed(lambda: vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33))
b, tb = timed(lambda: nat.convert(audio, 0, 0.0, 0.33, "v2", seed=0))
vc.check_errors()
sec = a.numel() / 48000
print(f"python host VC.pipeline_device: {ta:.2f} ms/clip, {sec / ta * 1e3:.0f} xRT")
print(f"C ABI rvc_vc_convert:           {tb:.2f} ms/clip, {sec / tb * 1e3:.0f} xRT")
print("bit-identical:", bool(torch.equal(a, b)))
