"""One long utterance over ranks (rvc_amd.longform) on the device: the RMVPE U-Net run on halo'd time tiles
against the whole-image pass (the halo covers the receptive field), and pipeline_sharded over 2 ranks
(gloo, both on this GPU) against the single-rank VC.pipeline_device of the same 50 s input."""
import os
import socket

import numpy as np
import pytest
import torch

from rvc_amd import longform, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _models(dev):
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(81), dev)
    rm = RMVPEAMD(synthetic.rmvpe_state_dict(82), dev)
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(48000, "v2", seed=83), dev)
    return hub, net_g, VC(48000, Config(dev), rmvpe=rm)


def test_unet_tiles_match_whole_image():
    _, _, vc = _models(DEV)
    rm = vc.rmvpe
    x = torch.from_numpy(synthetic.synthetic_audio(40.0, seed=61)).to(DEV)
    xp, _ = vc.filt(x, vc.t_pad)
    mel = rm.mel_spectrogram(xp)
    img, Tp = rm.mel_image(mel)
    whole = rm.unet_seq(img, Tp)
    for a, b, r0, r1 in longform.tile_plan(Tp, 3):
        tile = torch.zeros(1, r1 - r0 + 2, img.shape[-1], device=DEV, dtype=img.dtype)
        tile[0, 1:-1] = img[0, 1 + r0: 1 + r1]
        seq = rm.unet_seq(tile, r1 - r0)[:, a - r0: b - r0]
        err = (seq - whole[:, a:b]).abs().max().item()
        assert err <= 1e-4 * max(1.0, whole.abs().max().item()), (a, b, err)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, secs, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hub, net_g, vc = _models(DEV)
        audio = synthetic.synthetic_audio(secs, seed=62)
        vc.seed = 9
        out = longform.pipeline_sharded(vc, hub, net_g, 0, audio, 0, "v2", 0.33, dist)
        torch.cuda.synchronize()
        vc.check_errors()
        if rank == 0:
            vc.seed = 9
            ref = vc.pipeline_device(hub, net_g, 0, audio, 0, "v2", 0.33)
            q.put((out.cpu().numpy(), ref.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_pipeline_sharded_two_ranks_matches_single():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 50.0, q)) for r in range(2)]
    for p in procs:
        p.start()
    out, ref = q.get(timeout=350)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out.shape == ref.shape
    rel = np.sqrt(np.mean((out.astype(np.float64) - ref) ** 2) / np.mean(ref.astype(np.float64) ** 2))
    assert rel <= 1e-4, rel
