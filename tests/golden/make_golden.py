"""Generate golden vectors by running the REFERENCE (RVC-MAKER) itself on CPU.

Run in the survey container only (``/root/reference`` must exist):

    python tests/golden/make_golden.py

The reference is imported from ``/root/reference`` through a scratch working
directory (``main`` -> the reference's ``main``, ``assets/languages`` linked,
``assets/logs`` and ``assets/models`` writable) with stub modules for the
packages this image lacks: ``librosa`` (only ``filters.mel`` is
used on the path; the stub returns ``rvc_amd.melbasis`` -- parity vs librosa
itself is therefore unpinned), ``omegaconf``, ``faiss``, ``onnxruntime``,
``soundfile``, ``pydub``.  Weights are the seeded synthetic checkpoints of
``rvc_amd.synthetic`` written in the reference's own checkpoint layouts and
loaded through the reference's loaders.  Every RNG draw the reference makes
(``torch.randn_like`` / ``torch.rand``) is recorded and stored, so the HIP path
can be run with identical noise.

Outputs (data only -- inputs and expected outputs) go to ``tests/golden/*.npz``.
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
from rvc_amd import melbasis, synthetic  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")


def _stub_modules():
    lib = types.ModuleType("librosa")
    filt = types.ModuleType("librosa.filters")

    def mel(sr, n_fft, n_mels, fmin, fmax, htk=False, **kw):
        assert htk
        return melbasis.mel_filterbank(sr, n_fft, n_mels, fmin, fmax)

    filt.mel = mel
    lib.filters = filt
    # librosa.sequence.viterbi (CREPE's decode): the oracle's restatement of librosa >= 0.10 --
    # the CREPE golden therefore pins the network/preprocessing/postprocessing around it, not it
    seq = types.ModuleType("librosa.sequence")
    sys.path.insert(0, REPO)
    from oracle.crepe import viterbi_librosa
    seq.viterbi = viterbi_librosa
    lib.sequence = seq
    # librosa.feature.rms (change_rms, convert.py:150-152): the oracle's restatement -- unpinned vs librosa
    feat = types.ModuleType("librosa.feature")
    from oracle.pipeline import rms_librosa

    def rms(y=None, frame_length=2048, hop_length=512, **kw):
        return rms_librosa(y, frame_length, hop_length)

    feat.rms = rms
    lib.feature = feat
    sys.modules["librosa.feature"] = feat
    sys.modules["librosa"] = lib
    sys.modules["librosa.filters"] = filt
    sys.modules["librosa.sequence"] = seq
    om = types.ModuleType("omegaconf")
    om.DictConfig = dict

    class _Ctx:
        def __init__(self, x):
            self.x = x

        def __enter__(self):
            return self.x

        def __exit__(self, *a):
            return False

    om.open_dict = _Ctx
    sys.modules["omegaconf"] = om
    for name in ("faiss", "soundfile", "pydub"):
        m = types.ModuleType(name)
        sys.modules[name] = m
    sys.modules["pydub"].AudioSegment = object
    ort = types.ModuleType("onnxruntime")
    ort.get_available_providers = lambda: ["CPUExecutionProvider"]
    sys.modules["onnxruntime"] = ort


class NoiseRecorder:
    """Wraps torch.randn_like / torch.rand to record every draw in order."""

    def __init__(self):
        self.draws = []
        self._rl, self._r = torch.randn_like, torch.rand

    def __enter__(self):
        def rl(*a, **k):
            out = self._rl(*a, **k)
            self.draws.append(("randn_like", out.detach().clone()))
            return out

        def r(*a, **k):
            out = self._r(*a, **k)
            self.draws.append(("rand", out.detach().clone()))
            return out

        torch.randn_like, torch.rand = rl, r
        return self

    def __exit__(self, *a):
        torch.randn_like, torch.rand = self._rl, self._r


class Pbar:
    def update(self, n):
        pass


def setup_harness():
    work = tempfile.mkdtemp(prefix="rvc_golden_")
    os.symlink(os.path.join(REF, "main"), os.path.join(work, "main"))
    os.makedirs(os.path.join(work, "assets", "logs"))
    os.makedirs(os.path.join(work, "assets", "models", "predictors"))
    os.makedirs(os.path.join(work, "assets", "models", "embedders"))
    os.symlink(os.path.join(REF, "assets", "languages"), os.path.join(work, "assets", "languages"))
    os.chdir(work)
    sys.path.insert(0, work)
    sys.dont_write_bytecode = True
    _stub_modules()
    return work


def build_ref_synth(ckpt):
    from main.library.algorithm.synthesizers import Synthesizer
    version = ckpt["version"]
    net_g = Synthesizer(*ckpt["config"], use_f0=1, text_enc_hidden_dim=768 if version == "v2" else 256,
                        vocoder="Default", checkpointing=False)
    del net_g.enc_q
    missing, unexpected = net_g.load_state_dict(ckpt["weight"], strict=False)
    assert not missing and not unexpected, (missing, unexpected)
    return net_g.eval().float()


def gen_synth(name, sr, version, T, seed):
    """Synthesizer.infer on seeded phone / pitch / pitchf (synthesizers.py:446)."""
    ckpt = synthetic.make_synth_ckpt(sr, version, seed=seed)
    net_g = build_ref_synth(ckpt)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    emb = 768 if version == "v2" else 256
    phone = rng.standard_normal((1, T, emb)).astype(np.float32)
    pitch = rng.integers(1, 256, size=(1, T)).astype(np.int64)
    pitchf = rng.uniform(60, 500, size=(1, T)).astype(np.float32)
    pitchf[:, rng.random(T) < 0.25] = 0.0  # unvoiced frames
    sid = np.array([3], dtype=np.int64)
    torch.manual_seed(seed + 2)
    with torch.no_grad(), NoiseRecorder() as rec:
        o, x_mask, (z, z_p, m_p, logs_p) = net_g.infer(torch.from_numpy(phone), torch.tensor([T]),
                                                       torch.from_numpy(pitch), torch.from_numpy(pitchf),
                                                       torch.from_numpy(sid))
    kinds = [k for k, _ in rec.draws]
    assert kinds == ["randn_like", "rand", "randn_like"], kinds
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), sr=sr, version=version, seed=seed, T=T,
                        phone=phone, pitch=pitch, pitchf=pitchf, sid=sid,
                        z_noise=rec.draws[0][1].numpy(), sine_noise=rec.draws[2][1].numpy(),
                        o=o.numpy(), z=z.numpy(), z_p=z_p.numpy(), m_p=m_p.numpy(), logs_p=logs_p.numpy())
    print(name, "o rms", float(o.pow(2).mean().sqrt()))


def gen_contentvec(seconds, seed):
    from main.library.architectures import fairseq
    ck = synthetic.make_contentvec_ckpt(seed)
    path = os.path.join("assets", "models", "embedders", "contentvec_synth.pt")
    torch.save(ck, path)
    models, _, _ = fairseq.load_model(path)
    m = models[0].float().eval()
    audio = synthetic.synthetic_audio(seconds, seed=seed + 5)
    src = torch.from_numpy(audio).view(1, -1)
    with torch.no_grad():
        pm = torch.BoolTensor(src.shape).fill_(False)
        v2 = m.extract_features(source=src, padding_mask=pm, output_layer=12)[0]
        l9 = m.extract_features(source=src, padding_mask=pm, output_layer=9)[0]
        v1 = m.final_proj(l9)
        conv = m.extract_features(source=src, padding_mask=pm, ret_conv=True)[0]
    np.savez_compressed(os.path.join(OUT, "contentvec.npz"), seed=seed, audio=audio, feats_v2=v2.numpy(),
                        feats_v1=v1.numpy(), conv_feats=conv.numpy())
    print("contentvec", tuple(v2.shape), float(v2.std()))


def gen_rmvpe(seconds, seed):
    from main.library.predictors.RMVPE import RMVPE
    sd = synthetic.rmvpe_state_dict(seed)
    path = os.path.join("assets", "models", "predictors", "rmvpe.pt")
    torch.save(sd, path)
    r = RMVPE(path, is_half=False, device="cpu")
    audio = synthetic.synthetic_audio(seconds, seed=seed + 5).astype(np.float64)
    with torch.no_grad():
        mel = r.mel_extractor(torch.from_numpy(audio).float().unsqueeze(0), center=True)
        hidden = r.mel2hidden(mel)
    f0 = r.infer_from_audio(audio, thred=0.03)
    # decode on a peaked synthetic salience (exercises the 9-bin average and threshold)
    rng = np.random.Generator(np.random.PCG64(seed + 9))
    T = 257
    sal = (rng.random((T, 360)) * 0.02).astype(np.float32)
    c = rng.integers(0, 360, size=T)
    for i in range(T):
        for d in range(-4, 5):
            if 0 <= c[i] + d < 360:
                sal[i, c[i] + d] += np.float32(max(0.0, 0.9 - 0.2 * abs(d)) * rng.random())
    sal[::7] *= 0.5
    sal[::11] = (sal[::11] * 0.03).astype(np.float32)
    f0_kat = r.decode(sal, thred=0.03)
    np.savez_compressed(os.path.join(OUT, "rmvpe.npz"), seed=seed, audio=audio, mel=mel.numpy(),
                        hidden=hidden.numpy(), f0=f0, kat_salience=sal, kat_f0=f0_kat)
    print("rmvpe", tuple(mel.shape), tuple(hidden.shape), float(np.mean(f0)))


def write_hf_embedder(seed, name="contentvec_hf_synth"):
    """A transformers-layout ContentVec (config.json + model.safetensors, synthetic.make_hf_hubert) under
    assets/models/embedders/<name>, loaded through the reference's own load_embedders_model(.., "transformers")
    (main/library/utils.py:131-165: HubertModelWithFinalProj.from_pretrained)."""
    import json
    from safetensors.torch import save_file
    from main.library.utils import load_embedders_model
    cfg, sd = synthetic.make_hf_hubert(seed)
    d = os.path.join("assets", "models", "embedders", name)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(cfg, f)
    save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(d, "model.safetensors"))
    hub, _, suffix = load_embedders_model(name, "transformers")
    assert suffix == ".safetensors"
    return hub.float().eval()


def gen_contentvec_hf(seconds, seed):
    """The .safetensors embedder's outputs as VC.voice_conversion takes them (convert.py:342-345):
    model(feats)["last_hidden_state"] and final_proj of it (v1)."""
    hub = write_hf_embedder(seed)
    audio = synthetic.synthetic_audio(seconds, seed=seed + 5)
    with torch.no_grad():
        last = hub(torch.from_numpy(audio).view(1, -1))["last_hidden_state"]
        v1 = hub.final_proj(last[0]).unsqueeze(0)
    np.savez_compressed(os.path.join(OUT, "contentvec_hf.npz"), seed=seed, audio=audio, last_hidden_state=last.numpy(),
                        feats_v1=v1.numpy())
    print("contentvec_hf", tuple(last.shape), float(last.std()))


def gen_pipeline(name, sr, version, seconds, seed, pitch, protect, f0_autotune=False, f0_autotune_strength=1,
                 f0_lines=None, volume_envelope=1, embed=".pt"):
    import main.inference.convert as conv
    ck = synthetic.make_synth_ckpt(sr, version, seed=seed)
    net_g = build_ref_synth(ck)
    if embed == ".safetensors":
        hub = write_hf_embedder(seed + 1)
    else:
        from main.library.architectures import fairseq
        cpath = os.path.join("assets", "models", "embedders", "contentvec_synth.pt")
        torch.save(synthetic.make_contentvec_ckpt(seed + 1), cpath)
        hub = fairseq.load_model(cpath)[0][0].float().eval()
    torch.save(synthetic.rmvpe_state_dict(seed + 2), os.path.join("assets", "models", "predictors", "rmvpe.pt"))
    vc = conv.VC(sr, conv.config)
    audio = synthetic.synthetic_audio(seconds, seed=seed + 3)
    f0_file = None
    if f0_lines is not None:  # the reference reads f0_file.name (a gradio upload object)
        f0_file = types.SimpleNamespace(name=os.path.abspath(f"{name}_f0.txt"))
        with open(f0_file.name, "w") as f:
            f.write("\n".join(f0_lines) + "\n")
    torch.manual_seed(seed + 4)
    with NoiseRecorder() as rec:
        out = vc.pipeline(model=hub, net_g=net_g, sid=0, audio=audio.copy(), pitch=pitch, f0_method="rmvpe",
                          file_index="", index_rate=0.0, pitch_guidance=1, filter_radius=3,
                          volume_envelope=volume_envelope, version=version, protect=protect, hop_length=64,
                          f0_autotune=f0_autotune, f0_autotune_strength=f0_autotune_strength, suffix=".pth",
                          embed_suffix=embed, f0_file=f0_file, f0_onnx=False, pbar=Pbar())
    # transformers' HubertEncoder draws one scalar torch.rand([]) per layer for LayerDrop even in eval mode (its
    # value unused there): not a synthesizer draw
    rec.draws = [(k, t) for k, t in rec.draws if not (k == "rand" and t.dim() == 0)]
    kinds = [k for k, _ in rec.draws]
    assert len(kinds) % 3 == 0 and kinds[:3] == ["randn_like", "rand", "randn_like"], kinds
    nseg = len(kinds) // 3
    arrs = {}
    for s in range(nseg):
        arrs[f"z_noise_{s}"] = rec.draws[3 * s][1].numpy()
        arrs[f"sine_noise_{s}"] = rec.draws[3 * s + 2][1].numpy()
    opts = {}
    if f0_autotune:
        opts["f0_autotune_strength"] = f0_autotune_strength
    if f0_lines is not None:
        opts["f0_lines"] = np.array(f0_lines)
    if volume_envelope != 1:
        opts["volume_envelope"] = volume_envelope
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), sr=sr, version=version, seed=seed, pitch=pitch,
                        protect=protect, audio=audio, out=out, nseg=nseg, x_pad=conv.config.x_pad, embed=embed,
                        **arrs, **opts)
    print(name, "out", out.shape, float(np.sqrt(np.mean(out ** 2))), "segments", nseg)


def gen_convert(seed):
    """VoiceConverter.convert_audio (convert.py:479-523) -- the reference's own method, run on an instance
    built around the seeded synthetic models (its __init__ would load checkpoints from disk): load_audio
    returns the input array, sf.write captures the output.  Two speech bursts above 0.95 peak separated by
    digital silence, so the 0.95 peak limit, cut() into chunks, one VC.pipeline per chunk (every noise draw
    recorded, in order), restore() and, in the second case, clean_audio's spectral gate are all exercised."""
    import main.inference.convert as conv
    sr, version = 48000, "v2"
    ck = synthetic.make_synth_ckpt(sr, version, seed=seed)
    net_g = build_ref_synth(ck)
    from main.library.architectures import fairseq
    cpath = os.path.join("assets", "models", "embedders", "contentvec_synth.pt")
    torch.save(synthetic.make_contentvec_ckpt(seed + 1), cpath)
    hub = fairseq.load_model(cpath)[0][0].float().eval()
    torch.save(synthetic.rmvpe_state_dict(seed + 2), os.path.join("assets", "models", "predictors", "rmvpe.pt"))
    a = synthetic.synthetic_audio(5.5, seed=seed + 3)  # > the slicer's 5 s min_length, so cut() splits after it
    b = synthetic.synthetic_audio(2.0, seed=seed + 4)
    audio = np.concatenate([np.zeros(4000), a / np.abs(a).max() * 1.4, np.zeros(16000), b * 0.8,
                            np.zeros(3000)]).astype(np.float32)
    out = {"audio": audio, "sr": sr, "seed": seed, "pitch": 1, "protect": 0.33}
    for tag, clean in (("plain", False), ("clean", True)):
        vcv = conv.VoiceConverter.__new__(conv.VoiceConverter)
        vcv.config, vcv.device, vcv.sample_rate, vcv.checkpointing = conv.config, "cpu", 16000, False
        vcv.hubert_model, vcv.embed_suffix, vcv.suffix = hub, ".pt", ".pth"
        vcv.tgt_sr, vcv.net_g, vcv.sid, vcv.use_f0, vcv.version = sr, net_g, 0, 1, version
        vcv.vc = conv.VC(sr, conv.config)
        conv.load_audio = lambda *a, **k: audio.copy()
        written = []
        conv.sf.write = lambda path, data, rate, **k: written.append((data, rate))
        torch.manual_seed(seed + 5)
        with NoiseRecorder() as rec:
            vcv.convert_audio("in.wav", "out.wav", "", "contentvec_base", 1, "rmvpe", 0.0, 1, 0.33, 64, False, 1, 3,
                              clean, 0.5, "wav", split_audio=True)
        assert len(written) == 1, "reference convert_audio failed (it logs and returns)"
        kinds = [k for k, _ in rec.draws]
        assert len(kinds) % 3 == 0 and kinds[:3] == ["randn_like", "rand", "randn_like"], kinds
        out[f"{tag}_out"] = np.asarray(written[0][0], dtype=np.float32)
        out[f"{tag}_rate"] = written[0][1]
        out["nchunks"] = len(kinds) // 3
        for c in range(len(kinds) // 3):  # same seed, same draws in both cases: stored once
            for key, d in ((f"z_noise_{c}", rec.draws[3 * c][1]), (f"sine_noise_{c}", rec.draws[3 * c + 2][1])):
                if key in out:
                    assert np.array_equal(out[key], d.numpy())
                out[key] = d.numpy()
        print("convert", tag, out[f"{tag}_out"].shape, "chunks", len(kinds) // 3)
    np.savez_compressed(os.path.join(OUT, "convert.npz"), **out)


def gen_filtfilt(seed):
    from scipy import signal
    import main.inference.convert as conv
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.standard_normal(20000) * 0.3
    np.savez_compressed(os.path.join(OUT, "filtfilt.npz"), x=x, y=signal.filtfilt(conv.bh, conv.ah, x),
                        bh=conv.bh, ah=conv.ah)


def gen_crepe(seconds, seed):
    """VC.get_f0_crepe(x, "full") (convert.py:230-237) with synthetic Crepe-full weights; every
    scipy.stats.triang.rvs dither draw and every batch's network output are recorded."""
    import scipy.stats
    import main.inference.convert as conv
    from main.library.predictors import CREPE as RC
    torch.save(synthetic.crepe_state_dict(seed), os.path.join("assets", "models", "predictors", "crepe_full.pth"))
    vc = conv.VC(48000, conv.config)
    audio = synthetic.synthetic_audio(seconds, seed=seed + 1).astype(np.float64)
    draws, probs = [], []
    rvs0, post0 = scipy.stats.triang.rvs, RC.postprocess

    def rvs(*a, **k):
        v = rvs0(*a, **k)
        draws.append(np.asarray(v, dtype=np.float64).reshape(-1))
        return v

    def post(p, *a, **k):
        probs.append(p[0].t().numpy().copy())  # [T_batch][360]
        return post0(p, *a, **k)

    scipy.stats.triang.rvs, RC.postprocess = rvs, post
    np.random.seed(seed + 2)
    try:
        f0 = vc.get_f0_crepe(audio, "full")
    finally:
        scipy.stats.triang.rvs, RC.postprocess = rvs0, post0
    frames = next(RC.preprocess(torch.tensor(np.copy(audio))[None].float(), 16000, 160, 512, "cpu", True))
    np.savez_compressed(os.path.join(OUT, "crepe.npz"), seed=seed, audio=audio, f0=f0,
                        probs=np.concatenate(probs), dither=np.concatenate(draws), frames_head=frames[:40].numpy(),
                        batch_sizes=np.array([len(p) for p in probs]))
    print("crepe", f0.shape, float(np.mean(f0)), [len(p) for p in probs])


def gen_f0_opts(seed):
    """KATs of the reference's Autotune.autotune_f0 (f64 and f32 tracks, convert.py:168-179), get_f0's
    f0-file override (convert.py:304-323 with a recorded f0 track) and change_rms (convert.py:150-152)."""
    import main.inference.convert as conv
    vc = conv.VC(48000, conv.config)
    rng = np.random.Generator(np.random.PCG64(seed))
    f64 = rng.uniform(0, 1200, 997)
    f64[::9] = 0.0
    f64[5] = 50.455  # midway-ish between notes
    f32 = f64.astype(np.float32)
    at64 = conv.Autotune.autotune_f0(vc, f64.copy(), 0.75)
    at32 = conv.Autotune.autotune_f0(vc, f32.copy(), 0.75)
    # get_f0 with a stubbed method returning the recorded track (the f0 estimator is not under test)
    inp_f0 = np.array([[0.0, 220.0], [0.31, 330.0], [0.77, 180.5], [1.204, 410.25]], dtype=np.float32)
    x = np.zeros(16000 * 4)
    track = rng.uniform(80, 700, 1 + x.shape[0] // 160)
    vc.get_f0_rmvpe = lambda x, legacy=False, onnx=False: track.copy()
    coarse, f0 = vc.get_f0(x, x.shape[0] // 160, 3, "rmvpe", 3, 64, True, 0.6, inp_f0.copy())
    src = rng.standard_normal(16000 * 3) * np.linspace(0.01, 0.5, 16000 * 3)
    tgt = (rng.standard_normal(16000 * 9) * 0.2).astype(np.float32)
    cr = conv.change_rms(src, 16000, tgt.copy(), 16000, 0.35)
    np.savez_compressed(os.path.join(OUT, "f0_opts.npz"), f64=f64, f32=f32, at64=at64, at32=at32, inp_f0=inp_f0,
                        track=track, coarse=coarse, f0=f0, rms_src=src, rms_tgt=tgt, rms_out=cr)
    print("f0_opts", float(np.abs(at64 - f64).max()), coarse[:5], float(np.abs(cr).mean()))


def gen_edges(seed):
    """The reference's own silence slicer / RMS / restore (utils.py:172-250, preprocess.py:45-127) on
    the layouts of ``synthetic.SLICER_LAYOUTS`` (inputs rebuilt from their seeds on the test side)."""
    from main.library.utils import cut, restore
    from main.inference.preprocess import Slicer, get_rms
    out = {"seed": seed}
    for name, layout in synthetic.SLICER_LAYOUTS.items():
        audio = synthetic.silence_layout_audio(layout, seed=seed)
        chunks = cut(audio, 16000, db_thresh=-60, min_interval=500)
        out[f"{name}_bounds"] = np.array([[s, e] for _, s, e in chunks], dtype=np.int64)
        out[f"{name}_lens"] = np.array([len(c) for c, _, _ in chunks], dtype=np.int64)
        out[f"{name}_sums"] = np.array([float(np.sum(c, dtype=np.float64)) for c, _, _ in chunks])
        conv = [(s, e, np.repeat(c, 3) * 0.5) for c, s, e in chunks]  # stand-in "converted" chunks at 3x
        rest = restore(conv, total_len=len(audio), dtype=conv[0][2].dtype) if len(chunks) > 1 else conv[0][2]
        out[f"{name}_restore_len"] = np.int64(len(rest))
        out[f"{name}_restore_sum"] = float(np.sum(rest, dtype=np.float64))
        out[f"{name}_restore_nz"] = np.flatnonzero(rest == 0)[:: 997][:200]
        # dataset preprocessing slicer at a training rate (preprocess.py:131)
        a40 = synthetic.silence_layout_audio(layout, seed=seed, sr=40000)
        sl = Slicer(sr=40000, threshold=-42, min_length=1500, min_interval=400, hop_size=15, max_sil_kept=500)
        ch40 = sl.slice(a40)
        out[f"{name}_pre_lens"] = np.array([len(c) for c in ch40], dtype=np.int64)
        out[f"{name}_pre_sums"] = np.array([float(np.sum(c, dtype=np.float64)) for c in ch40])
        out[f"{name}_rms"] = get_rms(audio, 1280, 320).squeeze(0)
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    y = (rng.standard_normal(50000) * 0.1).astype(np.float32)
    out["rms_in"] = y
    out["rms_2048_512"] = get_rms(y, 2048, 512)
    # extract.py's coarse quantiser on f64 (RMVPE) and f32 (CREPE) tracks (extract.py:225-226)
    from main.inference.extract import FeatureInput
    fi = FeatureInput(device="cpu")
    f64 = rng.uniform(0, 1300, 4001)
    f64[::7] = 0.0
    out["coarse_in64"] = f64
    out["coarse_out64"] = fi.coarse_f0(f64)
    f32 = f64.astype(np.float32)
    out["coarse_in32"] = f32
    out["coarse_out32"] = fi.coarse_f0(f32)
    np.savez_compressed(os.path.join(OUT, "edges.npz"), **out)
    print("edges", {k: v.shape for k, v in out.items() if hasattr(v, "shape") and v.ndim})


def gen_denoise(seed):
    """noisereduce.reduce_noise (main/tools/noisereduce.py:199) as convert_audio calls it (convert.py:514-516):
    a single-chunk 48 kHz case at clean_strength 0.7, and a multi-chunk 44.1 kHz case (odd/even moving-mean
    window, chunk seams) with a small chunk_size / padding."""
    from main.tools.noisereduce import reduce_noise
    rng = np.random.default_rng(seed)
    out = {}
    cases = [("a", 48000, 2.0, 0.7, {}), ("b", 44100, 1.6, 1.0, dict(chunk_size=30000, padding=5000)),
             ("c", 40000, 1.2, 0.45, dict(chunk_size=20000, padding=3000))]
    for name, sr, secs, prop, kw in cases:
        n = int(sr * secs)
        t = np.arange(n) / sr
        y = (0.3 * np.sin(2 * np.pi * 220 * t) * (0.5 + 0.5 * np.sin(2 * np.pi * 0.7 * t)) +
             0.02 * rng.standard_normal(n)).astype(np.float32)
        y[n // 3: n // 3 + sr // 10] *= 0.01  # a near-silent gap
        o = reduce_noise(y=y, sr=sr, prop_decrease=prop, device="cpu", **kw)
        out[f"{name}_y"], out[f"{name}_out"] = y, np.asarray(o, dtype=np.float32)
        out[f"{name}_meta"] = np.array([sr, prop, kw.get("chunk_size", 600000), kw.get("padding", 30000)],
                                       dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "denoise.npz"), **out)
    print("denoise", {k: v.shape for k, v in out.items()})


class InjectNoise:
    """Replaces torch.randn_like during a reference VC.pipeline run with the draws the GPU parity tests inject
    (tests/test_gpu_configs.py SeededNoise): per segment s, the z_p draw then the SineGen draw, each
    torch.randn(shape, generator=manual_seed(salt + 13 s + len(kind))).  The reference's torch.rand draw
    (SineGen's random initial phase, zeroed at synthesizers.py:95) is left alone."""

    def __init__(self, salt):
        self.salt, self.n = salt, 0
        self._rl = torch.randn_like

    def __enter__(self):
        def rl(t, *a, **k):
            seg, kind = self.n // 2, ("z", "sine")[self.n % 2]
            self.n += 1
            g = torch.Generator().manual_seed(self.salt + 13 * seg + len(kind))
            return torch.randn(*t.shape, generator=g).to(t.dtype)
        torch.randn_like = rl
        return self

    def __exit__(self, *a):
        torch.randn_like = self._rl


def gen_ref_spread(seconds=30.0, seed=201, threads=(8, 7, 6, 5, 4, 3, 2, 1)):
    """The reference's OWN numerical spread on the headline clip (BASELINE configs[1]: 48k v2, RMVPE, 30 s,
    the models and input of tests/test_gpu_configs.py::test_cfg2_headline_30s_48k_fp32_vs_oracle): the
    reference's VC.pipeline (convert.py:388-458) run on CPU at several torch thread counts -- each an equally
    valid f32 evaluation of the same model -- plus one run whose f0 comes from the reference's RMVPE evaluated
    in float64 (model.double(), f64 mel), with the parity tests' injected noise so only arithmetic differs.
    Stored: every run's raw f0 track and salience-derived per-frame statistics, the pairwise waveform RMS
    spread, and the f64 salience's per-frame decision margins.  The headline parity test bounds the device
    against this spread."""
    import main.inference.convert as conv
    from main.library.predictors import RMVPE as RR
    ck = synthetic.make_synth_ckpt(48000, "v2", seed=seed)
    net_g = build_ref_synth(ck)
    from main.library.architectures import fairseq
    cpath = os.path.join("assets", "models", "embedders", "contentvec_synth.pt")
    torch.save(synthetic.make_contentvec_ckpt(seed + 1), cpath)
    hub = fairseq.load_model(cpath)[0][0].float().eval()
    rpath = os.path.join("assets", "models", "predictors", "rmvpe.pt")
    torch.save(synthetic.rmvpe_state_dict(seed + 2), rpath)
    audio = synthetic.synthetic_audio(seconds, seed=1000)
    sal_rec = []
    m2h0 = RR.RMVPE.mel2hidden

    def m2h(self, mel):
        h = m2h0(self, mel)
        sal_rec.append(h.squeeze(0).numpy().astype(np.float64))
        return h
    RR.RMVPE.mel2hidden = m2h

    def run(f0_override=None, x=None):
        vc = conv.VC(48000, conv.config)
        f0s = []
        g0 = vc.get_f0_rmvpe

        def gf(x, *a, **k):
            f = f0_override.copy() if f0_override is not None else g0(x, *a, **k)
            f0s.append(np.array(f, dtype=np.float64))
            return f
        vc.get_f0_rmvpe = gf
        with torch.no_grad(), InjectNoise(5):
            out = vc.pipeline(model=hub, net_g=net_g, sid=0, audio=(audio if x is None else x).copy(), pitch=0,
                              f0_method="rmvpe",
                              file_index="", index_rate=0.0, pitch_guidance=1, filter_radius=3, volume_envelope=1,
                              version="v2", protect=0.33, hop_length=64, f0_autotune=False, f0_autotune_strength=1,
                              suffix=".pth", embed_suffix=".pt", f0_file=None, f0_onnx=False, pbar=Pbar())
        assert len(f0s) == 1
        return np.asarray(out, np.float32), f0s[0]

    names, outs, f0s, sals = [], [], [], []
    for n in threads:
        torch.set_num_threads(n)
        sal_rec.clear()
        o, f = run()
        names.append(f"f32_threads{n}")
        outs.append(o)
        f0s.append(f)
        sals.append(sal_rec[0])
        print(names[-1], o.shape, float(np.sqrt(np.mean(o.astype(np.float64) ** 2))), flush=True)
    # the same input within its own f32 precision: every sample moved by one f32 ulp (toward +inf or -inf,
    # seeded) -- as numerically equivalent as the thread counts, and the size of a filtfilt evaluated in a
    # different (e.g. chunked) order (3e-8 of full scale)
    torch.set_num_threads(max(threads))
    for u in range(3):
        rng = np.random.default_rng(70 + u)
        x = np.nextafter(audio.astype(np.float32), np.where(rng.random(len(audio)) < 0.5, np.inf, -np.inf)
                         .astype(np.float32)).astype(audio.dtype)
        sal_rec.clear()
        o, f = run(x=x)
        names.append(f"f32_input_ulp{u}")
        outs.append(o)
        f0s.append(f)
        sals.append(sal_rec[0])
        print(names[-1], flush=True)
    # the reference's RMVPE in float64 on the same filtered, reflect-padded signal (convert.py:403,416,436)
    torch.set_num_threads(max(threads))
    r = RR.RMVPE(rpath, is_half=False, device="cpu")
    a = conv.signal.filtfilt(conv.bh, conv.ah, audio)
    ap = np.pad(a, (16000, 16000), mode="reflect")
    torch.set_default_dtype(torch.float64)
    try:
        me = RR.MelSpectrogram(False, 128, 16000, 1024, 160, None, 30, 8000).double()
        with torch.no_grad():
            mel = me(torch.from_numpy(ap).unsqueeze(0), center=True)
            nf = mel.shape[-1]
            mel = torch.nn.functional.pad(mel, (0, 32 * ((nf - 1) // 32 + 1) - nf), mode="reflect")
            s64 = r.model.double()(mel)[:, :nf].squeeze(0).numpy()
    finally:
        torch.set_default_dtype(torch.float32)
    f64 = r.decode(s64, thred=0.03)
    o64, _ = run(f0_override=f64)
    names.append("f64_rmvpe")
    outs.append(o64)
    f0s.append(f64)
    sals.append(s64)
    print("f64 rmvpe", flush=True)
    RR.RMVPE.mel2hidden = m2h0
    k = len(names)
    wav_rms = np.zeros((k, k))
    sal_max = np.zeros((k, k))
    for i in range(k):
        for j in range(k):
            wav_rms[i, j] = np.sqrt(np.mean((outs[i].astype(np.float64) - outs[j]) ** 2))
            sal_max[i, j] = np.abs(sals[i] - sals[j]).max()
    srt = np.sort(s64, axis=1)
    margin64 = np.minimum(srt[:, -1] - srt[:, -2], np.abs(srt[:, -1] - 0.03))
    # per frame: the largest |salience - f64 salience| over the f32 runs, and each run's decisions
    frame_spread = np.max([np.abs(s - s64).max(1) for s in sals[:-1]], 0)
    argmax = np.stack([s.argmax(1) for s in sals]).astype(np.int16)
    voiced = np.stack([s.max(1) > 0.03 for s in sals])
    # each run's salience at the f64 run's top-2 bins: the two values a frame's f0 decision compares
    # (argmax: top1 vs top2; voicing: top1 vs 0.03), so the reference's own decision noise per frame
    top2 = np.argsort(s64, axis=1)[:, -2:][:, ::-1].T.astype(np.int16)  # [2][F]: f64 top-1, top-2 bin
    fi = np.arange(s64.shape[0])
    sal_top2 = np.stack([np.stack([s[fi, top2[0]], s[fi, top2[1]]]) for s in sals])  # [runs][2][F] f64
    np.savez_compressed(os.path.join(OUT, "ref_spread_cfg2.npz"), seed=seed, seconds=seconds,
                        names=np.array(names), f0=np.stack(f0s), wav_rms=wav_rms, sal_max=sal_max,
                        out_rms=np.array([np.sqrt(np.mean(o.astype(np.float64) ** 2)) for o in outs]),
                        margin64=margin64.astype(np.float32), frame_spread=frame_spread.astype(np.float32),
                        argmax=argmax, voiced=voiced, sal64_max=srt[:, -1].astype(np.float32), top2=top2,
                        sal_top2=sal_top2)
    print("names", names)
    print("wav rms spread\n", np.array2string(wav_rms, precision=3))
    print("salience max abs spread\n", np.array2string(sal_max, precision=3))
    flips = [np.flatnonzero((argmax[i] != argmax[-1]) | (voiced[i] != voiced[-1])).tolist() for i in range(k - 1)]
    print("decision flips vs f64:", flips)


def main():
    os.makedirs(OUT, exist_ok=True)
    if len(sys.argv) > 1 and sys.argv[1] == "safetensors":
        # transformers probes its optional packages (librosa, ...) once, at import: import it before the stub
        # modules below exist, so that it sees the image as it is
        from transformers import HubertModel  # noqa: F401
    setup_harness()
    torch.set_num_threads(8)
    if len(sys.argv) > 1 and sys.argv[1] == "spread":
        gen_ref_spread()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "crepe":
        gen_crepe(6.0, seed=81)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "denoise":
        gen_denoise(seed=111)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "convert":
        gen_convert(seed=121)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "safetensors":
        gen_contentvec_hf(1.0, seed=131)
        gen_pipeline("pipeline_48k_v2_st", 48000, "v2", 2.0, seed=141, pitch=0, protect=0.33, embed=".safetensors")
        gen_pipeline("pipeline_32k_v1_st", 32000, "v1", 1.5, seed=142, pitch=3, protect=0.5, embed=".safetensors")
        return
    if len(sys.argv) > 1 and sys.argv[1] == "edges":
        gen_edges(seed=101)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "opts":
        gen_f0_opts(seed=91)
        gen_pipeline("pipeline_48k_v2_opts", 48000, "v2", 2.5, seed=53, pitch=2, protect=0.33, f0_autotune=True,
                     f0_autotune_strength=0.8, f0_lines=["0.0,200", "0.4,260.5", "0.9,150", "1.6,0", "2.0,310"],
                     volume_envelope=0.6)
        return
    gen_synth("synth_48k_v2", 48000, "v2", 120, seed=11)
    gen_synth("synth_40k_v2", 40000, "v2", 100, seed=12)
    gen_synth("synth_32k_v1", 32000, "v1", 100, seed=13)
    gen_contentvec(1.0, seed=21)
    gen_rmvpe(1.0, seed=31)
    gen_filtfilt(seed=41)
    gen_pipeline("pipeline_48k_v2", 48000, "v2", 2.0, seed=51, pitch=0, protect=0.33)
    gen_pipeline("pipeline_32k_v1", 32000, "v1", 1.5, seed=52, pitch=3, protect=0.5)
    gen_crepe(6.0, seed=81)
    gen_f0_opts(seed=91)
    gen_pipeline("pipeline_48k_v2_opts", 48000, "v2", 2.5, seed=53, pitch=2, protect=0.33, f0_autotune=True,
                 f0_autotune_strength=0.8, f0_lines=["0.0,200", "0.4,260.5", "0.9,150", "1.6,0", "2.0,310"],
                 volume_envelope=0.6)
    gen_edges(seed=101)
    gen_denoise(seed=111)


if __name__ == "__main__":
    main()
