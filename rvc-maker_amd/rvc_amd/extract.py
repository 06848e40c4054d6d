"""Training-side feature extraction: ``main/inference/extract.py`` on the same
device models as the conversion path, one process per GPU.

The reference extracts, for every 16 kHz slice of a training set,
  * the f0 track and its 1..255 coarse quantisation (``FeatureInput.process_file``, extract.py:228-238),
    sharded over the listed GPUs as ``paths[idx::len(gpus)]`` with a thread per GPU (:245-268);
  * the embedder features [T_f, 768] (v2) / [T_f, 256] (v1 final_proj) (``process_file_embedding``,
    :273-292), every file on every listed device in turn (:294-317);
then writes ``config.json`` and the shuffled ``filelist.txt`` (:52-77).

Here each rank (``torch.distributed`` process = one GPU) takes ``names[rank::world]`` for both passes --
the reference's pitch partition -- and runs RMVPE / CREPE and ContentVec through librvc_amd; the
files are the only output, so there is no data-path collective, only a barrier before rank 0 writes
the file list.  Host-side steps (coarse quantiser, file naming, list building) follow the reference
expression for expression; ``tests/golden/edges.npz`` pins ``coarse_f0`` against it.

f0 methods on the device: ``rmvpe`` and ``crepe-{tiny,...,full}`` (the reference's other estimators
-- pm, harvest, fcpe, ... -- are third-party or off the path and raise).  Embedders: fairseq
ContentVec (``embedders_mode="fairseq"``).
"""
from __future__ import annotations

import logging
import os
import random
import shutil

import numpy as np
import torch

from . import audio_io, ops

log = logging.getLogger(__name__)


class FeatureInputAMD:
    """extract.py:120-243 with the f0 estimators on the device."""

    def __init__(self, sample_rate=16000, hop_size=160, device="cuda:0", rmvpe=None, crepe=None):
        self.fs = sample_rate
        self.hop = hop_size
        self.f0_bin = 256
        self.f0_max = 1100.0
        self.f0_min = 50.0
        self.f0_mel_min = 1127 * np.log(1 + self.f0_min / 700)
        self.f0_mel_max = 1127 * np.log(1 + self.f0_max / 700)
        self.device = device
        self.rmvpe = rmvpe
        self.crepe = dict(crepe or {})

    def compute_f0(self, np_arr, f0_method, hop_length=160, f0_onnx=False):
        """extract.py:149-151 for the device methods: rmvpe -> f64 [1 + N//160] (RMVPE.infer_from_audio,
        thred 0.03); crepe-<cap> -> f32 [1 + N//160] (get_crepe, :173-180)."""
        if f0_onnx or "hybrid" in f0_method:
            raise NotImplementedError(f"f0 method {f0_method!r} (onnx / hybrid) is not on the device path")
        if f0_method == "rmvpe":
            if self.rmvpe is None:
                from .rmvpe import RMVPEAMD
                self.rmvpe = RMVPEAMD.from_file(os.path.join("assets", "models", "predictors", "rmvpe.pt"),
                                                self.device)
            return self.rmvpe.infer_from_audio(np_arr, thred=0.03)
        if f0_method.startswith("crepe-"):
            cap = f0_method.split("-", 1)[1]
            if cap not in self.crepe:
                from .crepe import CrepeAMD
                self.crepe[cap] = CrepeAMD.from_file(
                    os.path.join("assets", "models", "predictors", f"crepe_{cap}.pth"), cap, self.device)
            x = torch.from_numpy(np.copy(np_arr).astype(np.float32)).to(self.device)
            _, f0 = self.crepe[cap].f0_device(x, 0.0)
            return f0.cpu().numpy()
        raise NotImplementedError(f"f0 method {f0_method!r}: only rmvpe and crepe-* are on the device path")

    def coarse_f0(self, f0):
        """extract.py:225-226 (numpy, same expression and dtype promotion)."""
        return np.rint(np.clip(((1127 * np.log(1 + f0 / 700)) - self.f0_mel_min) * (self.f0_bin - 2) /
                               (self.f0_mel_max - self.f0_mel_min) + 1, 1, self.f0_bin - 1)).astype(int)

    def process_file(self, file_info, f0_method, hop_length, f0_onnx=False):
        """extract.py:228-238: f0_voiced/<name>.npy (raw f0) and f0/<name>.npy (coarse)."""
        inp_path, opt_path1, opt_path2, np_arr = file_info
        if os.path.exists(opt_path1 + ".npy") and os.path.exists(opt_path2 + ".npy"):
            return
        try:
            pit = self.compute_f0(np_arr, f0_method, hop_length, f0_onnx)
            if isinstance(pit, tuple):
                pit = pit[0]
            np.save(opt_path2, pit, allow_pickle=False)
            np.save(opt_path1, self.coarse_f0(pit), allow_pickle=False)
        except Exception as e:
            raise RuntimeError(f"extract f0 failed for {inp_path}: {e}") from e

    def process_files(self, files, f0_method, hop_length, f0_onnx=False, pbar=None):
        for info in files:
            self.process_file(info, f0_method, hop_length, f0_onnx)
            if pbar is not None:
                pbar.update()


def setup_paths(exp_dir, version=None):
    """extract.py:79-89."""
    wav_path = os.path.join(exp_dir, "sliced_audios_16k")
    if version:
        out_path = os.path.join(exp_dir, f"{version}_extracted")
        os.makedirs(out_path, exist_ok=True)
        return wav_path, out_path
    out1, out2 = os.path.join(exp_dir, "f0"), os.path.join(exp_dir, "f0_voiced")
    os.makedirs(out1, exist_ok=True)
    os.makedirs(out2, exist_ok=True)
    return wav_path, out1, out2


def run_pitch_extraction(exp_dir, f0_method, hop_length, feature_input: FeatureInputAMD, rank=0, world=1):
    """extract.py:245-268 for this rank's share (the reference's ``paths[idx::len(gpus)]``)."""
    input_root, out1, out2 = setup_paths(exp_dir)
    names = [n for n in sorted(os.listdir(input_root)) if "spec" not in n][rank::world]
    files = [(os.path.join(input_root, n), os.path.join(out1, n), os.path.join(out2, n),
              audio_io.load_audio(os.path.join(input_root, n), 16000)) for n in names]
    feature_input.process_files(files, f0_method, hop_length)
    return names


def read_wave(wav_path, normalize=False):
    """extract.py:91-100 -> f32 [1, N] (normalize: F.layer_norm over the whole signal; ContentVec's
    saved config has it off, and it is not on the device path)."""
    wav, sr = audio_io.read_wav(wav_path)
    if sr != 16000:
        raise ValueError(f"{wav_path}: sample rate {sr}, expected 16000")
    if wav.ndim == 2:
        wav = wav.mean(-1, dtype=np.float32)
    if normalize:
        raise NotImplementedError("normalize=True embedders are not on the device path")
    return wav.reshape(1, -1).astype(np.float32)


def embed_file(model, wav: np.ndarray, version: str, device) -> np.ndarray:
    """process_file_embedding's model call (extract.py:278-290) for the model's embedder kind (ContentVecAMD
    .embed_suffix): [T_f, 768] (v2) or [T_f, 256] (v1 final_proj; on layer 9 for ".pt", on the last layer for
    ".safetensors"), f32 on the host."""
    x = torch.from_numpy(np.ascontiguousarray(wav.reshape(-1))).to(device)
    feats = model.embed_cf(x, version)
    E, T = feats.shape
    out = torch.empty(T, E, device=x.device)
    ops.transpose(feats, out, 1, E, T)
    return out.cpu().numpy()


def process_file_embedding(file, wav_path, out_path, model, device, version, normalize=False):
    """extract.py:273-292."""
    out_file = os.path.join(out_path, file.replace("wav", "npy"))
    if os.path.exists(out_file):
        return
    feats = embed_file(model, read_wave(os.path.join(wav_path, file), normalize), version, device)
    if not np.isnan(feats).any():
        np.save(out_file, feats, allow_pickle=False)
    else:
        log.warning(f"{file} contains NaN")


def run_embedding_extraction(exp_dir, version, model, device, rank=0, world=1, normalize=False):
    """extract.py:294-317 for this rank's share."""
    wav_path, out_path = setup_paths(exp_dir, version)
    paths = sorted(f for f in os.listdir(wav_path) if f.endswith(".wav"))
    if not paths:
        raise FileNotFoundError(f"no .wav files in {wav_path}")
    mine = paths[rank::world]
    for f in mine:
        process_file_embedding(f, wav_path, out_path, model, device, version, normalize)
    return mine


def generate_config(rvc_version, sample_rate, model_path, configs_root=os.path.join("main", "configs")):
    """extract.py:52-54: copy configs/<version>/<sr>.json next to the experiment (reference layout)."""
    dst = os.path.join(model_path, "config.json")
    if not os.path.exists(dst):
        shutil.copy(os.path.join(configs_root, rvc_version, f"{sample_rate}.json"), dst)


def generate_filelist(pitch_guidance, model_path, rvc_version, sample_rate, embedders_mode="fairseq", rng=None):
    """extract.py:56-77: the names present in every output directory, plus two mute entries, shuffled."""
    gt_wavs_dir = os.path.join(model_path, "sliced_audios")
    feature_dir = os.path.join(model_path, f"{rvc_version}_extracted")
    f0_dir = f0nsf_dir = None
    if pitch_guidance:
        f0_dir, f0nsf_dir = os.path.join(model_path, "f0"), os.path.join(model_path, "f0_voiced")

    def stems(d):
        return set(name.split(".")[0] for name in os.listdir(d))

    names = stems(gt_wavs_dir) & stems(feature_dir)
    if pitch_guidance:
        names = names & stems(f0_dir) & stems(f0nsf_dir)
    options = []
    mute = os.path.join("assets", "logs", "mute" if embedders_mode != "spin" else "mute_spin")
    for name in names:
        options.append(f"{gt_wavs_dir}/{name}.wav|{feature_dir}/{name}.npy|{f0_dir}/{name}.wav.npy|"
                       f"{f0nsf_dir}/{name}.wav.npy|0" if pitch_guidance else
                       f"{gt_wavs_dir}/{name}.wav|{feature_dir}/{name}.npy|0")
    mute_audio = os.path.join(mute, "sliced_audios", f"mute{sample_rate}.wav")
    mute_feat = os.path.join(mute, f"{rvc_version}_extracted", "mute.npy")
    for _ in range(2):
        options.append(f"{mute_audio}|{mute_feat}|{os.path.join(mute, 'f0', 'mute.wav.npy')}|"
                       f"{os.path.join(mute, 'f0_voiced', 'mute.wav.npy')}|0" if pitch_guidance else
                       f"{mute_audio}|{mute_feat}|0")
    (rng or random).shuffle(options)
    with open(os.path.join(model_path, "filelist.txt"), "w") as f:
        f.write("\n".join(options))
    return options


def run_extract(exp_dir, version, f0_method, model, feature_input: FeatureInputAMD, device, hop_length=128,
                pitch_guidance=True, sample_rate=48000, dist=None, embedders_mode="fairseq", write_config=True):
    """extract.py:main (:319-358) for one rank: pitch + embedding passes on this rank's files, a
    barrier, then rank 0 writes config.json and filelist.txt."""
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    if pitch_guidance:
        run_pitch_extraction(exp_dir, f0_method, hop_length, feature_input, rank, world)
    run_embedding_extraction(exp_dir, version, model, device, rank, world)
    if dist is not None:
        dist.barrier()
    if rank == 0:
        if write_config:
            generate_config(version, sample_rate, exp_dir)
        generate_filelist(pitch_guidance, exp_dir, version, sample_rate, embedders_mode)
