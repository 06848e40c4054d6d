"""``VoiceConverter.convert_audio`` (main/inference/convert.py:479-523) and the batch-of-files loop of
``run_convert_script`` (:119-137) around the device ``VC.pipeline``: load, 0.95 peak limit, optional
silence split (edges.cut) with one ``pipeline()`` per chunk and zero-gap restore, resample to the
nearest standard rate, write.

Batch mode shards the files over ranks (one process per GPU, longest file first to the least-loaded
rank -- shard.shard_utterances); each rank writes its own outputs, so no waveform crosses ranks.

``clean_audio`` runs the spectral gate of main/tools/noisereduce.py on the device (rvc_amd.denoise).
Not on the device path (raise): formant shifting, non-WAV export.
Resampling (input != 16 kHz, or a model rate that is not a standard rate) is parity-unpinned
(audio_io module note).
"""
from __future__ import annotations

import logging
import os

import numpy as np

from . import audio_io, edges

log = logging.getLogger(__name__)

STANDARD_RATES = [8000, 11025, 12000, 16000, 22050, 24000, 32000, 44100, 48000, 96000]  # convert.py:495
AUDIO_EXTS = ("wav", "mp3", "flac", "ogg", "opus", "m4a", "mp4", "aac", "alac", "wma", "aiff", "webm", "ac3")


class VoiceConverterAMD:
    """The conversion front end over ``rvc_amd.pipeline.VC`` (already holding RMVPE / CREPE)."""

    def __init__(self, vc, net_g, hubert_model, tgt_sr, version="v2", sid=0, use_f0=1):
        self.vc = vc
        self.net_g = net_g
        self.hubert_model = hubert_model
        self.tgt_sr = tgt_sr
        self.version = version
        self.sid = sid
        self.use_f0 = use_f0
        self.sample_rate = 16000
        self.suffix = ".pth"
        # the loaded embedder's suffix (load_embedders_model returns it, utils.py:131-165); convert_audio checks it
        # against its embedders_mode argument
        self.embed_suffix = getattr(hubert_model, "embed_suffix", ".pt")

    def convert_audio(self, audio_input_path, audio_output_path, index_path="", embedder_model="contentvec_base",
                      pitch=0, f0_method="rmvpe", index_rate=0.5, volume_envelope=1, protect=0.5, hop_length=64,
                      f0_autotune=False, f0_autotune_strength=1, filter_radius=3, clean_audio=False,
                      clean_strength=0.7, export_format="wav", resample_sr=0, checkpointing=False, f0_file=None,
                      f0_onnx=False, embedders_mode="fairseq", formant_shifting=False, formant_qfrency=0.8,
                      formant_timbre=0.8, split_audio=False, pbar=None):
        """convert.py:479-523.  Like the reference, errors are logged and the call returns None;
        on success the written waveform is returned."""
        try:
            if formant_shifting:
                raise NotImplementedError("formant shifting is not on the MI355X path")
            if export_format != "wav":
                raise NotImplementedError("only WAV export (no soundfile / ffmpeg in this build)")
            embed_suffix = embed_suffix_of(embedders_mode)
            if embed_suffix != self.embed_suffix:
                raise ValueError(f"embedders_mode {embedders_mode!r} reads a {embed_suffix} embedder, but the loaded "
                                 f"model is a {self.embed_suffix} one")
            audio = audio_io.load_audio(audio_input_path, self.sample_rate)
            audio_max = np.abs(audio).max() / 0.95
            if audio_max > 1:
                audio /= audio_max
            if self.tgt_sr != resample_sr >= self.sample_rate:  # reference quirk: rebinds tgt_sr (:494)
                self.tgt_sr = resample_sr
            target_sr = min(STANDARD_RATES, key=lambda x: abs(x - self.tgt_sr))
            chunks = edges.cut(audio, self.sample_rate, db_thresh=-60, min_interval=500) if split_audio \
                else [(audio, 0, 0)]
            index = index_path.strip().strip('"').strip("\n").strip('"').strip().replace("trained", "added")
            converted = []
            for waveform, start, end in chunks:
                converted.append((start, end, self.vc.pipeline(
                    model=self.hubert_model, net_g=self.net_g, sid=self.sid, audio=waveform, pitch=pitch,
                    f0_method=f0_method, file_index=index, index_rate=index_rate, pitch_guidance=self.use_f0,
                    filter_radius=filter_radius, volume_envelope=volume_envelope, version=self.version,
                    protect=protect, hop_length=hop_length, f0_autotune=f0_autotune,
                    f0_autotune_strength=f0_autotune_strength, suffix=self.suffix, embed_suffix=embed_suffix,
                    f0_file=f0_file, f0_onnx=f0_onnx, pbar=pbar)))
            out = edges.restore(converted, total_len=len(audio), dtype=converted[0][2].dtype) if split_audio \
                else converted[0][2]
            if target_sr >= self.sample_rate and self.tgt_sr != target_sr:
                out = audio_io.resample(out, self.tgt_sr, target_sr)
            if clean_audio:  # convert.py:514-516
                from .denoise import reduce_noise
                out = reduce_noise(y=out, sr=target_sr, prop_decrease=clean_strength, device=self.vc.device)
            audio_io.write_wav(audio_output_path, out, target_sr)
            return out
        except Exception as e:  # noqa: BLE001 -- the reference logs and returns (convert.py:520-523)
            log.error(f"convert_audio: {e}")
            return None


def embed_suffix_of(embedders_mode):
    """main/library/utils.py:131-165: the suffix load_embedders_model returns for a mode ("fairseq" -> ".pt",
    "transformers" / "spin" -> ".safetensors"); ONNX embedders are not on the MI355X path."""
    if embedders_mode == "fairseq":
        return ".pt"
    if embedders_mode in ("transformers", "spin"):
        return ".safetensors"
    raise NotImplementedError(f"embedders_mode {embedders_mode!r}: fairseq and transformers are on the MI355X path")


def batch_files(input_path, export_format="wav"):
    """convert.py:119-131: (input, output) pairs of a directory, sorted for a stable sharding."""
    files = sorted(f for f in os.listdir(input_path) if f.lower().endswith(AUDIO_EXTS))
    return [(os.path.join(input_path, f), os.path.join(input_path, os.path.splitext(f)[0] + f"_output.{export_format}"))
            for f in files]


def convert_batch(cvt: VoiceConverterAMD, pairs, rank=0, world=1, **kw):
    """convert.py:129-135 over this rank's share (longest file first to the least-loaded rank, by file
    size); returns the (input, output) pairs this rank converted."""
    from .shard import shard_utterances
    sizes = [os.path.getsize(p) for p, _ in pairs]
    mine = [pairs[i] for i in shard_utterances(sizes, world)[rank]]
    for src, dst in mine:
        if os.path.exists(dst):
            os.remove(dst)
        cvt.convert_audio(src, dst, **kw)
    return mine
