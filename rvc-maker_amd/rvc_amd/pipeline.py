"""MI355X ``VC`` -- drop-in for ``main/inference/convert.py:VC`` (:181-458).

``VC(tgt_sr, config).pipeline(model, net_g, sid, audio, pitch, f0_method, file_index, index_rate,
pitch_guidance, filter_radius, volume_envelope, version, protect, hop_length, f0_autotune,
f0_autotune_strength, suffix, embed_suffix, f0_file=None, f0_onnx=False, pbar=None)`` keeps the
reference signature and returns float32 numpy audio at tgt_sr.  ``model`` is a
``ContentVecAMD`` (``.pt`` embedder), ``net_g`` a ``SynthesizerAMD`` (``.pth``); f0 is RMVPE
(``self.rmvpe``, loaded once from ``assets/models/predictors/rmvpe.pt`` or injected).

Everything runs on the device in the order of convert.py:388-458 -- the f64 filtfilt and
reflect padding included (filtfilt.hip), and the quiet-point search for inputs > x_max (pipeline.hip;
only its result, the segment plan, is read back to the host, which issues the segments).  The segment
loop keeps all tensors in HBM; ``pipeline_device`` is the HBM-resident form the bench times,
``pipeline`` adds the host copies of the reference signature.  ``VC.close()`` (or ``with VC(...)``)
releases the streams the library created for it.

FAISS retrieval (``file_index`` + ``index_rate``) runs on the device (retrieval.py / ivf.hip); the
index file is read without faiss (faiss_index.py) and kept resident per path.

f0 methods: "rmvpe" and "crepe-{tiny,small,medium,large,full}" (crepe.py), both on the device.

f0 autotune and f0 files run inside the f0 decode kernels; volume_envelope != 1 (change_rms) runs on
the device after the segment loop.  Embedders: fairseq ``.pt`` and transformers ``.safetensors``
(``ContentVecAMD.from_transformers``; the suffix picks the layer final_proj reads, convert.py:337-345).  Not on
this path (raise): other f0 methods, ONNX models, no-f0 models.
"""
from __future__ import annotations

import os
import weakref

import numpy as np
import torch
from scipy import signal

from . import contentvec as cvm
from . import ops

BH, AH = signal.butter(N=5, Wn=48, btype="high", fs=16000)  # convert.py:30


class _CuMaskedStream:
    """One stream restricted to part of the chip (rvc_stream_create_cu_mask), owned by a VC: ``close`` waits for
    its work and destroys it (rvc_stream_destroy).  Left to process teardown, such a stream crashed rocprofv3's
    kernel-trace finalisation."""

    def __init__(self, device, words):
        import ctypes
        out = ctypes.c_void_p()
        with torch.cuda.device(device):
            ops.check(ops._lib.load().rvc_stream_create_cu_mask(words, len(words), ctypes.byref(out)),
                      "stream_create_cu_mask")
        self.device, self.handle = device, out.value
        self.stream = torch.cuda.ExternalStream(out.value, device=device)

    def close(self):
        if self.handle:
            torch.cuda.synchronize(self.device)
            h, self.handle = self.handle, None
            ops.check(ops._lib.load().rvc_stream_destroy(h), "stream_destroy")


def _close_streams(owned, strict=False):
    """VC's finalizer (weakref.finalize: when the VC is collected or at interpreter exit) and ``VC.close``.  Only an
    explicit ``close()`` raises; the finalizer and ``__exit__`` under an exception log a failed release (e.g. after
    a sticky GPU error) and carry on, so they never bury the original failure."""
    first = None
    while owned:
        try:
            owned.pop().close()
        except Exception as e:  # noqa: BLE001
            if strict and first is None:
                first = e
            else:
                import logging
                logging.getLogger(__name__).warning(f"VC stream release failed: {e}")
    if first is not None:
        raise first


class Config:
    """The fields of main/configs/config.py:Config that VC reads (fp32 windows, config.py:83)."""

    def __init__(self, device="cuda:0", is_half=False):
        self.device = device
        self.is_half = is_half
        self.x_pad, self.x_query, self.x_center, self.x_max = (3, 10, 60, 65) if is_half else (1, 6, 38, 41)


class VC:
    CREPE_METHODS = {f"crepe-{c}": c for c in ("tiny", "small", "medium", "large", "full")}

    def __init__(self, tgt_sr, config, rmvpe=None, crepe=None):
        self.x_pad = config.x_pad
        self.x_query = config.x_query
        self.x_center = config.x_center
        self.x_max = config.x_max
        self.sample_rate = 16000
        self.window = 160
        self.t_pad = self.sample_rate * self.x_pad
        self.t_pad_tgt = tgt_sr * self.x_pad
        self.t_pad2 = self.t_pad * 2
        self.t_query = self.sample_rate * self.x_query
        self.t_center = self.sample_rate * self.x_center
        self.t_max = self.sample_rate * self.x_max
        self.f0_min, self.f0_max = 50, 1100
        self.device = config.device
        self.is_half = config.is_half
        self.rmvpe = rmvpe
        # library-created streams (CU-masked) this VC owns: destroyed by close() / at exit, after their work
        self._owned = []
        self._finalizer = weakref.finalize(self, _close_streams, self._owned)
        self.embed_suffix = None  # pipeline()'s embed_suffix during that call (convert.py:390); None = the model's own
        self.crepe = dict(crepe or {})  # capacity -> CrepeAMD (loaded on first use otherwise)
        self.noise_fn = None  # parity hook: noise_fn(seg, "z"|"sine", shape) -> device tensor
        self.seed = 0
        self._ws = None
        self.filt = ops.FiltFilt(BH, AH)

    # ------------------------------------------------------------------ host-side pieces
    def segment_points(self, audio: np.ndarray):
        """convert.py:404-412 on the host (numpy), as the reference computes it; pipeline_device runs the same
        search on the device (ops.quiet_points, tested equal)."""
        opt_ts = []
        audio_pad = np.pad(audio, (self.window // 2, self.window // 2), mode="reflect")
        if audio_pad.shape[0] > self.t_max:
            audio_sum = np.zeros_like(audio)
            for i in range(self.window):
                audio_sum += audio_pad[i: i - self.window]
            for t in range(self.t_center, audio.shape[0], self.t_center):
                seg = np.abs(audio_sum[t - self.t_query: t + self.t_query])
                opt_ts.append(t - self.t_query + np.where(seg == seg.min())[0][0])
        return opt_ts

    def _rmvpe(self):
        if self.rmvpe is None:
            from .rmvpe import RMVPEAMD
            self.rmvpe = RMVPEAMD.from_file(os.path.join("assets", "models", "predictors", "rmvpe.pt"), self.device)
        return self.rmvpe

    def _crepe(self, capacity):
        if capacity not in self.crepe:
            from .crepe import CrepeAMD
            self.crepe[capacity] = CrepeAMD.from_file(
                os.path.join("assets", "models", "predictors", f"crepe_{capacity}.pth"), capacity, self.device)
        return self.crepe[capacity]

    def f0_device(self, xp, pitch, f0_method="rmvpe", f0_autotune=False, f0_autotune_strength=1.0, inp_f0=None,
                  xp64=None):
        """VC.get_f0 (convert.py:304-323) on the device: (coarse int64 [T], pitchf f32 [T]).  Autotune
        and the f0-file override run inside the decode kernels, in the reference's order.  "pm" reads the
        f64 signal ``xp64`` (the reference hands parselmouth the f64 filtfilt output)."""
        post = None
        if f0_autotune or inp_f0 is not None:
            rep, off = f0_override(inp_f0, self.x_pad) if inp_f0 is not None else (None, 0)
            post = ops.F0Post(f0_autotune_strength if f0_autotune else None, rep, off, xp.device)
        if f0_method == "rmvpe":
            coarse, pitchf, _ = self._rmvpe().f0_device(xp, 0.03, float(pitch), post=post)
            return coarse, pitchf
        if f0_method in self.CREPE_METHODS:
            return self._crepe(self.CREPE_METHODS[f0_method]).f0_device(xp, float(pitch), post=post)
        if f0_method == "pm":
            if xp64 is None:
                raise ValueError("f0 method 'pm' reads the f64 filtered signal (xp64)")
            if getattr(self, "pm", None) is None:
                from .pm import PitchPM
                self.pm = PitchPM(xp64.device)
            return self.pm.f0_device(xp64, xp.numel() // self.window, float(pitch), post=post)
        raise NotImplementedError(f"f0 method {f0_method!r}: rmvpe, crepe-* and pm are on the MI355X path")

    # ------------------------------------------------------------------ device pieces
    def features_device(self, model, a0, version):
        """convert.py:337-345: embedder features of segment a0 [N] (or [B][N]), channels-first [(B)][E][T_f], for
        the pipeline's embed suffix (".pt": layer 9 + final_proj for v1; ".safetensors": the last layer)."""
        return model.embed_cf(a0, version, self.embed_suffix)

    def voice_conversion_device(self, model, net_g, sid, a0, pitch, pitchf, version, protect, seg, feats=None,
                                index=None, index_rate=0.0):
        """VC.voice_conversion (convert.py:328-386) on a device segment a0 [N] -> waveform [T*upp]."""
        prep = self.prior_device(model, net_g, sid, a0, pitch, pitchf, version, protect, seg, feats, index,
                                 index_rate, self.seed + seg)
        return self.generate_device(net_g, prep, seg, self.seed + seg)

    def prior_device(self, model, net_g, sid, a0, pitch, pitchf, version, protect, seg, feats=None, index=None,
                     index_rate=0.0, seed=0):
        """voice_conversion up to the generator: retrieval, phone upsample + protect (convert.py:347-378),
        TextEncoder, prior sample and flow^-1 (Synthesizer.infer, synthesizers.py:446-460) -> a dict for
        generate_device."""
        N = a0.numel()
        if feats is None:
            feats = self.features_device(model, a0, version)
        feats0 = feats  # convert.py:347: the protect blend uses the pre-retrieval features
        if index is not None and index_rate != 0:
            feats = index.retrieve_cf(feats, index_rate)
        E, Tf = feats.shape
        p_len = N // self.window
        T = min(2 * Tf, p_len)  # convert.py:364-370
        if 2 * Tf > p_len:
            raise NotImplementedError("phone longer than p_len (x_mask padding) never occurs in VC.pipeline")
        pitch, pitchf = pitch[:T], pitchf[:T]
        if pitch.numel() < T:
            raise ValueError("pitch shorter than the phone sequence")
        phone = torch.empty(E, T, device=a0.device)
        blend = protect < 0.5
        ops.phone_upsample(feats, feats0, pitchf if blend else None, phone, E, Tf, T, float(protect))
        zn = self.noise_fn(seg, "z", (1, net_g.inter, T)) if self.noise_fn else None
        z, _, _, gc = net_g.prior_cf(phone, pitch.contiguous(), sid, zn, seed)
        return {"z": z, "gc": gc, "pitchf": pitchf.contiguous(), "T": T}

    def voice_conversion_batch_device(self, model, net_g, sid, items, version, protect, index=None, index_rate=0.0,
                                      seeds=(), noise_segs=None):
        """``voice_conversion_device`` over B clips of one length with the synthesizer batched: retrieval and
        the phone upsample + protect per clip (convert.py:347-378), then TextEncoder, prior sample, flow^-1
        and the NSF generator as B-clip launches (Synthesizer.infer, synthesizers.py:446-465).  items: [(xp,
        coarse, pitchf, feats)] per clip; clip b draws its noise with seeds[b] (parity mode: noise_fn of
        segment noise_segs[b], default 0).  -> waveforms [B][T*upp]."""
        B = len(items)
        phone = pitch = pf = None
        for b, (xp, coarse, pitchf, feats) in enumerate(items):
            p_len = xp.numel() // self.window
            feats0 = feats  # convert.py:347: the protect blend uses the pre-retrieval features
            if index is not None and index_rate != 0:
                feats = index.retrieve_cf(feats, index_rate)
            E, Tf = feats.shape
            T = min(2 * Tf, p_len)  # convert.py:364-370
            if 2 * Tf > p_len:
                raise NotImplementedError("phone longer than p_len (x_mask padding) never occurs in VC.pipeline")
            if phone is None:
                phone = torch.empty(B, E, T, device=xp.device)
                pitch = torch.empty(B, T, dtype=coarse.dtype, device=xp.device)
                pf = torch.empty(B, T, dtype=pitchf.dtype, device=xp.device)
            elif phone.shape[2] != T:
                raise ValueError("voice_conversion_batch_device: clips of one length")
            if coarse.numel() < T:
                raise ValueError("pitch shorter than the phone sequence")
            ops.phone_upsample(feats, feats0, pitchf[:T] if protect < 0.5 else None, phone[b], E, Tf, T,
                               float(protect))
            pitch[b].copy_(coarse[:T])
            pf[b].copy_(pitchf[:T])
        T = phone.shape[2]
        zn = sn = None
        if self.noise_fn:
            segs = noise_segs or [0] * B
            zn = torch.stack([self.noise_fn(g, "z", (1, net_g.inter, T)).reshape(net_g.inter, T) for g in segs])
            sn = torch.stack([self.noise_fn(g, "sine", (1, T * net_g.upp, 1)).reshape(-1) for g in segs])
        z, _, _, gc = net_g.prior_batch(phone, pitch, sid, zn, seeds)
        return net_g.decode_batch(z, pf, gc, sn, seeds)

    def generate_device(self, net_g, prep, seg, seed):
        """The NSF generator on prior_device's z (synthesizers.py:461-465) -> waveform [T*upp]."""
        sn = self.noise_fn(seg, "sine", (1, prep["T"] * net_g.upp, 1)) if self.noise_fn else None
        return net_g.decode_cf(prep["z"], prep["pitchf"], prep["gc"], sn, seed)

    def pipeline_device(self, model, net_g, sid, audio, pitch, version, protect, index=None, index_rate=0.0,
                        f0_method="rmvpe", f0_autotune=False, f0_autotune_strength=1.0, inp_f0=None,
                        volume_envelope=1.0):
        """The hot path with inputs and output in HBM: audio device f32 [N] at 16 kHz (numpy accepted)
        -> device f32 waveform at tgt_sr.  filtfilt + reflect padding run on the device (f64)."""
        if not torch.is_tensor(audio):
            audio = torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)).to(self.device)
        N = audio.numel()
        long_input = N + self.window > self.t_max  # convert.py:406 (audio padded by window/2 each side)
        xp, xp64 = self.filt(audio.contiguous(), self.t_pad,
                             want_f64=long_input or volume_envelope != 1 or f0_method == "pm")
        opt_ts = []
        if long_input:  # quiet-point search on the filtered f64 signal (device; the plan reads the points back)
            opt_ts = ops.quiet_points(xp64[self.t_pad: self.t_pad + N], self.window, self.t_center, self.t_query,
                                      self.t_max)
        p_len = xp.numel() // self.window
        f0_opts = dict(f0_autotune=f0_autotune, f0_autotune_strength=f0_autotune_strength, inp_f0=inp_f0)
        src64 = xp64[self.t_pad: self.t_pad + N] if volume_envelope != 1 else None
        return self._pipeline_on_device(model, net_g, sid, xp, opt_ts, p_len, pitch, version, protect, index,
                                        index_rate, f0_method, f0_opts, volume_envelope, src64, xp64)

    def pipeline_device_batch(self, model, net_g, sid, audios, pitch, version, protect, index=None, index_rate=0.0,
                              f0_method="rmvpe"):
        """``pipeline_device`` over B equal-length clips at once (the chunk loop of convert.py:506-507 for
        equal-length chunks, BASELINE configs[2]): RMVPE (U-Net, W_ih, the B BiGRU recurrences side by side)
        and ContentVec run as B-batched launches on their two streams, then the synthesizer as B-clip launches
        (``voice_conversion_batch_device``; RVC_AMD_SYNTH_BATCH=0: per clip).  Clip b draws its noise with seed
        ``self.seed + b``: it equals ``pipeline_device`` of that clip with ``seed = self.seed + b``, up to the
        summation order of the batched launches (split-K / split-KV follow the batched grid).  Clips must fit one segment
        (N + window <= t_max, 41 s)."""
        B = len(audios)
        audios = [a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(
            self.device) for a in audios]
        N = audios[0].numel()
        if any(a.numel() != N for a in audios) or N + self.window > self.t_max:
            raise ValueError("pipeline_device_batch: equal-length clips of at most t_max samples")
        xpb = torch.stack([self.filt(a.contiguous(), self.t_pad)[0] for a in audios])  # [B][Np]
        p_len = xpb.shape[1] // self.window
        main = torch.cuda.current_stream(xpb.device)
        side = self._side_stream(xpb.device)
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(side):
            side.wait_event(ready)
            if f0_method == "rmvpe":
                coarse, pitchf = self._rmvpe().f0_device_batch(xpb, 0.03, float(pitch))
            else:
                pairs = [self.f0_device(xpb[b], pitch, f0_method) for b in range(B)]
                coarse, pitchf = torch.stack([c for c, _ in pairs]), torch.stack([f for _, f in pairs])
            f0_done = torch.cuda.Event()
            f0_done.record(side)
        feats = self.features_device(model, xpb, version)
        main.wait_event(f0_done)
        for t in (coarse, pitchf):
            t.record_stream(main)
        xpb.record_stream(side)
        tp = self.t_pad_tgt
        if self._ws is None:
            self._ws = torch.zeros(4, dtype=torch.int32, device=xpb.device)
        outs = []
        if B > 1 and self.SYNTH_BATCH:
            items = [(xpb[b], coarse[b], pitchf[b], feats[b]) for b in range(B)]
            ob = self.voice_conversion_batch_device(model, net_g, sid, items, version, protect, index, index_rate,
                                                    [self.seed + b for b in range(B)], list(range(B)))
            for b in range(B):
                out = ob[b, tp: ob.shape[1] - tp]
                ops.peak_normalize(out, self._ws)
                outs.append(out)
            return outs
        for b in range(B):
            o = self.voice_conversion_device(model, net_g, sid, xpb[b], coarse[b, :p_len], pitchf[b, :p_len], version,
                                             protect, b, feats=feats[b], index=index, index_rate=index_rate)
            out = o[tp: o.numel() - tp]
            ops.peak_normalize(out, self._ws)
            outs.append(out)
        return outs

    def pipeline_device_stream(self, model, net_g, sid, audios, pitch, version, protect, index=None, index_rate=0.0,
                               f0_method="rmvpe", batch=1, events=None, seeds=None, host_out=None):
        """``pipeline_device`` over a sequence of clips (the file / chunk loops of convert.py:129-135 and
        :506-507) with clip k+1's front end -- filtfilt, f0 on the side stream, ContentVec features -- issued
        on a front stream while clip k's synthesizer runs on a back stream.  The two are independent, so the
        front end's small, latency-bound launches (the U-Net's deep levels, the BiGRU's 32 workgroups, the
        ContentVec GEMMs) fill the CUs the generator's kernels leave between blocks and launches instead of
        running as a phase of their own.  ``batch`` > 1 runs the front end over groups of that many
        equal-length clips at once (``pipeline_device_batch``'s batched RMVPE and ContentVec), group g+1's
        under group g's synthesizer, which runs as B-clip launches (``voice_conversion_batch_device``).

        Clip k draws its noise with seed ``seeds[k]`` when ``seeds`` is given (a sharded job keys it to the global
        utterance index, so the output does not depend on the rank or world size), else ``self.seed + k`` (as
        ``pipeline_device_batch``): at batch 1 its
        waveform is bit-identical to ``pipeline_device`` of that clip at ``seed = self.seed + k`` -- every
        launch is the same launch on the same data, only its stream differs (batched groups: up to the
        batched launches' split-K / split-KV order, as ``pipeline_device_batch``).  Clips must fit one segment (N + window
        <= t_max, 41 s; longer inputs go through ``pipeline_device``'s host quiet-point search).  Returns the
        list of device waveforms, ordered on the caller's current stream.  ``events`` (a list) collects
        timing events (role, group, torch.cuda.Event) at each group's front / back start and end.  ``host_out``
        (a list of pinned host f32 tensors, one per clip, each at least the clip's output length) receives each
        waveform as it is finished: a non-blocking copy on the synthesizer's stream right after that clip,
        overlapping the next clips' front end (the reference's ``.cpu()`` of each output, convert.py:455)."""

        def mark(role, g, stream):
            if events is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(stream)
                events.append((role, g, ev))

        audios = [a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(
            self.device) for a in audios]
        if any(a.numel() + self.window > self.t_max for a in audios):
            raise ValueError("pipeline_device_stream: clips of at most t_max samples (one segment each)")
        if not audios:
            return []
        groups = [audios[i:i + max(1, batch)] for i in range(0, len(audios), max(1, batch))]
        if any(len({a.numel() for a in g}) > 1 for g in groups):
            raise ValueError("pipeline_device_stream: a batched group needs equal-length clips")
        dev = audios[0].device
        caller = torch.cuda.current_stream(dev)
        back = self._aux_stream(dev, "back")
        # front pipelines (front + fside stream pairs) taken in turn by consecutive groups, so that one
        # group's latency-bound front end (U-Net launches, the BiGRU recurrence) overlaps the next one's
        fronts = [(self._aux_stream(dev, "front", i), self._aux_stream(dev, "fside", i)) for i in range(self.FRONTS)]
        if self._ws is None:
            self._ws = torch.zeros(4, dtype=torch.int32, device=dev)
        seed0, tp = self.seed, self.t_pad_tgt
        if seeds is not None and len(seeds) != len(audios):
            raise ValueError("pipeline_device_stream: one seed per clip")
        if host_out is not None and len(host_out) != len(audios):
            raise ValueError("pipeline_device_stream: one host buffer per clip")
        seed_of = (lambda k: int(seeds[k])) if seeds is not None else (lambda k: seed0 + k)

        def emit(out):
            outs.append(out)
            if host_out is not None:
                # D2H of this clip on the back stream, right behind its synthesizer.  (On the caller's stream it made
                # the caller wait for each clip, and the front streams wait for the caller before every group: the
                # front end then never ran more than one clip ahead -- round 5 timeline, the back stream idle 35 %.)
                host_out[len(outs) - 1][: out.numel()].copy_(out, non_blocking=True)

        def issue_front(group, g):
            """front end of one group on the front / fside streams -> ([(xp, coarse, pitchf, feats)], event).
            (The synthesizer's TextEncoder / prior / flow stay on the back stream: moved to the front stream they
            made the front end the critical chain, 705 vs 820 xRT.)"""
            front, side = fronts[g % len(fronts)]
            with torch.cuda.stream(front):
                front.wait_stream(caller)  # the caller wrote the inputs on its own stream
                mark("front_start", g, front)
                for a in group:
                    a.record_stream(front)
                pm = f0_method == "pm"  # pm reads the f64 filtered signal
                filtered = [self.filt(a.contiguous(), self.t_pad, want_f64=pm) for a in group]
                xps, x64s = [f for f, _ in filtered], [f for _, f in filtered]
                xp = xps[0] if len(group) == 1 else torch.stack(xps)
                ready = torch.cuda.Event()
                ready.record(front)
                with torch.cuda.stream(side):
                    side.wait_event(ready)
                    if len(group) == 1:
                        coarse, pitchf = self.f0_device(xp, pitch, f0_method, xp64=x64s[0])
                    elif f0_method == "rmvpe":
                        coarse, pitchf = self._rmvpe().f0_device_batch(xp, 0.03, float(pitch))
                    else:
                        pairs = [self.f0_device(xp[b], pitch, f0_method, xp64=x64s[b]) for b in range(len(group))]
                        coarse, pitchf = torch.stack([c for c, _ in pairs]), torch.stack([f for _, f in pairs])
                    f0_done = torch.cuda.Event()
                    f0_done.record(side)
                feats = self.features_device(model, xp, version)
                front.wait_event(f0_done)
                for t in (coarse, pitchf):
                    t.record_stream(front)
                xp.record_stream(side)
                for t in x64s:
                    if t is not None:
                        t.record_stream(side)
                if len(group) == 1:
                    items = [(xp, coarse, pitchf, feats)]
                else:
                    items = [(xp[b], coarse[b], pitchf[b], feats[b]) for b in range(len(group))]
                done = torch.cuda.Event()
                done.record(front)
                mark("front_end", g, front)
            return items, done

        outs = []
        nxt = issue_front(groups[0], 0)
        try:
            for g in range(len(groups)):
                items, done = nxt
                if g + 1 < len(groups):
                    nxt = issue_front(groups[g + 1], g + 1)  # queued ahead of group g's synthesizers
                with torch.cuda.stream(back):
                    back.wait_event(done)
                    mark("back_start", g, back)
                    for it in items:
                        for t in it:
                            t.record_stream(back)
                    if len(items) > 1 and self.SYNTH_BATCH:
                        gseeds = [seed_of(len(outs) + b) for b in range(len(items))]
                        ob = self.voice_conversion_batch_device(model, net_g, sid, items, version, protect, index,
                                                                index_rate, gseeds)
                        for b in range(len(items)):
                            out = ob[b, tp: ob.shape[1] - tp]
                            ops.peak_normalize(out, self._ws)
                            emit(out)
                        items = []
                    for xp, coarse, pitchf, feats in items:
                        p_len = xp.numel() // self.window
                        self.seed = seed_of(len(outs))
                        o = self.voice_conversion_device(model, net_g, sid, xp, coarse[:p_len], pitchf[:p_len],
                                                         version, protect, 0, feats=feats, index=index,
                                                         index_rate=index_rate)
                        out = o[tp: o.numel() - tp]
                        ops.peak_normalize(out, self._ws)
                        emit(out)
                    mark("back_end", g, back)
        finally:
            self.seed = seed0
        caller.wait_stream(back)
        for o in outs:
            o.record_stream(caller)
        return outs

    # batched groups of the clip stream run one B-clip synthesizer (RVC_AMD_SYNTH_BATCH=0: one per clip)
    SYNTH_BATCH = os.environ.get("RVC_AMD_SYNTH_BATCH", "1") != "0"
    # clip-stream priorities (measured on one MI355X, 10 x 30 s clips: synthesizer stream high, front end
    # normal: 808 xRT; front end high: 781; per-call pipeline_device: 678)
    STREAM_PRIORITY = {"front": 0, "fside": 0, "back": -1}
    # pool slot per role: streams of equal priority and slot are one stream object
    STREAM_SLOT = {"front": 1, "fside": 0, "back": 0, "side": 0}
    # front pipelines of the clip stream (RVC_STREAM_FRONTS); pipeline i > 0 takes pool slots 2i, 2i + 1.
    # Each needs its own hardware queues: the process's GPU_MAX_HW_QUEUES must cover 2 + 2 * FRONTS streams.
    FRONTS = max(1, int(os.environ.get("RVC_STREAM_FRONTS", "1")))

    def _aux_stream(self, device, role, pipe=0):
        """The clip stream's streams: "front" (filtfilt, ContentVec), "fside" (its f0 branch) and "back" (the
        synthesizer).  The back stream runs at high priority: the synthesizers form the critical chain of
        the stream, and the front end's few-block, latency-bound launches fill the CUs between them
        (RVC_AMD_{FRONT,FSIDE,BACK}_PRIORITY override)."""
        prio = int(os.environ.get(f"RVC_AMD_{role.upper()}_PRIORITY", str(self.STREAM_PRIORITY[role])))
        slot = self.STREAM_SLOT[role] if pipe == 0 else 2 * pipe + (role == "front")
        return self._pooled_stream(device, prio, slot, self.BACK_CU_MASK if role == "back" else "none")

    def _pooled_stream(self, device, prio, slot, mask="none"):
        """Streams are pooled by (priority, slot) and shared between roles that never run at once (the
        per-call side stream is the clip stream's back stream, ClipGraph's normal-priority fork its fside
        stream).  The device has GPU_MAX_HW_QUEUES = 4 hardware queues per process: with the default stream,
        these three fill them, and a fifth stream would share a queue -- serialising, for example, RMVPE
        behind ContentVec (measured: a per-call pass 30 % slower once a fifth stream existed)."""
        key = f"{device}/{prio}/{slot}" + (f"/{mask}" if mask != "none" else "")
        if getattr(self, "_streams", None) is None:
            self._streams = {}
        if key not in self._streams:
            if mask != "none":
                owner = _CuMaskedStream(device, self._cu_mask_words(device, mask))
                self._owned.append(owner)
                self._streams[key] = owner.stream
            else:
                self._streams[key] = torch.cuda.Stream(device=device, priority=prio)
        return self._streams[key]

    def close(self, strict=True):
        """Wait for and destroy the streams the library created for this VC (also done when the VC is collected
        and at interpreter exit); the VC creates new ones if used again.  ``strict`` False logs a failed release
        instead of raising."""
        self._finalizer.detach()
        owned = self._owned
        self._streams = {}
        self._owned = []
        self._finalizer = weakref.finalize(self, _close_streams, self._owned)
        _close_streams(owned, strict=strict)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, *exc):
        self.close(strict=exc_type is None)  # under an exception, never replace it with a release failure

    # The synthesizer (back) stream is created through hipExtStreamCreateWithCUMask (RVC_BACK_CU_MASK:
    # "mod:m:r", "top:n" or "none").  What a mask does was probed in round 4 (scripts/cu_mask_probe.hip,
    # profiles/r4_cu_mask_probe.txt): mask bit i lands on XCD i mod 8, so "mod:8:7" names all 32 CUs of one XCD,
    # and the runtime then applies no mask at all -- its launches still run on all 256 CUs; "top:32" does
    # leave 4 CUs on each XCD (28 of 32 used per XCD).  The default "mod:8:7" is therefore an unmasked stream of
    # default priority on a hardware queue of its own; that is what the round-3 numbers measured (986-990 xRT
    # against 899-1003 for the high-priority back stream, "none"), while the real 4-CU-per-XCD mask ("top:32")
    # ran 798-801.  With the f64 RMVPE (round 4, interleaved on one box, 2 runs each): "none" 861 / 861,
    # "mod:8:7" 842 / 842, "none" at normal back priority 669 / 667 -- so the default is now the plain
    # high-priority back stream.  A masked stream is its own pooled stream, apart from the per-call side stream
    # (sharing it: 805 -> 650 xRT per call).
    BACK_CU_MASK = os.environ.get("RVC_BACK_CU_MASK", "none")

    @staticmethod
    def _cu_mask_words(device, spec):
        """The CU mask of BACK_CU_MASK's form: "top:n" leaves out the last n CUs of the mask, "mod:m:r" every CU
        whose index is r mod m."""
        import ctypes
        ncu = torch.cuda.get_device_properties(device).multi_processor_count
        kind, *arg = spec.split(":")
        keep = [True] * ncu
        for i in range(ncu):
            if kind == "top":
                keep[i] = i < ncu - int(arg[0])
            elif kind == "mod":
                keep[i] = i % int(arg[0]) != int(arg[1])
            else:
                raise ValueError(f"RVC_BACK_CU_MASK: unknown form {spec!r}")
        words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
        for i in range(ncu):
            if keep[i]:
                words[i // 32] |= 1 << (i % 32)
        return words

    def _side_stream(self, device):
        # RMVPE / CREPE (the longer branch, with the BiGRU's co-resident workgroups) on a high-priority
        # stream so that its launches are dispatched ahead of the ContentVec ones: +1.5 % eager (603 ->
        # 612 xRT).  A captured graph runs 17 % slower with it, so ClipGraph sets side_priority = 0.
        # With the masked synthesizer stream (BACK_CU_MASK) the high-priority side stream would be a fifth stream
        # on the process's 4 hardware queues, sharing one (per call 805 -> 550 xRT): it is then the clip stream's
        # fside stream (normal priority), which is idle whenever a per-call pass runs.
        dflt = "-1" if self.BACK_CU_MASK == "none" else "0"
        prio = self.side_priority if getattr(self, "side_priority", None) is not None \
            else int(os.environ.get("RVC_AMD_SIDE_PRIORITY", dflt))
        return self._pooled_stream(device, prio, self.STREAM_SLOT["side"])

    def _pipeline_on_device(self, model, net_g, sid, xp, opt_ts, p_len, pitch, version, protect, index=None,
                            index_rate=0.0, f0_method="rmvpe", f0_opts=None, volume_envelope=1.0, src64=None, xp64=None):
        # Segments of convert.py:419-440: [s, t + t_pad2 + w) for each quiet point t, then [t, end).
        w, tp = self.window, self.t_pad_tgt
        segs, s = [], 0
        for t in opt_ts:
            t = t // w * w
            segs.append((s, t + self.t_pad2 + w, s // w, (t + self.t_pad2) // w))
            s = t
        last = opt_ts[-1] // w * w if opt_ts else None
        segs.append((last or 0, xp.numel(), (last or 0) // w, None))
        # RMVPE (f0 over the whole padded signal) runs on a side stream, concurrently with the
        # ContentVec features of every segment on the main stream: the two networks are independent
        # until the synthesizer, and RMVPE's BiGRU recurrence occupies only 32 CUs.
        main = torch.cuda.current_stream(xp.device)
        side = self._side_stream(xp.device)
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(side):
            side.wait_event(ready)
            coarse, pitchf = self.f0_device(xp, pitch, f0_method, xp64=xp64, **(f0_opts or {}))
            f0_done = torch.cuda.Event()
            f0_done.record(side)
        feats = [self.features_device(model, xp[a:b], version) for a, b, _, _ in segs]
        main.wait_event(f0_done)
        coarse.record_stream(main)
        pitchf.record_stream(main)
        xp.record_stream(side)
        if xp64 is not None:
            xp64.record_stream(side)
        coarse, pitchf = coarse[:p_len], pitchf[:p_len]
        outs = []
        for seg, ((a, b, fa, fb), fe) in enumerate(zip(segs, feats)):
            o = self.voice_conversion_device(model, net_g, sid, xp[a:b], coarse[fa:fb], pitchf[fa:fb], version,
                                             protect, seg, feats=fe, index=index, index_rate=index_rate)
            outs.append(o[tp: o.numel() - tp])
        out = torch.cat(outs) if len(outs) > 1 else outs[0].contiguous()
        if volume_envelope != 1:  # convert.py:449: both envelopes at the 16 kHz rate (reference quirk)
            ops.change_rms(None, src64, out, self.sample_rate // 2, volume_envelope)
        if self._ws is None:
            self._ws = torch.zeros(4, dtype=torch.int32, device=xp.device)
        ops.peak_normalize(out, self._ws)
        if os.environ.get("RVC_AMD_CHECK"):  # debugging: synchronous check inside the device pass
            self.check_errors()
        return out

    def check_errors(self):
        """Raise if a device-side failure was flagged since the last check: the RMVPE BiGRU's hand-off
        timeout (f0 would be garbage).  ``pipeline()`` calls it after its output copy (one 4-byte read
        behind a sync that happens anyway); HBM-resident callers (``pipeline_device``, ClipGraph replays,
        the bench) call it once after their own synchronisation."""
        if self.rmvpe is not None:
            self.rmvpe.check_error()

    def _index(self, path):
        """Device-resident IVF-Flat index per path (the reference re-reads it every call)."""
        from .retrieval import IVFFlatDevice
        cache = self.__dict__.setdefault("_indexes", {})
        if path not in cache:
            cache[path] = IVFFlatDevice.from_file(path, self.device)
        return cache[path]

    # ------------------------------------------------------------------ reference signature
    def pipeline(self, model, net_g, sid, audio, pitch, f0_method, file_index, index_rate, pitch_guidance,
                 filter_radius, volume_envelope, version, protect, hop_length, f0_autotune, f0_autotune_strength,
                 suffix, embed_suffix, f0_file=None, f0_onnx=False, pbar=None):
        if (f0_method not in ("rmvpe", "pm") and f0_method not in self.CREPE_METHODS) or f0_onnx:
            raise NotImplementedError(f"f0 method {f0_method!r}: rmvpe, crepe-* and pm are on the MI355X path")
        index = None
        if file_index != "" and os.path.exists(file_index) and index_rate != 0:  # convert.py:392-399
            index = self._index(file_index)
        if not pitch_guidance:
            raise NotImplementedError("no-f0 models: the reference's no-f0 Generator is not buildable (SURVEY §0)")
        if suffix != ".pth" or embed_suffix not in (".pt", ".safetensors"):
            raise NotImplementedError("ONNX models are not on the MI355X path")
        if pbar is not None:
            pbar.update(1)
        inp_f0 = read_f0_file(f0_file)
        if pbar is not None:
            pbar.update(1)
        # convert.py:390 keeps the suffix on the VC; here it holds for this call only, so a later pipeline_device /
        # clip-stream call reads the model's own suffix again
        prev, self.embed_suffix = self.embed_suffix, embed_suffix
        try:
            out = self.pipeline_device(model, net_g, int(sid), np.asarray(audio, dtype=np.float32), pitch, version,
                                       protect, index, index_rate, f0_method, bool(f0_autotune), f0_autotune_strength,
                                       inp_f0, volume_envelope)
        finally:
            self.embed_suffix = prev
        if pbar is not None:
            pbar.update(2)
        out = out.cpu().numpy()
        self.check_errors()
        return out


def read_f0_file(f0_file):
    """convert.py:425-436: an object with ``.name`` naming a text file of "time,f0" lines -> f32 [n][2]
    (None when absent, empty or unreadable; the reference logs and carries on)."""
    if not hasattr(f0_file, "name"):
        return None
    try:
        with open(f0_file.name, "r") as f:
            raw = f.read()
        if len(raw) == 0:
            return None
        return np.array([[float(v) for v in line.split(",")] for line in raw.strip("\n").split("\n")],
                        dtype=np.float32)
    except Exception as e:  # noqa: BLE001 -- the reference's bare except + log
        import logging
        logging.getLogger(__name__).error(f"f0 file: {e}")
        return None


def f0_override(inp_f0, x_pad, tf0=100):
    """convert.py:316-318: the f0 file resampled to 100 frames/s by np.interp (f64), written over the
    frames starting at x_pad * tf0.  Returns (values, first frame); the decode kernels clip it to the track."""
    n = np.round((inp_f0[:, 0].max() - inp_f0[:, 0].min()) * tf0 + 1).astype(np.int16)
    rep = np.interp(list(range(n)), inp_f0[:, 0] * 100, inp_f0[:, 1])
    return rep, x_pad * tf0
