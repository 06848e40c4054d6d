"""hipGraph-captured clip loop: ``VC.pipeline_device`` for one fixed clip length, captured once and
replayed per chunk (BASELINE configs[4]: "per-GPU hipGraph-captured chunk loop").

The reference runs one eager ``VC.pipeline`` per chunk (convert.py:129-135, 506-507).  Here the
whole device pass -- filtfilt, RMVPE or CREPE on the side stream, ContentVec, the synthesizer and
the peak normalisation, ~400 kernel launches over two streams -- becomes one graph launch per chunk:
the host issues nothing per kernel, and the side-stream fork/join is captured as graph edges.

Constraints (checked): inputs at most ``t_max`` long (no quiet-point segmentation, which needs the
filtered signal on the host), no f0 file / autotune (their host-side tables are per call).  The
device noise (Philox) is drawn from a seed held in device memory, so each replay draws fresh
noise: ``ClipGraph(...)(audio, seed=s)`` gives the same waveform as the eager path at ``vc.seed = s``.
"""
from __future__ import annotations

import torch

from . import ops


class ClipGraph:
    """``g = ClipGraph(vc, model, net_g, sid, n_samples, ...)``; ``out = g(audio_dev, seed)``.

    ``out`` is a view of the graph's static output buffer, overwritten by the next replay."""

    def __init__(self, vc, model, net_g, sid, n_samples: int, pitch=0, version="v2", protect=0.33, index=None,
                 index_rate=0.0, f0_method="rmvpe", volume_envelope=1.0, warmup: int = 1):
        if n_samples + vc.window > vc.t_max:
            raise ValueError(f"ClipGraph: a {n_samples}-sample clip is segmented on the host (> t_max); "
                             "split it into chunks first")
        self.vc = vc
        dev = torch.device(vc.device)
        self.n = int(n_samples)
        self.inp = torch.zeros(self.n, device=dev)
        self.seed = torch.zeros(1, dtype=torch.int64, device=dev)
        args = (model, net_g, sid, self.inp, pitch, version, protect, index, index_rate, f0_method)
        kw = dict(volume_envelope=volume_envelope)
        seed0, vc.seed = vc.seed, 0  # the captured seed is 0 + the device seed
        prio0, vc.side_priority = getattr(vc, "side_priority", None), 0  # normal-priority fork in graphs
        try:
            self._capture(vc, dev, args, kw, warmup)
        finally:
            vc.seed = seed0
            vc.side_priority = prio0

    def _capture(self, vc, dev, args, kw, warmup):
        # warm up on a side stream (allocator pools, per-stream workspaces, lazily created streams)
        # The graph owns its scratch: every split-K / split-KV / decode workspace its kernels point at
        # lives in self.workspaces for the graph's lifetime, shared with no eager pass or other graph.
        self.workspaces = {}
        # warm-up and capture on a pooled normal-priority stream (no extra stream: the process has 4 hardware
        # queues, pipeline._pooled_stream)
        s = vc._pooled_stream(dev, 0, vc.STREAM_SLOT["front"])
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s), ops.device_seed(self.seed), ops.private_workspaces(self.workspaces):
            for _ in range(max(1, warmup)):
                vc.pipeline_device(*args, **kw)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=s), ops.device_seed(self.seed), ops.private_workspaces(self.workspaces):
            self.out = vc.pipeline_device(*args, **kw)

    def __call__(self, audio: torch.Tensor, seed: int | None = None) -> torch.Tensor:
        if audio.numel() != self.n:
            raise ValueError(f"ClipGraph captured for {self.n} samples, got {audio.numel()}")
        self.inp.copy_(audio.reshape(-1))
        self.seed.fill_(int(self.vc.seed if seed is None else seed))
        self.graph.replay()
        return self.out
