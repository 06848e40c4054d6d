"""One long utterance across ranks (the exchange the utterance sharding of shard.py cannot
do): ``VC.pipeline`` on a single input without ``split_audio``, split over ``world`` GPUs.

The reference computes f0 ONCE over the whole padded utterance (``convert.py:436``), so RMVPE's BiGRU
spans all of it, then converts the quiet-point segments one by one (``convert.py:442-447``).  Here:

  1. every rank filters the input (f64 filtfilt, reflect pad) and rank 0's quiet-point search is
     broadcast (``convert.py:404-412``);
  2. RMVPE's convolutional part is sharded by time: rank r runs the U-Net + cnn head on its 32-aligned
     frame tile plus a ``halo``-frame margin each side (>= the U-Net's receptive field, ~845 frames),
     and keeps the tile's own rows -- the same values as the whole-image pass up to the summation order
     of the smaller grids' split-K;
  3. the exchange: one all_gather of the tiles' 384-row GRU inputs; every rank then runs W_ih, the
     bidirectional GRU over the whole utterance, the classifier and the decode (redundantly: f0 is then
     local everywhere and no broadcast is needed);
  4. the segments are sharded longest-first over the ranks (ContentVec + synthesizer per segment, the
     noise of segment s seeded ``vc.seed + s`` as in the single-rank pass), and the converted pieces are
     gathered to rank 0 (RCCL over xGMI with "nccl"), concatenated in segment order and peak-normalised.

Rank 0 returns the waveform (device f32, identical in layout to ``VC.pipeline_device``), the others None.
The plan helpers (``tile_plan``, ``assemble``) are pure host code, tested over gloo on CPU.
"""
from __future__ import annotations

import torch

from . import ops
from .shard import gather_waveforms, shard_utterances

HALO = 1024  # frames each side; the U-Net's receptive-field radius is ~845 frames
ALIGN = 32   # mel2hidden pads to 32 frames and the encoder pools 5 times by 2: tiles start on 32s


def tile_plan(Tp: int, world: int, halo: int = HALO, align: int = ALIGN):
    """Frame tiles of a Tp-frame image (Tp % align == 0) over ``world`` ranks: per rank
    (a, b, r0, r1) = kept rows [a, b) and computed rows [r0, r1) = [a - halo, b + halo) clipped; all
    boundaries on multiples of ``align``.  Ranks past the last block get empty tiles (a == b)."""
    if Tp % align or halo % align:
        raise ValueError("Tp and halo must be multiples of align")
    blocks = Tp // align
    per, extra = divmod(blocks, world)
    plan, a = [], 0
    for r in range(world):
        b = a + (per + (r < extra)) * align
        plan.append((a, b, max(0, a - halo), min(Tp, b + halo)))
        a = b
    return plan


def assemble(parts, plan, rows: int, Tp: int, like: torch.Tensor):
    """Gathered padded tiles (one [rows][maxlen] per rank) -> the whole [rows][Tp] image of kept rows."""
    out = torch.empty(rows, Tp, dtype=like.dtype, device=like.device)
    for (a, b, _, _), t in zip(plan, parts):
        out[:, a:b] = t[:, : b - a]
    return out


def _coll(dist, t):
    """Tensors for a collective: gloo (CPU tests, ranks sharing one GPU) moves them through host memory."""
    return t.cpu() if dist.get_backend() == "gloo" else t


def exchange_tiles(compute_tile, rows: int, Tp: int, dist, device, halo: int = HALO, dtype=None):
    """The sharded-by-time pass + its exchange: rank r computes rows [r0, r1) with ``compute_tile(r0, r1)``
    -> [rows][r1 - r0], keeps its [a, b), and one all_gather gives every rank the whole [rows][Tp]."""
    rank, world = dist.get_rank(), dist.get_world_size()
    plan = tile_plan(Tp, world, halo)
    a, b, r0, r1 = plan[rank]
    maxlen = max(pb - pa for pa, pb, _, _ in plan)
    tile = compute_tile(r0, r1) if b > a else None
    # every rank must gather one dtype: pass it when a rank may have no tile
    mine = torch.zeros(rows, maxlen, device=device,
                       dtype=dtype or (tile.dtype if tile is not None else torch.float32))
    if tile is not None:
        mine[:, : b - a] = tile[:, a - r0: b - r0]
    mine = _coll(dist, mine)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)  # the exchange
    return assemble(parts, plan, rows, Tp, mine).to(device)


def sharded_f0(vc, xp: torch.Tensor, pitch, dist, halo: int = HALO):
    """Steps 2-3: (coarse int64 [F], pitchf f32 [F]) of the padded signal xp on every rank."""
    rm = vc._rmvpe()
    mel = rm.mel_spectrogram(xp)  # replicated: ~0.1 GFLOP per 10 s
    F = mel.shape[-1]
    img, Tp = rm.mel_image(mel)  # [1][Tp+2][130]

    def unet_tile(r0, r1):
        tile = torch.zeros(1, r1 - r0 + 2, img.shape[-1], device=xp.device, dtype=img.dtype)
        tile[0, 1:-1] = img[0, 1 + r0: 1 + r1]  # interior rows; the tile's own border rows stay zero
        return rm.unet_seq(tile, r1 - r0)

    # 384 x Tp GRU inputs (f64 in the f64 RMVPE: 3 KB per frame)
    seq_all = exchange_tiles(unet_tile, 384, Tp, dist, xp.device, halo, dtype=img.dtype)
    sal = rm.head(seq_all)
    coarse, pitchf, _ = rm.decode(sal, Tp, F, 0.03, float(pitch))
    return coarse, pitchf


def pipeline_sharded(vc, model, net_g, sid, audio, pitch, version, protect, dist, index=None, index_rate=0.0,
                     halo: int = HALO):
    """VC.pipeline_device of ONE utterance over all ranks of ``dist`` (see the module note).  ``audio``:
    the whole 16 kHz input on every rank (device f32 [N] or numpy)."""
    import numpy as np
    rank, world = dist.get_rank(), dist.get_world_size()
    if not torch.is_tensor(audio):
        audio = torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)).to(vc.device)
    N = audio.numel()
    long_input = N + vc.window > vc.t_max
    xp, xp64 = vc.filt(audio.contiguous(), vc.t_pad, want_f64=long_input and rank == 0)
    opt_ts = [ops.quiet_points(xp64[vc.t_pad: vc.t_pad + N], vc.window, vc.t_center, vc.t_query, vc.t_max)] \
        if long_input and rank == 0 else [None]
    if long_input:
        dist.broadcast_object_list(opt_ts, src=0)
    opt_ts = opt_ts[0] or []
    p_len = xp.numel() // vc.window
    coarse, pitchf = sharded_f0(vc, xp, pitch, dist, halo)
    coarse, pitchf = coarse[:p_len], pitchf[:p_len]
    w, tp = vc.window, vc.t_pad_tgt
    segs, s = [], 0  # convert.py:419-447, as VC._pipeline_on_device
    for t in opt_ts:
        t = t // w * w
        segs.append((s, t + vc.t_pad2 + w, s // w, (t + vc.t_pad2) // w))
        s = t
    last = opt_ts[-1] // w * w if opt_ts else None
    segs.append((last or 0, xp.numel(), (last or 0) // w, None))
    mine = shard_utterances([bb - aa for aa, bb, _, _ in segs], world)[rank]
    outs = []
    for si in mine:
        a, b, fa, fb = segs[si]
        feats = vc.features_device(model, xp[a:b], version)
        o = vc.voice_conversion_device(model, net_g, sid, xp[a:b], coarse[fa:fb], pitchf[fa:fb], version, protect,
                                       si, feats=feats, index=index, index_rate=index_rate)
        outs.append(o[tp: o.numel() - tp].contiguous())
    got = gather_waveforms([_coll(dist, o) for o in outs], dist, dst=0)
    if rank != 0:
        return None
    owner = shard_utterances([bb - aa for aa, bb, _, _ in segs], world)
    pieces = [None] * len(segs)
    for r in range(world):
        for si, part in zip(owner[r], got[r]):
            pieces[si] = part.to(xp.device)
    out = torch.cat(pieces) if len(pieces) > 1 else pieces[0].contiguous()
    if vc._ws is None:
        vc._ws = torch.zeros(4, dtype=torch.int32, device=out.device)
    ops.peak_normalize(out, vc._ws)
    return out
