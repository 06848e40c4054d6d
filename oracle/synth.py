"""Oracle: ``Synthesizer.infer`` (TextEncoder -> flow^-1 -> NSF-HiFiGAN) on torch-CPU.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates
``main/library/algorithm/synthesizers.py``, ``residuals.py``, ``modules.py`` and
``commons.py`` functionally, over a plain dict of fp32 tensors.  Noise is an
explicit input (three RNG draws per call).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

LRELU_SLOPE = 0.1  # residuals.py:14


def load_weights(ckpt_weight: dict) -> dict:
    """fp16 ckpt tensors -> fp32, weight-norm folded the way torch's parametrization
    computes it (``torch._weight_norm(v, g, dim)``), as ``Synthesizer.load_state_dict``
    + ``.float()`` does at ``convert.py:564-569``."""
    W = {}
    for k, v in ckpt_weight.items():
        if k.endswith(".weight_v"):
            base = k[: -len(".weight_v")]
            g = ckpt_weight[base + ".weight_g"].float()
            W[base + ".weight"] = torch._weight_norm(v.float(), g, 0)
        elif k.endswith(".weight_g"):
            continue
        else:
            W[k] = v.float()
    return W


def _conv(W, name, x, stride=1, padding=0, dilation=1, bias=True):
    return F.conv1d(x, W[name + ".weight"], W.get(name + ".bias") if bias else None, stride, padding, dilation)


def sequence_mask(length, max_length):
    """commons.py:43-46"""
    return torch.arange(max_length, dtype=length.dtype).unsqueeze(0) < length.unsqueeze(1)


def _layer_norm(x, gamma, beta, eps=1e-5):
    """synthesizers.py:170-181 (channels-first LayerNorm)."""
    x = x.transpose(1, -1)
    return F.layer_norm(x, (x.size(-1),), gamma, beta, eps).transpose(1, -1)


def _mha(W, p, x, attn_mask, n_heads, window=10):
    """synthesizers.py:221-251: rel-pos MHA (heads_share, window 10).  The relative
    terms are only non-zero inside |j-i| <= window (zero-padded embeddings,
    synthesizers.py:259-269), so they are added on that band directly."""
    q = _conv(W, p + "conv_q", x)
    k = _conv(W, p + "conv_k", x)
    v = _conv(W, p + "conv_v", x)
    b, d, t = k.shape
    kc = d // n_heads
    qh = q.view(b, n_heads, kc, t).transpose(2, 3) / math.sqrt(kc)  # [b,h,t,kc]
    kh = k.view(b, n_heads, kc, t).transpose(2, 3)
    vh = v.view(b, n_heads, kc, t).transpose(2, 3)
    scores = torch.matmul(qh, kh.transpose(-2, -1))
    ek = W[p + "emb_rel_k"][0]  # [2w+1, kc]
    ev = W[p + "emb_rel_v"][0]
    rel = torch.matmul(qh, ek.t())  # [b,h,t,2w+1]
    idx_i = torch.arange(t)
    for r in range(2 * window + 1):
        off = r - window
        lo, hi = max(0, -off), min(t, t - off)
        if hi > lo:
            ii = idx_i[lo:hi]
            scores[:, :, ii, ii + off] += rel[:, :, ii, r]
    scores = scores.masked_fill(attn_mask == 0, -1e4)
    p_attn = F.softmax(scores, dim=-1)
    out = torch.matmul(p_attn, vh)
    band = torch.zeros(b, n_heads, t, 2 * window + 1)
    for r in range(2 * window + 1):
        off = r - window
        lo, hi = max(0, -off), min(t, t - off)
        if hi > lo:
            ii = idx_i[lo:hi]
            band[:, :, ii, r] = p_attn[:, :, ii, ii + off]
    out = out + torch.matmul(band, ev)
    out = out.transpose(2, 3).contiguous().view(b, d, t)
    return _conv(W, p + "conv_o", out)


def _ffn(W, p, x, x_mask, k=3):
    """synthesizers.py:302-315 (same padding, ReLU)."""
    pl, pr = (k - 1) // 2, k // 2
    x = F.conv1d(F.pad(x * x_mask, (pl, pr)), W[p + "conv_1.weight"], W[p + "conv_1.bias"])
    x = torch.relu(x) * x_mask
    x = F.conv1d(F.pad(x, (pl, pr)), W[p + "conv_2.weight"], W[p + "conv_2.bias"])
    return x * x_mask


def text_encoder(W, cfg, phone, pitch, lengths):
    """synthesizers.py:366-371 + Encoder.forward 340-348."""
    hidden, n_heads, n_layers, ksz = cfg[3], cfg[5], cfg[6], cfg[7]
    x = F.linear(phone, W["enc_p.emb_phone.weight"], W["enc_p.emb_phone.bias"])
    if pitch is not None:
        x = x + F.embedding(pitch, W["enc_p.emb_pitch.weight"])
    x = F.leaky_relu(x * math.sqrt(hidden), 0.1)
    x = torch.transpose(x, 1, -1)
    x_mask = torch.unsqueeze(sequence_mask(lengths, x.size(2)), 1).to(x.dtype)
    attn_mask = x_mask.unsqueeze(2) * x_mask.unsqueeze(-1)
    x = x * x_mask
    x = x * x_mask
    for i in range(n_layers):
        y = _mha(W, f"enc_p.encoder.attn_layers.{i}.", x, attn_mask, n_heads)
        x = _layer_norm(x + y, W[f"enc_p.encoder.norm_layers_1.{i}.gamma"], W[f"enc_p.encoder.norm_layers_1.{i}.beta"])
        y = _ffn(W, f"enc_p.encoder.ffn_layers.{i}.", x, x_mask, ksz)
        x = _layer_norm(x + y, W[f"enc_p.encoder.norm_layers_2.{i}.gamma"], W[f"enc_p.encoder.norm_layers_2.{i}.beta"])
    x = x * x_mask
    stats = _conv(W, "enc_p.proj", x) * x_mask
    m, logs = torch.split(stats, cfg[2], dim=1)
    return m, logs, x_mask


def _wavenet(W, p, x, x_mask, g, hidden, n_layers=3, k=5):
    """modules.py:35-51 with commons.py:35-41 fused gate."""
    output = torch.zeros_like(x)
    gc = _conv(W, p + "cond_layer", g)
    for i in range(n_layers):
        x_in = _conv(W, p + f"in_layers.{i}", x, padding=(k - 1) // 2)
        g_l = gc[:, i * 2 * hidden:(i + 1) * 2 * hidden, :]
        in_act = x_in + g_l
        acts = torch.tanh(in_act[:, :hidden, :]) * torch.sigmoid(in_act[:, hidden:, :])
        rs = _conv(W, p + f"res_skip_layers.{i}", acts)
        if i < n_layers - 1:
            x = (x + rs[:, :hidden, :]) * x_mask
            output = output + rs[:, hidden:, :]
        else:
            output = output + rs
    return output * x_mask


def flow_reverse(W, cfg, z_p, x_mask, g):
    """residuals.py:87-95 (reverse) + ResidualCouplingLayer 127-137 (mean_only)."""
    hidden = cfg[3]
    half = cfg[2] // 2
    x = z_p
    for f in reversed(range(4)):
        x = torch.flip(x, [1])
        p = f"flow.flows.{2 * f}."
        x0, x1 = torch.split(x, [half, half], 1)
        h = _conv(W, p + "pre", x0) * x_mask
        h = _wavenet(W, p + "enc.", h, x_mask, g, hidden)
        m = _conv(W, p + "post", h) * x_mask
        logs = torch.zeros_like(m)
        x1 = (x1 - m) * torch.exp(-logs) * x_mask
        x = torch.cat([x0, x1], 1)
    return x


def sine_source(W, f0, upp, sr, sine_noise, rand_ini=None):
    """SineGen + SourceModuleHnNSF (synthesizers.py:69-112), harmonic_num = 0.

    f0: [1, T] f32; sine_noise: [1, T*upp, 1] (the ``randn_like`` draw);
    rand_ini is zeroed for dim 0 by the reference, so it never contributes.
    Returns har_source [1, 1, T*upp]."""
    sine_amp, noise_std = 0.1, 0.003
    f0 = f0.unsqueeze(-1)
    rad = f0 / sr * torch.arange(1, upp + 1, dtype=f0.dtype)
    rad = rad + F.pad((torch.fmod(rad[:, :-1, -1:].float() + 0.5, 1.0) - 0.5).cumsum(dim=1).fmod(1.0).to(f0),
                      (0, 0, 1, 0), mode="constant")
    rad = rad.reshape(f0.shape[0], -1, 1)
    sine = torch.sin(2 * np.pi * rad) * sine_amp
    uv = torch.ones_like(f0) * (f0 > 0)
    uv = F.interpolate(uv.transpose(2, 1), scale_factor=float(upp), mode="nearest").transpose(2, 1)
    sine = sine * uv + ((uv * noise_std + (1 - uv) * sine_amp / 3) * sine_noise)
    har = torch.tanh(F.linear(sine, W["dec.m_source.l_linear.weight"], W["dec.m_source.l_linear.bias"]))
    return har.transpose(1, 2)


def _resblock(W, p, x, k, dilations):
    """residuals.py:32-36 (x_mask None)."""
    for m, d in enumerate(dilations):
        xt = F.leaky_relu(x, LRELU_SLOPE)
        xt = _conv(W, p + f"convs1.{m}", xt, padding=(k * d - d) // 2, dilation=d)
        xt = F.leaky_relu(xt, LRELU_SLOPE)
        xt = _conv(W, p + f"convs2.{m}", xt, padding=(k - 1) // 2)
        x = xt + x
    return x


def generator(W, cfg, x, f0, g, sine_noise):
    """GeneratorNSF.forward (synthesizers.py:144-161)."""
    rks, rds, ur, uic, uks, sr = cfg[10], cfg[11], cfg[12], cfg[13], cfg[14], cfg[17]
    upp = math.prod(ur)
    nk = len(rks)
    har = sine_source(W, f0, upp, sr, sine_noise)
    x = _conv(W, "dec.conv_pre", x, padding=3)
    x = x + _conv(W, "dec.cond", g)
    nup = len(ur)
    strides = [math.prod(ur[i + 1:]) if i + 1 < nup else 1 for i in range(nup)]
    for i, (u, k) in enumerate(zip(ur, uks)):
        x = F.leaky_relu(x, LRELU_SLOPE)
        pad = ((k - u) // 2) if u % 2 == 0 else (u // 2 + u % 2)
        x = F.conv_transpose1d(x, W[f"dec.ups.{i}.weight"], W[f"dec.ups.{i}.bias"], u, pad, u % 2)
        s = strides[i]
        kn = 1 if s == 1 else s * 2 - s % 2
        x = x + _conv(W, f"dec.noise_convs.{i}", har, stride=s, padding=0 if s == 1 else (kn - s) // 2)
        xs = 0
        for j in range(nk):
            xs = xs + _resblock(W, f"dec.resblocks.{i * nk + j}.", x, rks[j], rds[j])
        x = xs / nk
    x = F.leaky_relu(x)
    return torch.tanh(F.conv1d(x, W["dec.conv_post.weight"], None, 1, 3))


def infer(W, cfg, phone, phone_lengths, pitch, nsff0, sid, z_noise, sine_noise):
    """Synthesizer.infer (synthesizers.py:446-465) with injected noise.

    z_noise [1, inter, T] replaces ``randn_like(m_p)``; sine_noise [1, T*upp, 1]
    replaces SineGen's ``randn_like``.  Returns (o, x_mask, (z, z_p, m_p, logs_p))."""
    g = F.embedding(sid, W["emb_g.weight"]).unsqueeze(-1)
    m_p, logs_p, x_mask = text_encoder(W, cfg, phone, pitch, phone_lengths)
    z_p = (m_p + torch.exp(logs_p) * z_noise * 0.66666) * x_mask
    z = flow_reverse(W, cfg, z_p, x_mask, g)
    o = generator(W, cfg, z * x_mask, nsff0, g, sine_noise)
    return o, x_mask, (z, z_p, m_p, logs_p)
