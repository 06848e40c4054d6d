"""MI355X ContentVec / HuBERT feature extractor: drop-in for ``HubertModel.extract_features``
(main/library/architectures/fairseq.py:1459 -> forward :1412-1431), the ``model`` that
``VC.voice_conversion`` calls at convert.py:337-340.

Loaded from a fairseq ``.pt`` dict (``fairseq.py:30-36``); pos_conv weight-norm (dim 2)
folded on the host at load.  Activations stay channels-first [C][T] on the device:

  conv FE   conv1d(1->512, k10 s5) + chnorm_gelu (GroupNorm(512,512) + GELU), 6 x conv1d(k3/k2, s2) + GELU
  proj      layernorm_cf(512) + conv1d(K=1, 512->768)
  encoder   pos_conv (grouped conv k128, SamePad, GELU, +x fused) + LN, then post-LN layers:
            fused QKV conv, flash attention (12 x 64), out_proj, LN(x+y), fc1+GELU, fc2, LN(x+y)

The reference pads T to a multiple of 2 with one masked key (fairseq.py:1106-1111); a masked
key gets softmax weight exactly 0 and the padded row is dropped, so this runs unpadded.
"""
from __future__ import annotations

import torch

from . import ops
from .ops import ACT_GELU, Conv

FE_LAYERS = [(512, 10, 5)] + [(512, 3, 2)] * 4 + [(512, 2, 2)] * 2


def frames(n: int) -> int:
    for _, k, s in FE_LAYERS:
        n = (n - k) // s + 1
    return n


class _FinalProj:
    """``model.final_proj`` as the reference calls it on [1, T, 768] (convert.py:340)."""

    def __init__(self, conv: Conv):
        self.conv = conv

    def __call__(self, x):
        B, T, C = x.shape
        xc = torch.empty(C, T, device=x.device)
        ops.transpose(x.contiguous(), xc, 1, T, C)
        y = self.conv(xc)
        out = torch.empty(1, T, y.shape[0], device=x.device)
        ops.transpose(y, out, 1, y.shape[0], T)
        return out


class ContentVecAMD:
    def __init__(self, ckpt: dict, device: str = "cuda"):
        cfg = ckpt["cfg"]["model"]
        if cfg.get("extractor_mode", "default") != "default" or cfg.get("layer_norm_first", False):
            raise NotImplementedError("ContentVec/HuBERT-base layout only (extractor 'default', post-LN)")
        sd = ckpt["model"]
        W = {}
        for k, v in sd.items():
            if k.endswith(".weight_v"):
                base = k[: -len(".weight_v")]
                W[base + ".weight"] = torch._weight_norm(v.float(), sd[base + ".weight_g"].float(), 2)
            elif not k.endswith(".weight_g") and v.is_floating_point():
                W[k] = v.float()
        dev = device
        self.E = cfg.get("encoder_embed_dim", 768)
        self.heads = cfg.get("encoder_attention_heads", 12)
        self.fe = [Conv(W[f"feature_extractor.conv_layers.{i}.0.weight"], None, device=dev) for i in range(7)]
        self.gn = (W["feature_extractor.conv_layers.0.2.weight"].to(dev), W["feature_extractor.conv_layers.0.2.bias"].to(dev))
        self.ln = (W["layer_norm.weight"].to(dev), W["layer_norm.bias"].to(dev))
        self.proj = Conv(W["post_extract_proj.weight"].unsqueeze(-1), W["post_extract_proj.bias"], device=dev)
        self.pos_conv = Conv(W["encoder.pos_conv.0.weight"], W["encoder.pos_conv.0.bias"], groups=cfg.get("conv_pos_groups", 16),
                             device=dev)
        self.pos_k = self.pos_conv.K
        self.enc_ln = (W["encoder.layer_norm.weight"].to(dev), W["encoder.layer_norm.bias"].to(dev))
        self.layers = []
        i = 0
        while f"encoder.layers.{i}.fc1.weight" in W:
            p = f"encoder.layers.{i}."
            wqkv = torch.cat([W[p + f"self_attn.{n}_proj.weight"] for n in "qkv"], 0).unsqueeze(-1)
            bqkv = torch.cat([W[p + f"self_attn.{n}_proj.bias"] for n in "qkv"], 0)
            self.layers.append(dict(
                qkv=Conv(wqkv, bqkv, device=dev),
                o=Conv(W[p + "self_attn.out_proj.weight"].unsqueeze(-1), W[p + "self_attn.out_proj.bias"], device=dev),
                ln1=(W[p + "self_attn_layer_norm.weight"].to(dev), W[p + "self_attn_layer_norm.bias"].to(dev)),
                fc1=Conv(W[p + "fc1.weight"].unsqueeze(-1), W[p + "fc1.bias"], device=dev),
                fc2=Conv(W[p + "fc2.weight"].unsqueeze(-1), W[p + "fc2.bias"], device=dev),
                ln2=(W[p + "final_layer_norm.weight"].to(dev), W[p + "final_layer_norm.bias"].to(dev)),
            ))
            i += 1
        self.final_proj = _FinalProj(Conv(W["final_proj.weight"].unsqueeze(-1), W["final_proj.bias"], device=dev))
        self.device = dev

    def features_cf(self, wav: torch.Tensor, output_layer: int = 12) -> torch.Tensor:
        """wav: device f32 [N] (16 kHz) -> encoder output after ``output_layer`` layers, [768][T_f];
        or B equal-length signals [B][N] -> [B][768][T_f] (every conv / norm / attention batched)."""
        dev = wav.device
        batched = wav.dim() == 2
        B, N = (wav.shape[0], wav.shape[1]) if batched else (1, wav.numel())
        x = wav.reshape(B, 1, N) if batched else wav.view(1, N)
        for i, (c, k, s) in enumerate(FE_LAYERS):
            if i == 0:
                x = self.fe[0](x, stride=s)
                ops.chnorm_gelu(x, self.gn[0], self.gn[1], x, B, c, x.shape[-1])
            else:
                x = self.fe[i](x, stride=s, out_act=ACT_GELU)
        T = x.shape[-1]
        ops.layernorm_cf(x, None, self.ln[0], self.ln[1], x, B, 512, T)
        x = self.proj(x)  # [(B)][768][T]
        E = self.E
        bs = (B,) if batched else ()
        x2 = torch.empty(*bs, E, T, device=dev)
        self.pos_conv(x, pad=self.pos_k // 2, Lout=T, out=x2, out_act=ACT_GELU, res=x)  # SamePad drops the last col
        x = x2
        ops.layernorm_cf(x, None, self.enc_ln[0], self.enc_ln[1], x, B, E, T)
        H = self.heads
        D = E // H
        o = torch.empty(*bs, E, T, device=dev)
        y = torch.empty(*bs, E, T, device=dev)
        for L in self.layers[:output_layer]:
            qkv = L["qkv"](x)
            k, v = (qkv[:, E:], qkv[:, 2 * E:]) if batched else (qkv[E:], qkv[2 * E:])
            ops.attention(qkv, k, v, o, B=B, H=H, D=D, T=T, ldc=T, q_hs=D * T, k_hs=D * T, v_hs=D * T,
                          o_hs=D * T, scale=D ** -0.5, q_bs=3 * E * T, k_bs=3 * E * T, v_bs=3 * E * T, o_bs=E * T)
            L["o"](o, out=y)
            ops.layernorm_cf(x, y, L["ln1"][0], L["ln1"][1], x, B, E, T)
            h = L["fc1"](x, out_act=ACT_GELU)
            L["fc2"](h, out=y)
            ops.layernorm_cf(x, y, L["ln2"][0], L["ln2"][1], x, B, E, T)
        return x

    # ------------------------------------------------------------------ reference API
    def extract_features(self, source, padding_mask=None, mask=False, ret_conv=False, output_layer=None):
        """fairseq.py:1459: source [1, N] -> (x [1, T_f, 768], padding_mask [1, T_f])."""
        if source.shape[0] != 1:
            raise NotImplementedError("batch 1 (as VC.voice_conversion calls it)")
        if padding_mask is not None and bool(padding_mask.any()):
            raise NotImplementedError("padded sources are not on the hot path (VC passes an all-False mask)")
        xc = self.features_cf(source.reshape(-1).float().contiguous(), output_layer or len(self.layers))
        E, T = xc.shape
        out = torch.empty(1, T, E, device=xc.device)
        ops.transpose(xc, out, 1, E, T)
        pm = torch.zeros(1, T, dtype=torch.bool, device=xc.device)
        return out, pm

    def to(self, *a, **k):
        return self

    def float(self):
        return self

    def eval(self):
        return self
