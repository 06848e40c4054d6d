"""MI355X ContentVec / HuBERT feature extractor: drop-in for ``HubertModel.extract_features``
(main/library/architectures/fairseq.py:1459 -> forward :1412-1431), the ``model`` that
``VC.voice_conversion`` calls at convert.py:337-340.

Loaded from a fairseq ``.pt`` dict (``fairseq.py:30-36``), or (``from_transformers``) from the transformers
layout the reference loads for a ``.safetensors`` embedder (``HubertModelWithFinalProj.from_pretrained``,
main/library/utils.py:157-165: config.json + model.safetensors); pos_conv weight-norm (dim 2) folded on the
host at load.  The two layouts are the same network; the embed suffix only changes which layer feeds
final_proj (``embed_cf``, convert.py:337-345).  Activations stay channels-first [C][T] on the device:

  conv FE   fe0_gn_gelu (conv1d(1->512, k10 s5) + GroupNorm(512,512) + GELU fused), 6 x conv1d(k3/k2, s2) + GELU
  proj      layernorm_cf(512) + conv1d(K=1, 512->768)
  encoder   pos_conv (grouped conv k128, SamePad, GELU, +x fused) + LN, then post-LN layers:
            fused QKV conv, flash attention (12 x 64), out_proj, LN(x+y), fc1+GELU, fc2, LN(x+y)

The reference pads T to a multiple of 2 with one masked key (fairseq.py:1106-1111); a masked
key gets softmax weight exactly 0 and the padded row is dropped, so this runs unpadded.
"""
from __future__ import annotations

import os

import torch

from . import ops
from .ops import ACT_GELU, Conv

# ContentVec's K = 1 GEMMs take their split-fp16 scale from the producers' published |max| (LayerNorm, attention, fc1);
# RVC_AMD_CV_AMAX=0: the 6-pass split-bf16 arithmetic of round 4
CV_AMAX = os.environ.get("RVC_AMD_CV_AMAX", "1") != "0"
# round 6: the feature extractor's convs publish and read cells too (layer 0's fused GELU output, then each stride-2
# conv + GELU), so layers 1-6 run split-fp16; RVC_AMD_FE_AMAX=0: 6-pass split-bf16 there (the round-5 form)
FE_AMAX = os.environ.get("RVC_AMD_FE_AMAX", "1") != "0"
# round 6: the attention's two products in split-fp16 from the QKV projection's published |max| (RVC_AMD_ATTN_F16=0:
# the f32-MFMA kernel; synth.py and both native hosts read the same switch)
ATTN_F16 = os.environ.get("RVC_AMD_ATTN_F16", "1") != "0"

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


# transformers HubertModel parameter names -> fairseq's (the layout ContentVecAMD is built from); the weight-norm
# pair is "parametrizations.weight.original0 / 1" (torch.nn.utils.parametrizations) or "weight_g / weight_v"
_HF_TOP = {"masked_spec_embed": "mask_emb",
           "feature_extractor.conv_layers.0.layer_norm.weight": "feature_extractor.conv_layers.0.2.weight",
           "feature_extractor.conv_layers.0.layer_norm.bias": "feature_extractor.conv_layers.0.2.bias",
           "feature_projection.layer_norm.weight": "layer_norm.weight",
           "feature_projection.layer_norm.bias": "layer_norm.bias",
           "feature_projection.projection.weight": "post_extract_proj.weight",
           "feature_projection.projection.bias": "post_extract_proj.bias",
           "encoder.pos_conv_embed.conv.bias": "encoder.pos_conv.0.bias",
           "encoder.pos_conv_embed.conv.parametrizations.weight.original0": "encoder.pos_conv.0.weight_g",
           "encoder.pos_conv_embed.conv.parametrizations.weight.original1": "encoder.pos_conv.0.weight_v",
           "encoder.pos_conv_embed.conv.weight_g": "encoder.pos_conv.0.weight_g",
           "encoder.pos_conv_embed.conv.weight_v": "encoder.pos_conv.0.weight_v",
           "encoder.layer_norm.weight": "encoder.layer_norm.weight", "encoder.layer_norm.bias": "encoder.layer_norm.bias",
           "final_proj.weight": "final_proj.weight", "final_proj.bias": "final_proj.bias"}
_HF_LAYER = {"attention.q_proj": "self_attn.q_proj", "attention.k_proj": "self_attn.k_proj",
             "attention.v_proj": "self_attn.v_proj", "attention.out_proj": "self_attn.out_proj",
             "layer_norm": "self_attn_layer_norm", "feed_forward.intermediate_dense": "fc1",
             "feed_forward.output_dense": "fc2", "final_layer_norm": "final_layer_norm"}


def hf_to_fairseq(sd: dict) -> dict:
    """A transformers ``HubertModel(WithFinalProj)`` state dict under fairseq's names; raises on a key this
    network does not have (a different architecture must not load silently)."""
    import re
    out = {}
    for k, v in sd.items():
        k2 = k[len("hubert."):] if k.startswith("hubert.") else k
        if k2 in _HF_TOP:
            out[_HF_TOP[k2]] = v
            continue
        m = re.fullmatch(r"feature_extractor\.conv_layers\.(\d+)\.conv\.weight", k2)
        if m:
            out[f"feature_extractor.conv_layers.{m.group(1)}.0.weight"] = v
            continue
        m = re.fullmatch(r"encoder\.layers\.(\d+)\.(.+)\.(weight|bias)", k2)
        if m and m.group(2) in _HF_LAYER:
            out[f"encoder.layers.{m.group(1)}.{_HF_LAYER[m.group(2)]}.{m.group(3)}"] = v
            continue
        raise ValueError(f"ContentVecAMD.from_transformers: unexpected parameter {k!r}")
    return out


def hf_config_to_fairseq(c: dict) -> dict:
    """The transformers HubertConfig fields this build runs -> fairseq cfg["model"]; NotImplementedError for
    another layout (stable layer norm, layer-normed extractor, other conv stacks or activations)."""
    want = dict(feat_extract_norm="group", do_stable_layer_norm=False, conv_bias=False, hidden_act="gelu",
                feat_extract_activation="gelu", conv_dim=[512] * 7, conv_stride=[5, 2, 2, 2, 2, 2, 2],
                conv_kernel=[10, 3, 3, 3, 3, 2, 2], num_conv_pos_embeddings=128)
    for k, v in want.items():
        got = c.get(k, v)
        if (list(got) if isinstance(got, (list, tuple)) else got) != v:
            raise NotImplementedError(f"transformers HuBERT with {k}={got!r}: ContentVec/HuBERT-base layout only")
    if c.get("feat_proj_layer_norm", True) is not True or abs(c.get("layer_norm_eps", 1e-5) - 1e-5) > 1e-12:
        raise NotImplementedError("transformers HuBERT: feat_proj_layer_norm with eps 1e-5 only")
    return dict(extractor_mode="default", layer_norm_first=False, encoder_embed_dim=c.get("hidden_size", 768),
                encoder_attention_heads=c.get("num_attention_heads", 12),
                conv_pos_groups=c.get("num_conv_pos_embedding_groups", 16))


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
        self.embed_suffix = ".pt"

    @classmethod
    def from_transformers(cls, path: str, device: str = "cuda") -> "ContentVecAMD":
        """``HubertModelWithFinalProj.from_pretrained(path)`` (main/library/utils.py:157-165) without transformers:
        ``path`` is the model directory (config.json + model.safetensors, or the shards that
        model.safetensors.index.json lists, as from_pretrained reads them) or a .safetensors file with config.json
        beside it.  A tensor named by two files raises."""
        import json
        import os
        from safetensors.torch import load_file
        d = path if os.path.isdir(path) else os.path.dirname(path)
        if not os.path.isdir(path):
            files = [path]
        elif os.path.exists(os.path.join(d, "model.safetensors")):
            files = [os.path.join(d, "model.safetensors")]
        elif os.path.exists(os.path.join(d, "model.safetensors.index.json")):
            with open(os.path.join(d, "model.safetensors.index.json")) as f:
                files = [os.path.join(d, fn) for fn in sorted(set(json.load(f)["weight_map"].values()))]
        else:
            raise FileNotFoundError(f"no model.safetensors or model.safetensors.index.json under {path}")
        with open(os.path.join(d, "config.json")) as f:
            cfg = json.load(f)
        sd = {}
        for fn in files:
            part = load_file(fn)
            dup = sd.keys() & part.keys()
            if dup:
                raise ValueError(f"{fn}: tensors {sorted(dup)[:4]} already loaded from another file")
            sd.update(part)
        m = cls({"cfg": {"model": hf_config_to_fairseq(cfg)}, "model": hf_to_fairseq(sd)}, device)
        m.embed_suffix = ".safetensors"
        return m

    def embed_cf(self, wav: torch.Tensor, version: str, embed_suffix: str | None = None) -> torch.Tensor:
        """The features VC.voice_conversion takes from the embedder (convert.py:337-345), channels-first:
        ".pt" (fairseq extract_features): layer 9 + final_proj for v1, layer 12 for v2; ".safetensors"
        (transformers, ``model(feats)["last_hidden_state"]``): the last layer, + final_proj for v1."""
        suffix = embed_suffix or self.embed_suffix
        if suffix == ".safetensors":
            feats = self.features_cf(wav, len(self.layers))
        elif suffix == ".pt":
            feats = self.features_cf(wav, 9 if version == "v1" else 12)
        else:
            raise NotImplementedError(f"embedder {suffix!r}: .pt and .safetensors are on the MI355X path")
        return self.final_proj.conv(feats) if version == "v1" else feats

    def __call__(self, feats: torch.Tensor) -> dict:
        """The transformers forward as convert.py:343 calls it: feats [1, N] -> {"last_hidden_state": [1, T_f, 768]}."""
        xc = self.features_cf(feats.reshape(-1).float().contiguous(), len(self.layers))
        E, T = xc.shape
        out = torch.empty(1, T, E, device=xc.device)
        ops.transpose(xc, out, 1, E, T)
        return {"last_hidden_state": out}

    def features_cf(self, wav: torch.Tensor, output_layer: int = 12) -> torch.Tensor:
        """wav: device f32 [N] (16 kHz) -> encoder output after ``output_layer`` layers, [768][T_f];
        or B equal-length signals [B][N] -> [B][768][T_f] (every conv / norm / attention batched)."""
        dev = wav.device
        batched = wav.dim() == 2
        B, N = (wav.shape[0], wav.shape[1]) if batched else (1, wav.numel())
        x = wav.reshape(B, 1, N) if batched else wav.view(1, N)
        # |max| cells (CV_AMAX): every LayerNorm, attention and fc1 publishes its output's |max| and the K = 1 GEMM that
        # reads it runs split-fp16 from that scale (ops.conv_passes), no pre-pass; so do the feature extractor's layers
        # 0-5 (round 6): layers 1-6 (stride 2) run split-fp16 from their input's cell (cells 2 + 4 nl + i)
        nl = min(output_layer, len(self.layers))
        nfe = len(FE_LAYERS) - 1
        # ... and (round 6) each layer's QKV projection publishes max |q|, |k|, |v| (cells 2 + 4 nl + nfe + i): the
        # attention runs split-fp16 from it (ops.attention amax_in)
        cells = ops.AmaxSlots(2 + 5 * nl + nfe, dev, B) if CV_AMAX else None
        cell = (lambda k: cells[k]) if CV_AMAX else (lambda k: None)
        fe_cell = (lambda i: cells[2 + 4 * nl + i]) if CV_AMAX and FE_AMAX else (lambda i: None)
        for i, (c, k, s) in enumerate(FE_LAYERS):
            if i == 0:  # conv + GroupNorm + GELU in one pass over the signal (rvc_fe0_gn_gelu)
                x = ops.fe0_gn_gelu(wav.contiguous(), self.fe[0].w, self.gn[0], self.gn[1], B, N, c, k, s,
                                    amax_out=fe_cell(0))
            else:
                x = self.fe[i](x, stride=s, out_act=ACT_GELU, amax_in=fe_cell(i - 1),
                               amax_out=fe_cell(i) if i < nfe else None)
        T = x.shape[-1]
        ops.layernorm_cf(x, None, self.ln[0], self.ln[1], x, B, 512, T, amax_out=cell(0))
        x = self.proj(x, amax_in=cell(0))  # [(B)][768][T]
        E = self.E
        bs = (B,) if batched else ()
        x2 = torch.empty(*bs, E, T, device=dev)
        self.pos_conv(x, pad=self.pos_k // 2, Lout=T, out=x2, out_act=ACT_GELU, res=x)  # SamePad drops the last col
        x = x2
        ops.layernorm_cf(x, None, self.enc_ln[0], self.enc_ln[1], x, B, E, T, amax_out=cell(1))
        H = self.heads
        D = E // H
        o = torch.empty(*bs, E, T, device=dev)
        y = torch.empty(*bs, E, T, device=dev)
        for i, L in enumerate(self.layers[:output_layer]):
            # layer i reads cell 4 i + 1 (the encoder LayerNorm's, then the previous layer's ln2) and fills 4 i + 2 .. 5
            c_in, c_at, c_l1, c_f1, c_l2 = (cell(4 * i + 1), cell(4 * i + 2), cell(4 * i + 3), cell(4 * i + 4),
                                            cell(4 * i + 5))
            c_qkv = cell(2 + 4 * nl + nfe + i) if ATTN_F16 else None
            qkv = L["qkv"](x, amax_in=c_in, amax_out=c_qkv)
            k, v = (qkv[:, E:], qkv[:, 2 * E:]) if batched else (qkv[E:], qkv[2 * E:])
            ops.attention(qkv, k, v, o, B=B, H=H, D=D, T=T, ldc=T, q_hs=D * T, k_hs=D * T, v_hs=D * T,
                          o_hs=D * T, scale=D ** -0.5, q_bs=3 * E * T, k_bs=3 * E * T, v_bs=3 * E * T, o_bs=E * T,
                          amax_out=c_at, amax_in=c_qkv)
            L["o"](o, out=y, amax_in=c_at)
            ops.layernorm_cf(x, y, L["ln1"][0], L["ln1"][1], x, B, E, T, amax_out=c_l1)
            h = L["fc1"](x, out_act=ACT_GELU, amax_in=c_l1, amax_out=c_f1)
            L["fc2"](h, out=y, amax_in=c_f1)
            ops.layernorm_cf(x, y, L["ln2"][0], L["ln2"][1], x, B, E, T, amax_out=c_l2)
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
