"""Oracle: ContentVec / HuBERT ``extract_features`` on torch-CPU.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Restates the inference
path of ``main/library/architectures/fairseq.py``:
``HubertModel.extract_features`` (:1459) -> ``forward`` (:1412-1431) ->
``ConvFeatureExtractionModel`` (:1165-1195) -> ``TransformerEncoder.extract_features``
(:1102-1141) -> post-LN ``TransformerSentenceEncoderLayer`` (:778-814).

The encoder pads T to a multiple of 2 with a masked key (:1106-1111); a masked
key gets softmax weight exactly 0 and the padded query row is dropped, so this
restatement runs unpadded (verified bitwise identical).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

FE_LAYERS = [(512, 10, 5)] + [(512, 3, 2)] * 4 + [(512, 2, 2)] * 2


def load_weights(ckpt: dict) -> dict:
    """fairseq ``.pt`` dict -> fp32 tensors; pos_conv weight-norm (dim=2) folded (:585-592)."""
    sd = ckpt["model"]
    W = {}
    for k, v in sd.items():
        if k.endswith(".weight_v"):
            base = k[: -len(".weight_v")]
            W[base + ".weight"] = torch._weight_norm(v.float(), sd[base + ".weight_g"].float(), 2)
        elif k.endswith(".weight_g"):
            continue
        elif v.is_floating_point():
            W[k] = v.float()
    return W


def frames(n: int) -> int:
    """Output length of the conv feature extractor for n input samples."""
    for _, k, s in FE_LAYERS:
        n = (n - k) // s + 1
    return n


def feature_extractor(W, source):
    """ConvFeatureExtractionModel.forward (:1191-1195), mode "default"."""
    x = source.unsqueeze(1)
    for i, (c, k, s) in enumerate(FE_LAYERS):
        x = F.conv1d(x, W[f"feature_extractor.conv_layers.{i}.0.weight"], None, s)
        if i == 0:
            x = F.group_norm(x.float(), c, W["feature_extractor.conv_layers.0.2.weight"],
                             W["feature_extractor.conv_layers.0.2.bias"], 1e-5)
        x = F.gelu(x)
    return x


def _layer(W, p, x, n_heads=12):
    """TransformerSentenceEncoderLayer.forward, layer_norm_first=False (:795-803); x [T, C]."""
    T, C = x.shape
    hd = C // n_heads
    q = F.linear(x, W[p + "self_attn.q_proj.weight"], W[p + "self_attn.q_proj.bias"])
    k = F.linear(x, W[p + "self_attn.k_proj.weight"], W[p + "self_attn.k_proj.bias"])
    v = F.linear(x, W[p + "self_attn.v_proj.weight"], W[p + "self_attn.v_proj.bias"])
    q = q.view(T, n_heads, hd).transpose(0, 1) * (hd ** -0.5)
    k = k.view(T, n_heads, hd).transpose(0, 1)
    v = v.view(T, n_heads, hd).transpose(0, 1)
    a = torch.softmax(torch.bmm(q, k.transpose(1, 2)), dim=-1)
    o = torch.bmm(a, v).transpose(0, 1).reshape(T, C)
    o = F.linear(o, W[p + "self_attn.out_proj.weight"], W[p + "self_attn.out_proj.bias"])
    x = F.layer_norm(x + o, (C,), W[p + "self_attn_layer_norm.weight"], W[p + "self_attn_layer_norm.bias"], 1e-5)
    h = F.gelu(F.linear(x, W[p + "fc1.weight"], W[p + "fc1.bias"]).float())
    h = F.linear(h, W[p + "fc2.weight"], W[p + "fc2.bias"])
    return F.layer_norm(x + h, (C,), W[p + "final_layer_norm.weight"], W[p + "final_layer_norm.bias"], 1e-5)


def extract_features(W, source, output_layer=12):
    """HubertModel.extract_features(source [1, N], padding_mask=all False, output_layer) -> [1, T_f, 768]."""
    feats = feature_extractor(W, source)  # [1, 512, T]
    x = F.layer_norm(feats.transpose(1, 2), (512,), W["layer_norm.weight"], W["layer_norm.bias"], 1e-5)
    x = F.linear(x, W["post_extract_proj.weight"], W["post_extract_proj.bias"])  # [1, T, 768]
    pc = F.conv1d(x.transpose(1, 2), W["encoder.pos_conv.0.weight"], W["encoder.pos_conv.0.bias"], 1, 64, 1, 16)
    pc = F.gelu(pc[:, :, :-1])  # SamePad(128) drops one sample
    x = x + pc.transpose(1, 2)
    x = F.layer_norm(x, (768,), W["encoder.layer_norm.weight"], W["encoder.layer_norm.bias"], 1e-5)
    y = x[0]
    for i in range(output_layer):
        y = _layer(W, f"encoder.layers.{i}.", y)
    return y.unsqueeze(0)


def final_proj(W, x):
    return F.linear(x, W["final_proj.weight"], W["final_proj.bias"])


def n_layers(W):
    """Encoder layers in the weight dict (transformers' last_hidden_state runs all of them)."""
    n = 0
    while f"encoder.layers.{n}.fc1.weight" in W:
        n += 1
    return n
