"""Deterministic synthetic checkpoints and audio for the VC hot path.

No pretrained weights exist offline, so every test and the bench
use true-shape weights generated here from a seed.  The generator writes the
three checkpoint layouts the reference loads:

* voice model ``.pth``  -- ``{"weight": {k: fp16}, "config": [18 items], "f0",
  "version", "vocoder", "sr", ...}`` exactly as
  ``main/inference/train.py:729-742`` saves it (weight-norm stored as
  ``.weight_g`` / ``.weight_v``, ``enc_q`` dropped);
* embedder ``.pt``     -- fairseq ``{"cfg": {"model": HubertConfig kwargs,
  "task": {}}, "model": state_dict}`` read by
  ``main/library/architectures/fairseq.py:30-36``;
* ``rmvpe.pt``         -- a plain ``E2E(4, 1, (2, 2))`` state dict
  (``main/library/predictors/RMVPE.py:196-198``).

Values come from numpy's PCG64 so the same seed gives the same bytes on this
container and on the GPU box.  Scales are chosen so activations stay O(1)
through every stage (the reference's own init zeroes the flow's ``post`` conv,
which would make the flow an identity and hide it from parity tests).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch

# main/configs/v{1,2}/{32000,40000,48000}.json ("model" + "data" sections).
_SR_TABLE = {
    32000: dict(filter_length=1024, v1=dict(upsample_rates=[10, 4, 2, 2, 2], upsample_kernel_sizes=[16, 16, 4, 4, 4]),
                v2=dict(upsample_rates=[10, 8, 2, 2], upsample_kernel_sizes=[20, 16, 4, 4])),
    40000: dict(filter_length=2048, v1=dict(upsample_rates=[10, 10, 2, 2], upsample_kernel_sizes=[16, 16, 4, 4]),
                v2=dict(upsample_rates=[10, 10, 2, 2], upsample_kernel_sizes=[16, 16, 4, 4])),
    48000: dict(filter_length=2048, v1=dict(upsample_rates=[10, 6, 2, 2, 2], upsample_kernel_sizes=[16, 16, 4, 4, 4]),
                v2=dict(upsample_rates=[12, 10, 2, 2], upsample_kernel_sizes=[24, 20, 4, 4])),
}


def synth_config(sr: int = 48000, version: str = "v2", spk_embed_dim: int = 109) -> list:
    """The 18-item ``cpt["config"]`` list (``train.py:730``)."""
    t = _SR_TABLE[sr]
    v = t[version]
    return [t["filter_length"] // 2 + 1, 32, 192, 192, 768, 2, 6, 3, 0, "1", [3, 7, 11],
            [[1, 3, 5], [1, 3, 5], [1, 3, 5]], list(v["upsample_rates"]), 512,
            list(v["upsample_kernel_sizes"]), spk_embed_dim, 256, sr]


class _Gen:
    def __init__(self, seed: int):
        self.rng = np.random.Generator(np.random.PCG64(seed))

    def normal(self, shape, std):
        return torch.from_numpy((self.rng.standard_normal(size=shape) * std).astype(np.float32))

    def uniform(self, shape, lo, hi):
        return torch.from_numpy(self.rng.uniform(lo, hi, size=shape).astype(np.float32))


def _wn(g: _Gen, sd, name, shape, std, dim=0):
    """Weight-norm pair: v ~ N(0, std); g = ||v|| * U(0.7, 1.3) (so the fold is exercised)."""
    v = g.normal(shape, std)
    dims = [d for d in range(len(shape)) if d != dim]
    norm = v.pow(2).sum(dim=dims, keepdim=True).sqrt()
    sd[name + ".weight_g"] = norm * g.uniform(norm.shape, 0.7, 1.3)
    sd[name + ".weight_v"] = v


def _conv(g: _Gen, sd, name, co, ci, k, gain=1.0, bias=True):
    sd[name + ".weight"] = g.normal((co, ci, k), gain / math.sqrt(ci * k))
    if bias:
        sd[name + ".bias"] = g.normal((co,), 0.02)


def synth_state_dict(cfg: list, seed: int = 1234, emb_dim: int = 768) -> "OrderedDict[str, torch.Tensor]":
    """fp32 state dict of ``Synthesizer`` minus ``enc_q`` (``synthesizers.py:396-426``)."""
    (_, _, inter, hidden, filt, n_heads, n_layers, ksz, _, _, rks, rds, ur, uic, uks, spk, gin, sr) = cfg
    g = _Gen(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    kc = hidden // n_heads
    # TextEncoder (synthesizers.py:350-371)
    sd["enc_p.emb_phone.weight"] = g.normal((hidden, emb_dim), 1.0 / math.sqrt(emb_dim))
    sd["enc_p.emb_phone.bias"] = g.normal((hidden,), 0.02)
    sd["enc_p.emb_pitch.weight"] = g.normal((256, hidden), 0.1)
    for i in range(n_layers):
        p = f"enc_p.encoder.attn_layers.{i}."
        sd[p + "emb_rel_k"] = g.normal((1, 21, kc), kc ** -0.5)
        sd[p + "emb_rel_v"] = g.normal((1, 21, kc), kc ** -0.5)
        for n in ("q", "k", "v", "o"):
            _conv(g, sd, p + f"conv_{n}", hidden, hidden, 1)
        sd[f"enc_p.encoder.norm_layers_1.{i}.gamma"] = g.uniform((hidden,), 0.8, 1.2)
        sd[f"enc_p.encoder.norm_layers_1.{i}.beta"] = g.normal((hidden,), 0.05)
        _conv(g, sd, f"enc_p.encoder.ffn_layers.{i}.conv_1", filt, hidden, ksz)
        _conv(g, sd, f"enc_p.encoder.ffn_layers.{i}.conv_2", hidden, filt, ksz)
        sd[f"enc_p.encoder.norm_layers_2.{i}.gamma"] = g.uniform((hidden,), 0.8, 1.2)
        sd[f"enc_p.encoder.norm_layers_2.{i}.beta"] = g.normal((hidden,), 0.05)
    _conv(g, sd, "enc_p.proj", inter * 2, hidden, 1, gain=0.5)
    # GeneratorNSF (synthesizers.py:114-161)
    sd["dec.m_source.l_linear.weight"] = g.uniform((1, 1), 0.5, 1.5)
    sd["dec.m_source.l_linear.bias"] = g.normal((1,), 0.02)
    _conv(g, sd, "dec.conv_pre", uic, inter, 7)
    nup = len(ur)
    chans = [uic // (2 ** (i + 1)) for i in range(nup)]
    strides = [math.prod(ur[i + 1:]) if i + 1 < nup else 1 for i in range(nup)]
    for i, (u, k) in enumerate(zip(ur, uks)):
        cin = uic // (2 ** i)
        sd[f"dec.ups.{i}.bias"] = g.normal((chans[i],), 0.02)
        _wn(g, sd, f"dec.ups.{i}", (cin, chans[i], k), 1.0 / math.sqrt(cin * k / u))
        s = strides[i]
        kn = 1 if s == 1 else s * 2 - s % 2
        _conv(g, sd, f"dec.noise_convs.{i}", chans[i], 1, kn, gain=0.5)
    j = 0
    for i in range(nup):
        c = chans[i]
        for k, ds in zip(rks, rds):
            for m in range(len(ds)):
                for nm in ("convs1", "convs2"):
                    sd[f"dec.resblocks.{j}.{nm}.{m}.bias"] = g.normal((c,), 0.02)
                    _wn(g, sd, f"dec.resblocks.{j}.{nm}.{m}", (c, c, k), 0.5 / math.sqrt(c * k))
            j += 1
    sd["dec.conv_post.weight"] = g.normal((1, chans[-1], 7), 1.0 / math.sqrt(chans[-1] * 7))
    _conv(g, sd, "dec.cond", uic, gin, 1, gain=0.5)
    # ResidualCouplingBlock (residuals.py:71-140) + WaveNet (modules.py:9-59)
    half = inter // 2
    for f in range(4):
        p = f"flow.flows.{2 * f}."
        _conv(g, sd, p + "pre", hidden, half, 1)
        for l in range(3):
            sd[p + f"enc.in_layers.{l}.bias"] = g.normal((2 * hidden,), 0.02)
            _wn(g, sd, p + f"enc.in_layers.{l}", (2 * hidden, hidden, 5), 1.0 / math.sqrt(hidden * 5))
            rs = hidden if l == 2 else 2 * hidden
            sd[p + f"enc.res_skip_layers.{l}.bias"] = g.normal((rs,), 0.02)
            _wn(g, sd, p + f"enc.res_skip_layers.{l}", (rs, hidden, 1), 1.0 / math.sqrt(hidden))
        sd[p + "enc.cond_layer.bias"] = g.normal((2 * hidden * 3,), 0.02)
        _wn(g, sd, p + "enc.cond_layer", (2 * hidden * 3, gin, 1), 0.5 / math.sqrt(gin))
        _conv(g, sd, p + "post", half, hidden, 1, gain=0.3)
    sd["emb_g.weight"] = g.normal((spk, gin), 1.0)
    return sd


def make_synth_ckpt(sr: int = 48000, version: str = "v2", seed: int = 1234) -> dict:
    """A voice-model checkpoint dict in the ``train.py:729-742`` layout (fp16 weights)."""
    cfg = synth_config(sr, version)
    sd = synth_state_dict(cfg, seed, emb_dim=768 if version == "v2" else 256)
    opt = OrderedDict(weight=OrderedDict((k, v.half()) for k, v in sd.items()))
    opt["config"] = cfg
    opt["epoch"] = "1epoch"
    opt["step"] = 1
    opt["sr"] = f"{sr // 1000}k"
    opt["f0"] = 1
    opt["version"] = version
    opt["model_name"] = f"synthetic_{sr // 1000}k_{version}_s{seed}"
    opt["vocoder"] = "Default"
    return opt


# ---------------------------------------------------------------- ContentVec
HUBERT_CFG = dict(_name="hubert", label_rate=50, encoder_layers_1=3, logit_temp_ctr=0.1, num_negatives=100,
                  cross_sample_negatives=0, ctr_layers=[-6], extractor_mode="default", encoder_layers=12,
                  encoder_embed_dim=768, encoder_ffn_embed_dim=3072, encoder_attention_heads=12,
                  activation_fn="gelu", layer_type="transformer", dropout=0.1, attention_dropout=0.1,
                  activation_dropout=0.0, encoder_layerdrop=0.0, dropout_input=0.0, dropout_features=0.0,
                  final_dim=256, untie_final_proj=False, layer_norm_first=False,
                  conv_feature_layers="[(512,10,5)] + [(512,3,2)] * 4 + [(512,2,2)] * 2", conv_bias=False,
                  conv_pos=128, conv_pos_groups=16, required_seq_len_multiple=2)
FE_LAYERS = [(512, 10, 5)] + [(512, 3, 2)] * 4 + [(512, 2, 2)] * 2


def contentvec_state_dict(seed: int = 4321) -> "OrderedDict[str, torch.Tensor]":
    """fp32 ``HubertModel`` state dict (``fairseq.py:1326-1372``), ContentVec shapes."""
    g = _Gen(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    E, F = 768, 3072
    sd["mask_emb"] = g.uniform((E,), 0, 1)
    sd["label_embs_concat"] = g.uniform((504, 256), 0, 1)
    cin = 1
    for i, (c, k, s) in enumerate(FE_LAYERS):
        sd[f"feature_extractor.conv_layers.{i}.0.weight"] = g.normal((c, cin, k), math.sqrt(2.0 / (cin * k)))
        if i == 0:
            sd["feature_extractor.conv_layers.0.2.weight"] = g.uniform((c,), 0.8, 1.2)
            sd["feature_extractor.conv_layers.0.2.bias"] = g.normal((c,), 0.05)
        cin = c
    sd["layer_norm.weight"] = g.uniform((512,), 0.8, 1.2)
    sd["layer_norm.bias"] = g.normal((512,), 0.05)
    sd["post_extract_proj.weight"] = g.normal((E, 512), 1 / math.sqrt(512))
    sd["post_extract_proj.bias"] = g.normal((E,), 0.02)
    sd["encoder.pos_conv.0.bias"] = g.normal((E,), 0.02)
    _wn(g, sd, "encoder.pos_conv.0", (E, E // 16, 128), math.sqrt(4.0 / (128 * E)), dim=2)
    sd["encoder.layer_norm.weight"] = g.uniform((E,), 0.8, 1.2)
    sd["encoder.layer_norm.bias"] = g.normal((E,), 0.05)
    for i in range(12):
        p = f"encoder.layers.{i}."
        for n in ("k_proj", "v_proj", "q_proj", "out_proj"):
            sd[p + f"self_attn.{n}.weight"] = g.normal((E, E), 1 / math.sqrt(E))
            sd[p + f"self_attn.{n}.bias"] = g.normal((E,), 0.02)
        sd[p + "self_attn_layer_norm.weight"] = g.uniform((E,), 0.8, 1.2)
        sd[p + "self_attn_layer_norm.bias"] = g.normal((E,), 0.05)
        sd[p + "fc1.weight"] = g.normal((F, E), 1 / math.sqrt(E))
        sd[p + "fc1.bias"] = g.normal((F,), 0.02)
        sd[p + "fc2.weight"] = g.normal((E, F), 1 / math.sqrt(F))
        sd[p + "fc2.bias"] = g.normal((E,), 0.02)
        sd[p + "final_layer_norm.weight"] = g.uniform((E,), 0.8, 1.2)
        sd[p + "final_layer_norm.bias"] = g.normal((E,), 0.05)
    sd["final_proj.weight"] = g.normal((256, E), 1 / math.sqrt(E))
    sd["final_proj.bias"] = g.normal((256,), 0.02)
    return sd


def make_contentvec_ckpt(seed: int = 4321) -> dict:
    return {"cfg": {"model": dict(HUBERT_CFG), "task": {"sample_rate": 16000}}, "model": contentvec_state_dict(seed)}


# transformers' HubertConfig for the same network (HubertModelWithFinalProj, main/library/utils.py:157-165)
HF_HUBERT_CONFIG = dict(model_type="hubert", architectures=["HubertModelWithFinalProj"], hidden_size=768,
                        num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072, hidden_act="gelu",
                        feat_extract_norm="group", feat_extract_activation="gelu", conv_dim=[512] * 7,
                        conv_stride=[5, 2, 2, 2, 2, 2, 2], conv_kernel=[10, 3, 3, 3, 3, 2, 2], conv_bias=False,
                        num_conv_pos_embeddings=128, num_conv_pos_embedding_groups=16, do_stable_layer_norm=False,
                        layer_norm_eps=1e-5, feat_proj_layer_norm=True, classifier_proj_size=256)


def make_hf_hubert(seed: int = 4321) -> tuple[dict, dict]:
    """(config.json dict, state dict) of a transformers-layout ContentVec (``HubertModelWithFinalProj``, the
    ``.safetensors`` embedder of convert.py:342-345) holding the values of ``contentvec_state_dict(seed)`` under
    transformers' parameter names (the weight-norm pair as ``parametrizations.weight.original0 / 1``)."""
    src = contentvec_state_dict(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    sd["masked_spec_embed"] = src["mask_emb"]
    for i in range(len(FE_LAYERS)):
        sd[f"feature_extractor.conv_layers.{i}.conv.weight"] = src[f"feature_extractor.conv_layers.{i}.0.weight"]
    sd["feature_extractor.conv_layers.0.layer_norm.weight"] = src["feature_extractor.conv_layers.0.2.weight"]
    sd["feature_extractor.conv_layers.0.layer_norm.bias"] = src["feature_extractor.conv_layers.0.2.bias"]
    sd["feature_projection.layer_norm.weight"] = src["layer_norm.weight"]
    sd["feature_projection.layer_norm.bias"] = src["layer_norm.bias"]
    sd["feature_projection.projection.weight"] = src["post_extract_proj.weight"]
    sd["feature_projection.projection.bias"] = src["post_extract_proj.bias"]
    sd["encoder.pos_conv_embed.conv.bias"] = src["encoder.pos_conv.0.bias"]
    sd["encoder.pos_conv_embed.conv.parametrizations.weight.original0"] = src["encoder.pos_conv.0.weight_g"]
    sd["encoder.pos_conv_embed.conv.parametrizations.weight.original1"] = src["encoder.pos_conv.0.weight_v"]
    sd["encoder.layer_norm.weight"] = src["encoder.layer_norm.weight"]
    sd["encoder.layer_norm.bias"] = src["encoder.layer_norm.bias"]
    for i in range(12):
        a, b = f"encoder.layers.{i}.", f"encoder.layers.{i}."
        for n in ("k_proj", "v_proj", "q_proj", "out_proj"):
            for t in ("weight", "bias"):
                sd[f"{b}attention.{n}.{t}"] = src[f"{a}self_attn.{n}.{t}"]
        for hf, fs in (("layer_norm", "self_attn_layer_norm"), ("feed_forward.intermediate_dense", "fc1"),
                       ("feed_forward.output_dense", "fc2"), ("final_layer_norm", "final_layer_norm")):
            for t in ("weight", "bias"):
                sd[f"{b}{hf}.{t}"] = src[f"{a}{fs}.{t}"]
    sd["final_proj.weight"] = src["final_proj.weight"]
    sd["final_proj.bias"] = src["final_proj.bias"]
    return dict(HF_HUBERT_CONFIG), sd


# ---------------------------------------------------------------- RMVPE
def _bn(g: _Gen, sd, name, c):
    sd[name + ".weight"] = g.uniform((c,), 0.8, 1.2)
    sd[name + ".bias"] = g.normal((c,), 0.05)
    sd[name + ".running_mean"] = g.normal((c,), 0.05)
    sd[name + ".running_var"] = g.uniform((c,), 0.5, 1.5)
    sd[name + ".num_batches_tracked"] = torch.tensor(100, dtype=torch.long)


def _conv2(g: _Gen, sd, name, co, ci, k, bias=False, gain=1.0):
    sd[name + ".weight"] = g.normal((co, ci, k, k), gain * math.sqrt(2.0 / (ci * k * k)))
    if bias:
        sd[name + ".bias"] = g.normal((co,), 0.02)


def _cbr(g: _Gen, sd, name, ci, co):
    """ConvBlockRes (RMVPE.py:11-22)."""
    _conv2(g, sd, name + ".conv.0", co, ci, 3, gain=0.7)
    _bn(g, sd, name + ".conv.1", co)
    _conv2(g, sd, name + ".conv.3", co, co, 3, gain=0.7)
    _bn(g, sd, name + ".conv.4", co)
    if ci != co:
        _conv2(g, sd, name + ".shortcut", co, ci, 1, bias=True, gain=0.7)


def rmvpe_state_dict(seed: int = 777) -> "OrderedDict[str, torch.Tensor]":
    """fp32 ``E2E(4, 1, (2, 2))`` state dict (``RMVPE.py:125-144,254-260``)."""
    g = _Gen(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    nb = 4
    _bn(g, sd, "unet.encoder.bn", 1)
    ci, co = 1, 16
    for l in range(5):
        for b in range(nb):
            _cbr(g, sd, f"unet.encoder.layers.{l}.conv.{b}", ci if b == 0 else co, co)
        ci, co = co, co * 2
    ci, co = 256, 512
    for l in range(4):
        for b in range(nb):
            _cbr(g, sd, f"unet.intermediate.layers.{l}.conv.{b}", (ci if l == 0 else co) if b == 0 else co, co)
    cin = 512
    for l in range(5):
        cout = cin // 2
        sd[f"unet.decoder.layers.{l}.conv1.0.weight"] = g.normal((cin, cout, 3, 3), math.sqrt(2.0 / (cin * 9 / 4)) * 0.7)
        _bn(g, sd, f"unet.decoder.layers.{l}.conv1.1", cout)
        for b in range(nb):
            _cbr(g, sd, f"unet.decoder.layers.{l}.conv2.{b}", cout * 2 if b == 0 else cout, cout)
        cin = cout
    _conv2(g, sd, "cnn", 3, 16, 3, bias=True)
    H, I = 256, 384
    for sfx in ("", "_reverse"):
        sd[f"fc.0.gru.weight_ih_l0{sfx}"] = g.normal((3 * H, I), 1 / math.sqrt(I))
        sd[f"fc.0.gru.weight_hh_l0{sfx}"] = g.normal((3 * H, H), 1 / math.sqrt(H))
        sd[f"fc.0.gru.bias_ih_l0{sfx}"] = g.normal((3 * H,), 0.05)
        sd[f"fc.0.gru.bias_hh_l0{sfx}"] = g.normal((3 * H,), 0.05)
    sd["fc.1.weight"] = g.normal((360, 512), 1 / math.sqrt(512))
    sd["fc.1.bias"] = g.normal((360,), 0.05)
    return sd


# ---------------------------------------------------------------- CREPE
CREPE_CAPACITY = {
    "full": ([1, 1024, 128, 128, 128, 256], [1024, 128, 128, 128, 256, 512], 2048),
    "large": ([1, 768, 96, 96, 96, 192], [768, 96, 96, 96, 192, 384], 1536),
    "medium": ([1, 512, 64, 64, 64, 128], [512, 64, 64, 64, 128, 256], 1024),
    "small": ([1, 256, 32, 32, 32, 64], [256, 32, 32, 32, 64, 128], 512),
    "tiny": ([1, 128, 16, 16, 16, 32], [128, 16, 16, 16, 32, 64], 256),
}


def crepe_state_dict(seed: int = 999, capacity: str = "full") -> "OrderedDict[str, torch.Tensor]":
    """fp32 ``Crepe(capacity)`` state dict (``CREPE.py:11-58``): conv{i} (k x 1 kernels), conv{i}_BN,
    classifier."""
    g = _Gen(seed)
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    cin, cout, nfeat = CREPE_CAPACITY[capacity]
    for i in range(6):
        k = 512 if i == 0 else 64
        sd[f"conv{i + 1}.weight"] = g.normal((cout[i], cin[i], k, 1), math.sqrt(2.0 / (cin[i] * k)))
        sd[f"conv{i + 1}.bias"] = g.normal((cout[i],), 0.02)
        _bn(g, sd, f"conv{i + 1}_BN", cout[i])
    sd["classifier.weight"] = g.normal((360, nfeat), 2.0 / math.sqrt(nfeat))
    sd["classifier.bias"] = g.normal((360,), 0.5)
    return sd


# ---------------------------------------------------------------- audio
def synthetic_audio(seconds: float, seed: int = 1000, sr: int = 16000) -> np.ndarray:
    """SURVEY §8(d) test signal: 3-harmonic glide (60-240 Hz) + 200 ms gaps every 5 s + noise, peak <= 0.9."""
    n = int(round(seconds * sr))
    t = np.arange(n, dtype=np.float64) / sr
    f0 = 120.0 * 2.0 ** np.sin(2 * np.pi * 0.25 * t)
    phi = 2 * np.pi * np.cumsum(f0) / sr
    x = sum(0.5 ** (h - 1) * np.sin(h * phi) for h in (1, 2, 3)) * 0.3
    env = np.ones(n)
    for s0 in np.arange(5.0, seconds, 5.0):
        a, b = int((s0 - 0.1) * sr), int((s0 + 0.1) * sr)
        env[max(a, 0):min(b, n)] = 0.0
    rng = np.random.Generator(np.random.PCG64(seed))
    x = env * x + 0.003 * rng.standard_normal(n)
    peak = np.abs(x).max()
    if peak > 0.9:
        x *= 0.9 / peak
    return x.astype(np.float32)


def silence_layout_audio(layout, seed: int = 5000, sr: int = 16000, floor: float = 1e-5) -> np.ndarray:
    """Test signal for the silence slicer (edges.py): ``layout`` = [(seconds, voiced?), ...]; voiced
    spans are the §8(d) glide, silent spans seeded noise at ``floor`` (≈ -100 dBFS, no exact ties)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parts = []
    for k, (sec, voiced) in enumerate(layout):
        n = int(round(sec * sr))
        if voiced:
            parts.append(synthetic_audio(sec, seed=seed + 1 + k, sr=sr)[:n].astype(np.float64))
        else:
            parts.append(floor * rng.standard_normal(n))
    return np.concatenate(parts).astype(np.float32)


# slicer cases: leading / short (< max_sil_kept) / medium (1-2x) / long (> 2x) middle silences, trailing
SLICER_LAYOUTS = {
    "mixed": [(1.0, 0), (6.0, 1), (0.7, 0), (6.0, 1), (7.0, 0), (6.0, 1), (11.0, 0), (5.0, 1), (2.0, 0)],
    "no_silence": [(8.0, 1)],
    "short_input": [(0.5, 0), (3.0, 1)],
    "lead_long": [(12.0, 0), (6.0, 1), (0.3, 0), (2.0, 1)],
}
