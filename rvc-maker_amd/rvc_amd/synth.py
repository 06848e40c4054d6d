"""MI355X Synthesizer: drop-in for ``Synthesizer.infer`` (main/library/algorithm/synthesizers.py:446-465).

Built from a voice-model checkpoint in the reference layout (``train.py:729-742``):
weight-norm folded once in fp32 on the host at load (``torch._weight_norm``, as the
reference's parametrization computes it), weights packed K-major and uploaded.
All compute runs in librvc_amd.so kernels on the current torch stream:

  TextEncoder  conv1d(K=1) + textenc_embed + 6 x [fused QKV conv, rel-pos flash attention,
               conv_o, LN, FFN (conv k3 ReLU, conv k3), LN] + proj + prior_sample
  flow^-1      4 x [flip, pre, WaveNet(3 x conv k5 + gate + res/skip convs), post (fused x1 - m)]
  NSF-HiFiGAN  sine_source, conv_pre(+cond), 4 x [ConvT (polyphase, lrelu fused on staging, noise_conv fused in
               its epilogue) + 3 ResBlocks (lrelu fused, residual / running sum
               fused in the epilogue; at 32 / 64 channels each conv pair is one fused launch,
               csrc/resblock.hip)], conv_post (lrelu 0.01 + tanh fused)

Only full-length phones are supported (x_mask all ones): in ``VC.voice_conversion``
``p_len == phone length`` always holds (2*T_f <= N//160).
"""
from __future__ import annotations

import math

import torch

from . import ops
from .ops import ACT_LRELU, ACT_RELU, ACT_TANH, Conv, ConvT

import os

LRELU_SLOPE = 0.1
# the generator's |max| side channel (RVC_AMD_AMAX=0: per-tile pre-passes, the round-4 form; rvc_model.cpp reads the
# same switch): cells per upsample stage -- y, then each unfused pair's c1 output and non-last c2 output
AMAX = os.environ.get("RVC_AMD_AMAX", "1") != "0"
# the upsampling convs' inputs through |max| cells too (conv_pre's output, each unfused stage's output; A/B switch)
AMAX_UPS = os.environ.get("RVC_AMD_AMAX_UPS", "1") != "0"
AMAX_PER_STAGE = 16
# round 6: noise_convs[i](har) as a source pass inside ups[i]'s call (x = ups(x) + noise_convs(har), synthesizers.py:156;
# rvc_conv1d_args.src_*).  Off by default (RVC_AMD_FUSED_NOISE=1 turns it on; +1.3 % in the clip stream, r6h): with it
# on, the clip stream's first clip -- the one whose synthesizer runs beside the next clip's front end -- intermittently
# departs from the per-call pipeline by 2e-3 to 9e-3, first at this stage's output (z and g identical;
# scripts/stream_stage_diff.py).  Until that race is found, the two-launch form.
FUSED_NOISE = os.environ.get("RVC_AMD_FUSED_NOISE", "0") != "0"
# round 6: the TextEncoder's rel-pos attention in split-fp16 from the QKV projection's |max| (contentvec.ATTN_F16): the
# TextEncoder alone, 30 s, 2.89 -> 2.64 ms (scripts/synth_stage_time.py, r6d)
ATTN_F16 = os.environ.get("RVC_AMD_ATTN_F16", "1") != "0"
# round 6: the TextEncoder's GEMMs in split-fp16 from their producers' |max| cells (the embedding's, every LayerNorm's,
# ffn1's, the attention's) -- off by default: on these 192-channel, 3000-frame GEMMs split-fp16 ran slower than the
# 6-pass split-bf16 form (TextEncoder alone 2.14 -> 2.64 ms; clip stream 979 -> 949 xRT with the flow's below, r6d).
# Kept as RVC_AMD_TE_AMAX=1 (tested); the QKV projection publishes its cell for the attention either way.
TE_AMAX = os.environ.get("RVC_AMD_TE_AMAX", "0") != "0"
# ... and the flow's (RVC_AMD_FLOW_AMAX=1; off by default: flow^-1 alone 0.93 -> 1.50 ms with it, r6d; rvc_model.cpp
# reads both switches)
FLOW_AMAX = os.environ.get("RVC_AMD_FLOW_AMAX", "0") != "0"


def fold_weight_norm(weight: dict) -> dict:
    """ckpt ``{..., x.weight_g, x.weight_v}`` (fp16) -> fp32 ``{x.weight}`` (dim 0 norm)."""
    W = {}
    for k, v in weight.items():
        if k.endswith(".weight_v"):
            base = k[: -len(".weight_v")]
            W[base + ".weight"] = torch._weight_norm(v.float(), weight[base + ".weight_g"].float(), 0)
        elif not k.endswith(".weight_g"):
            W[k] = v.float()
    return W


class SynthesizerAMD:
    def __init__(self, cpt: dict, device: str = "cuda"):
        cfg = list(cpt["config"])
        cfg[-3] = cpt["weight"]["emb_g.weight"].shape[0]  # convert.py:558
        self.cfg = cfg
        (_, _, self.inter, self.hidden, self.filt, self.n_heads, self.n_layers, self.ksz, _, _, self.rks, self.rds,
         self.ur, self.uic, self.uks, self.spk, self.gin, self.sr) = cfg
        self.version = cpt.get("version", "v1")
        if cpt.get("f0", 1) != 1 or cpt.get("vocoder", "Default") != "Default":
            raise NotImplementedError("rvc_amd: only NSF-HiFiGAN (f0=1, vocoder Default) models are on the hot path")
        self.upp = math.prod(self.ur)
        self.device = device
        W = fold_weight_norm(cpt["weight"])
        dev = device
        H = self.hidden
        self.kc = H // self.n_heads
        # ---- TextEncoder
        self.emb_dim = W["enc_p.emb_phone.weight"].shape[1]
        self.emb_phone = Conv(W["enc_p.emb_phone.weight"].unsqueeze(-1), W["enc_p.emb_phone.bias"], device=dev)
        self.emb_pitch = W["enc_p.emb_pitch.weight"].contiguous().to(dev)
        self.layers = []
        for i in range(self.n_layers):
            p = f"enc_p.encoder.attn_layers.{i}."
            wqkv = torch.cat([W[p + "conv_q.weight"], W[p + "conv_k.weight"], W[p + "conv_v.weight"]], 0)
            bqkv = torch.cat([W[p + "conv_q.bias"], W[p + "conv_k.bias"], W[p + "conv_v.bias"]], 0)
            ek = W[p + "emb_rel_k"][0]  # [21, kc]
            L = dict(
                qkv=Conv(wqkv, bqkv, device=dev),
                relk=Conv(ek.unsqueeze(-1), None, device=dev),  # Rk[r][t] = Ek[r] . q[:, t]
                ev=W[p + "emb_rel_v"][0].contiguous().to(dev),
                o=Conv(W[p + "conv_o.weight"], W[p + "conv_o.bias"], device=dev),
                ln1=(W[f"enc_p.encoder.norm_layers_1.{i}.gamma"].to(dev), W[f"enc_p.encoder.norm_layers_1.{i}.beta"].to(dev)),
                ffn1=Conv(W[f"enc_p.encoder.ffn_layers.{i}.conv_1.weight"], W[f"enc_p.encoder.ffn_layers.{i}.conv_1.bias"], device=dev),
                ffn2=Conv(W[f"enc_p.encoder.ffn_layers.{i}.conv_2.weight"], W[f"enc_p.encoder.ffn_layers.{i}.conv_2.bias"], device=dev),
                ln2=(W[f"enc_p.encoder.norm_layers_2.{i}.gamma"].to(dev), W[f"enc_p.encoder.norm_layers_2.{i}.beta"].to(dev)),
            )
            self.layers.append(L)
        self.proj = Conv(W["enc_p.proj.weight"], W["enc_p.proj.bias"], device=dev)
        # ---- speaker conditioning: all cond convs stacked (4 flows x 3*2H, then dec.cond)
        conds_w = [W[f"flow.flows.{2 * f}.enc.cond_layer.weight"] for f in range(4)] + [W["dec.cond.weight"]]
        conds_b = [W[f"flow.flows.{2 * f}.enc.cond_layer.bias"] for f in range(4)] + [W["dec.cond.bias"]]
        self.cond = Conv(torch.cat(conds_w, 0), torch.cat(conds_b, 0), device=dev)
        self.emb_g = W["emb_g.weight"].contiguous().to(dev)
        # ---- flow
        self.flows = []
        for f in range(4):
            p = f"flow.flows.{2 * f}."
            F = dict(pre=Conv(W[p + "pre.weight"], W[p + "pre.bias"], device=dev), ins=[], rs_a=[], rs_b=[],
                     post=Conv(W[p + "post.weight"], W[p + "post.bias"], device=dev))
            for l in range(3):
                F["ins"].append(Conv(W[p + f"enc.in_layers.{l}.weight"], W[p + f"enc.in_layers.{l}.bias"], device=dev))
                rw, rb = W[p + f"enc.res_skip_layers.{l}.weight"], W[p + f"enc.res_skip_layers.{l}.bias"]
                if l < 2:
                    F["rs_a"].append(Conv(rw[:H], rb[:H], device=dev))
                    F["rs_b"].append(Conv(rw[H:], rb[H:], device=dev))
                else:
                    F["rs_b"].append(Conv(rw, rb, device=dev))
            self.flows.append(F)
        # ---- generator
        self.lin_w = float(W["dec.m_source.l_linear.weight"].reshape(-1)[0])
        self.lin_b = float(W["dec.m_source.l_linear.bias"].reshape(-1)[0])
        self.conv_pre = Conv(W["dec.conv_pre.weight"], W["dec.conv_pre.bias"], device=dev)
        nup = len(self.ur)
        self.chans = [self.uic // (2 ** (i + 1)) for i in range(nup)]
        strides = [math.prod(self.ur[i + 1:]) if i + 1 < nup else 1 for i in range(nup)]
        self.ups, self.noise, self.res = [], [], []
        for i, (u, k) in enumerate(zip(self.ur, self.uks)):
            if u % 2:
                raise NotImplementedError("odd upsample rates (output_padding) are not used by any shipped config")
            self.ups.append(ConvT(W[f"dec.ups.{i}.weight"], W[f"dec.ups.{i}.bias"], u, (k - u) // 2, device=dev))
            s = strides[i]
            kn = 1 if s == 1 else s * 2 - s % 2
            self.noise.append((Conv(W[f"dec.noise_convs.{i}.weight"], W[f"dec.noise_convs.{i}.bias"], device=dev), s,
                               0 if s == 1 else (kn - s) // 2))
            blocks = []
            for j, (kk, ds) in enumerate(zip(self.rks, self.rds)):
                rb = f"dec.resblocks.{i * len(self.rks) + j}."
                blocks.append((kk, [(d, Conv(W[rb + f"convs1.{m}.weight"], W[rb + f"convs1.{m}.bias"], device=dev),
                                     Conv(W[rb + f"convs2.{m}.weight"], W[rb + f"convs2.{m}.bias"], device=dev))
                                    for m, d in enumerate(ds)]))
            self.res.append(blocks)
        self.conv_post = Conv(W["dec.conv_post.weight"], None, device=dev)

    # ------------------------------------------------------------------ stages (B clips of one length T:
    # every launch takes the clip batch; B = 1 issues exactly the single-clip launches)
    def text_encoder(self, phone_cf, pitch, T, B=1):
        """TextEncoder.forward (synthesizers.py:366-371) on phone [B][E][T] -> stats [B][2*inter][T]."""
        H, dev, nh, kc = self.hidden, phone_cf.device, self.n_heads, self.kc
        lin = self.emb_phone(phone_cf.reshape(B, -1, T))
        x = torch.empty(B, H, T, device=dev)
        # |max| cells (round 6): the QKV projection's (ATTN_F16: the split-fp16 attention's scale) and, with TE_AMAX, the
        # embedding's, every LayerNorm's, the attention output's (its rel-v band kernel publishes) and ffn1's, the GEMM
        # reading each then running split-fp16 from it; cell 0 the embedding's, then per layer (qkv, o, ln1, ffn1, ln2)
        nl = len(self.layers)
        cells = ops.AmaxSlots(1 + 5 * nl, dev, B) if (TE_AMAX or ATTN_F16) else None
        cell = (lambda k: cells[k]) if (cells is not None and TE_AMAX) else (lambda k: None)
        qkv_cell = (lambda li: cells[1 + 5 * li]) if (cells is not None and ATTN_F16) else (lambda li: None)
        ops.textenc_embed(lin, self.emb_pitch if pitch is not None else None, pitch, x, B, H, T, math.sqrt(H), 0.1,
                          amax_out=cell(0))
        x_cell = cell(0)
        tmp = torch.empty(B, H, T, device=dev)
        o = torch.empty(B, H, T, device=dev)
        ml = torch.empty(B, nh, 2, T, device=dev)
        rk = torch.empty(B, nh, 21, T, device=dev)
        scale = 1.0 / math.sqrt(kc)
        for li, L in enumerate(self.layers):
            c_o, c_l1, c_f1, c_l2 = (cell(2 + 5 * li + k) for k in range(4))
            c_qkv = qkv_cell(li)
            qkv = L["qkv"](x, amax_in=x_cell, amax_out=c_qkv)
            for b in range(B):  # Rk of clip b's heads: one K=1 conv over its nh query slices
                L["relk"](qkv[b] if B > 1 else qkv, B=nh, Lin=T, x_bstride=kc * T, Lout=T, out_scale=scale,
                          out=rk[b])
            qb = qkv.view(B, 3 * H, T)
            ops.attention(qb, qb[:, H:], qb[:, 2 * H:], o, B=B, H=nh, D=kc, T=T, ldc=T, q_hs=kc * T,
                          k_hs=kc * T, v_hs=kc * T, o_hs=kc * T, q_bs=3 * H * T, k_bs=3 * H * T, v_bs=3 * H * T,
                          o_bs=H * T, scale=scale, rk=rk, ev=L["ev"], ml=ml, W=10,
                          amax_in=c_qkv, amax_out=c_o)
            y = L["o"](o, out=tmp, amax_in=c_o)
            ops.layernorm_cf(x, y, L["ln1"][0], L["ln1"][1], x, B, H, T, amax_out=c_l1)
            h = L["ffn1"](x, pad=(self.ksz - 1) // 2, out_act=ACT_RELU, amax_in=c_l1, amax_out=c_f1)
            y = L["ffn2"](h, pad=(self.ksz - 1) // 2, out=tmp, amax_in=c_f1)
            ops.layernorm_cf(x, y, L["ln2"][0], L["ln2"][1], x, B, H, T, amax_out=c_l2)
            x_cell = c_l2
        return self.proj(x, amax_in=x_cell).view(B, 2 * self.inter, T)

    def flow_reverse(self, z_p, gc, T, B=1):
        """ResidualCouplingBlock reverse (residuals.py:87-95, 127-137) + WaveNet (modules.py:35-51);
        z_p [B][inter][T]."""
        H, I, half, dev = self.hidden, self.inter, self.inter // 2, z_p.device
        x = z_p
        bufs = (torch.empty(B, I, T, device=dev), torch.empty(B, I, T, device=dev))
        h = torch.empty(B, H, T, device=dev)
        acts = torch.empty(B, H, T, device=dev)
        out_acc = torch.empty(B, H, T, device=dev)
        # |max| cells (round 6, FLOW_AMAX): per flow the WaveNet's h (pre, then each rs_a), the skip sum (the last rs_b) and
        # post's output x1 (the next flow's pre input, flipped) publish; the gate's output is tanh * sigmoid, |.| < 1,
        # so the res/skip convs take a constant 1.0 cell (cell 0)
        cells = ops.AmaxSlots(1 + 5 * 4, dev, B) if FLOW_AMAX else None
        cell = (lambda k: cells[k]) if cells is not None else (lambda k: None)
        if cells is not None:
            cells[0].view(B, ops.AMAX_SHARDS)[:, 0].fill_(0x3F800000)  # 1.0f
        unit = cell(0)
        post_cell = None
        for n, f in enumerate(reversed(range(4))):
            F = self.flows[f]
            c_h = [cell(1 + 5 * n + k) for k in range(3)]
            c_acc, c_post = cell(1 + 5 * n + 3), cell(1 + 5 * n + 4)
            xf = bufs[0] if x is not bufs[0] else bufs[1]
            ops.flip_channels(x, xf, B, I, T)
            # x0 = xf[:, :half], x1 = xf[:, half:]: batch stride I*T
            F["pre"](xf, B=B, Lin=T, x_bstride=I * T, out=h, amax_in=post_cell, amax_out=c_h[0])
            for l in range(3):
                g_l = gc[f * 6 * H + l * 2 * H: f * 6 * H + (l + 1) * 2 * H]
                xin = F["ins"][l](h, pad=2, bias2=g_l, amax_in=c_h[l])
                ops.gate(xin, acts, B, H, T)
                if l < 2:
                    F["rs_a"][l](acts, out=h, res=h, amax_in=unit, amax_out=c_h[l + 1])
                    F["rs_b"][l](acts, out=out_acc, accumulate=(l > 0), amax_in=unit)
                else:
                    F["rs_b"][l](acts, out=out_acc, accumulate=True, amax_in=unit, amax_out=c_acc)
            x1 = xf[:, half:]
            F["post"](out_acc, out=x1, res=x1, y_bstride=I * T, res_bstride=I * T, out_scale=-1.0, amax_in=c_acc,
                      amax_out=c_post)
            post_cell = c_post
            x = xf
        return x

    def generator(self, z, nsff0, gdec, T, sine_noise, B=1):
        """GeneratorNSF.forward (synthesizers.py:144-161) on z [B][inter][T] -> [B][1][T*upp]."""
        dev = z.device
        L = T * self.upp
        har = torch.empty(B, L, device=dev)
        work = torch.empty(B, T, device=dev)
        ops.sine_source(nsff0, sine_noise, har, work, B, T, self.upp, float(self.sr), self.lin_w, self.lin_b)
        nst = len(self.ur)
        cells = ops.AmaxSlots(AMAX_PER_STAGE * nst + nst + 1, dev, B) if AMAX else None
        # cells after the stages' own: one per stage for its output xs (published by the last resblock's last c2 when
        # that pair is unfused), one for conv_pre's output -- the upsampling convs' inputs
        out_cell = (lambda k: cells[AMAX_PER_STAGE * nst + k]) if AMAX else (lambda k: None)
        x = self.conv_pre(z.reshape(B, self.inter, T), pad=3, bias2=gdec, amax_out=out_cell(nst))
        x_cell = out_cell(nst)
        scale = 1.0
        nk = len(self.rks)
        # the |max| side channel (ops.AmaxSlots, include/rvc_amd.h): in each stage y (written last by the noise conv),
        # every unfused c1 output t1 and every non-last c2 output publish their |max|, and the convs reading them take
        # their split-fp16 activation scale from it -- no per-tile pre-pass, so split-fp16 pays at k = 3 and 256
        # channels too (rvc_model.cpp mirrors this cell by cell)
        for i in range(nst):
            up = self.ups[i]
            nc, s, pad = self.noise[i]
            base = AMAX_PER_STAGE * i
            ncell = 1
            if FUSED_NOISE:  # y = ups(x) + noise_convs(har) in one launch, which publishes y's |max|
                y = up(x, in_act=ACT_LRELU, in_slope=LRELU_SLOPE, in_scale=scale,
                       amax_in=x_cell if AMAX_UPS else None, src=(nc, har, s, pad),
                       amax_out=cells[base] if cells else None)
                Li = y.shape[-1]
            else:
                y = up(x, in_act=ACT_LRELU, in_slope=LRELU_SLOPE, in_scale=scale,
                       amax_in=x_cell if AMAX_UPS else None)
                Li = y.shape[-1]
                nc(har.view(B, 1, L), Lout=Li, stride=s, pad=pad, out=y, accumulate=True,
                   amax_out=cells[base] if cells else None)
            x_cell = None
            C = self.chans[i]
            t1 = None  # c1 output of the unfused pairs
            xa = torch.empty(B, C, Li, device=dev)
            xb = torch.empty(B, C, Li, device=dev)
            xs = torch.empty(B, C, Li, device=dev)
            y = y.view(B, C, Li)
            for j, (kk, pairs) in enumerate(self.res[i]):
                cur = y
                cur_cell = cells[base] if cells else None
                for m, (d, c1, c2) in enumerate(pairs):
                    last = m == len(pairs) - 1
                    if ops.resblock_fusable(c1, c2, d):  # one launch, c1's output stays in LDS
                        nxt = xs if last else (xa if cur is not xa else xb)
                        ops.resblock_pair(cur, nxt, c1, c2, d, LRELU_SLOPE, accumulate=last and j > 0)
                        cur = nxt
                        cur_cell = None
                        continue
                    if t1 is None:
                        t1 = torch.empty(B, C, Li, device=dev)
                    t1_cell = None
                    if cells and ncell < AMAX_PER_STAGE:
                        t1_cell, ncell = cells[base + ncell], ncell + 1
                    c1(cur, pad=(kk * d - d) // 2, dil=d, out=t1, in_act=ACT_LRELU, in_slope=LRELU_SLOPE,
                       amax_in=cur_cell, amax_out=t1_cell)
                    if m == len(pairs) - 1:
                        # the last resblock's last c2 writes the stage output's final values: its |max| cell
                        xo_cell = out_cell(i) if j == nk - 1 else None
                        c2(t1, pad=(kk - 1) // 2, out=xs, res=cur, in_act=ACT_LRELU, in_slope=LRELU_SLOPE,
                           accumulate=(j > 0), amax_in=t1_cell, amax_out=xo_cell)
                        if xo_cell is not None:
                            x_cell = xo_cell
                        cur_cell = None
                    else:
                        nxt = xa if cur is not xa else xb
                        nxt_cell = None
                        if cells and ncell < AMAX_PER_STAGE:
                            nxt_cell, ncell = cells[base + ncell], ncell + 1
                        c2(t1, pad=(kk - 1) // 2, out=nxt, res=cur, in_act=ACT_LRELU, in_slope=LRELU_SLOPE,
                           amax_in=t1_cell, amax_out=nxt_cell)
                        cur, cur_cell = nxt, nxt_cell
            del t1, xa, xb, y
            x = xs
            scale = 1.0 / nk
        return self.conv_post(x, pad=3, in_act=ACT_LRELU, in_slope=0.01, in_scale=scale, out_act=ACT_TANH)

    # ------------------------------------------------------------------ public API
    def speaker_cond(self, sid: int):
        g = self.emb_g[sid].view(self.gin, 1)
        return self.cond(g).view(-1)

    def prior_batch(self, phone_cf, pitch, sid: int, z_noise=None, seeds=(0,)):
        """Synthesizer.infer up to the generator (synthesizers.py:446-460) over B clips of one length:
        phone [B][E][T], pitch int64 [B][T] -> (z, z_p, stats) [B][.][T] and gc.  Clip b draws its prior
        noise with seeds[b] (exactly the draw of a single-clip call with that seed)."""
        B, E, T = phone_cf.shape
        dev = phone_cf.device
        if E != self.emb_dim:
            raise ValueError(f"phone dim {E} != model's {self.emb_dim}")
        if z_noise is None and len(seeds) != B:
            raise ValueError("prior_batch: one seed per clip")
        gc = self.speaker_cond(sid)
        stats = self.text_encoder(phone_cf, pitch, T, B)
        if z_noise is None:
            z_noise = torch.empty(B, self.inter, T, device=dev)
            for b in range(B):
                ops.randn(z_noise[b], seeds[b], 0)
        z_p = torch.empty(B, self.inter, T, device=dev)
        ops.prior_sample(stats, z_noise.reshape(B, self.inter, T), z_p, B, self.inter, T, 0.66666)
        z = self.flow_reverse(z_p, gc, T, B)
        return z, z_p, stats, gc

    def decode_batch(self, z, nsff0, gc, sine_noise=None, seeds=(0,)):
        """The NSF generator on z [B][inter][T] (synthesizers.py:461-465) -> o [B][T*upp]; clip b's sine
        noise from seeds[b]."""
        B, _, T = z.shape
        L = T * self.upp
        if sine_noise is None:
            if len(seeds) != B:
                raise ValueError("decode_batch: one seed per clip")
            sine_noise = torch.empty(B, L, device=z.device)
            for b in range(B):
                ops.randn(sine_noise[b], seeds[b], 1 << 40)
        o = self.generator(z, nsff0.reshape(B, T).float().contiguous(), gc[4 * 6 * self.hidden:], T,
                           sine_noise.reshape(B, L), B)
        return o.view(B, L)

    def prior_cf(self, phone_cf, pitch, sid: int, z_noise=None, seed: int = 0):
        """Synthesizer.infer up to the generator (synthesizers.py:446-460): TextEncoder, prior sample, flow^-1.
        phone [E][T], pitch int64 [T] -> (z, z_p, stats, gc)."""
        E, T = phone_cf.shape
        z, z_p, stats, gc = self.prior_batch(phone_cf.view(1, E, T), pitch, sid,
                                             None if z_noise is None else z_noise.reshape(1, self.inter, T), (seed,))
        return z[0], z_p[0], stats[0], gc

    def decode_cf(self, z, nsff0, gc, sine_noise=None, seed: int = 0):
        """The NSF generator on z [inter][T] (synthesizers.py:461-465) -> o [T*upp]."""
        T = z.shape[-1]
        return self.decode_batch(z.reshape(1, self.inter, T), nsff0, gc, sine_noise, (seed,)).view(-1)

    def infer_cf(self, phone_cf, pitch, nsff0, sid: int, z_noise=None, sine_noise=None, seed: int = 0):
        """Channels-first core: phone [E][T], pitch int64 [T], nsff0 f32 [T] -> (o [T*upp], z, z_p, stats)."""
        z, z_p, stats, gc = self.prior_cf(phone_cf, pitch, sid, z_noise, seed)
        return self.decode_cf(z, nsff0, gc, sine_noise, seed), z, z_p, stats

    def infer(self, phone, phone_lengths, pitch=None, nsff0=None, sid=None, rate=None, z_noise=None,
              sine_noise=None, seed: int = 0):
        """Synthesizer.infer signature (synthesizers.py:446): phone [1, T, E] -> (o [1,1,L], x_mask, (z, z_p, m_p, logs_p)).

        z_noise [1, inter, T] / sine_noise [1, T*upp, 1] inject the reference's randn_like draws
        (parity mode); None draws them on the device (Philox, ``seed``)."""
        if rate is not None:
            raise NotImplementedError("rate (partial inference) is not used by VC.pipeline")
        if pitch is None or nsff0 is None:
            raise NotImplementedError("only f0 (NSF) models are on the hot path")
        B, T, E = phone.shape
        if B != 1:
            raise NotImplementedError("batch 1 (as VC.voice_conversion calls it)")
        if int(phone_lengths.reshape(-1)[0]) != T:
            raise NotImplementedError("phone_lengths must equal the phone length (always true in VC.pipeline)")
        dev = phone.device
        phone_cf = torch.empty(E, T, device=dev)
        ops.transpose(phone.contiguous().float(), phone_cf, 1, T, E)
        sid_i = int(sid.reshape(-1)[0]) if torch.is_tensor(sid) else int(sid)
        o, z, z_p, stats = self.infer_cf(phone_cf, pitch.reshape(T).to(torch.int64).contiguous(), nsff0, sid_i,
                                         z_noise, sine_noise, seed)
        m_p, logs_p = stats[: self.inter], stats[self.inter:]
        x_mask = torch.ones(1, 1, T, device=dev)
        return o.view(1, 1, -1), x_mask, (z.unsqueeze(0), z_p.unsqueeze(0), m_p.unsqueeze(0), logs_p.unsqueeze(0))
