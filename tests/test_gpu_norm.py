"""LayerNorm over channels and the per-channel GroupNorm(+GELU) against torch fp32 (F.layer_norm,
F.group_norm + exact GELU): shapes of ContentVec (768 / 512 channels), the TextEncoder (192) and the
feature extractor's first block, batched, ragged T, and rows whose mean is large against their spread."""
import pytest
import torch
import torch.nn.functional as F

from rvc_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("B,C,T,res", [(1, 768, 1599, True), (2, 192, 3198, True), (1, 512, 17, False), (3, 768, 1, True)])
def test_layernorm_cf(B, C, T, res):
    g = torch.Generator().manual_seed(C + T)
    x = torch.randn(B, C, T, generator=g) * 3 + 1.5
    r = torch.randn(B, C, T, generator=g) if res else None
    gm, bt = torch.randn(C, generator=g), torch.randn(C, generator=g)
    out = torch.empty(B, C, T, device=DEV)
    ops.layernorm_cf(x.to(DEV), r.to(DEV) if res else None, gm.to(DEV), bt.to(DEV), out, B, C, T)
    v = x + r if res else x
    ref = F.layer_norm(v.transpose(1, 2), (C,), gm, bt, 1e-5).transpose(1, 2)
    assert (out.cpu() - ref).abs().max().item() <= 2e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("B,C,L,offset", [(1, 512, 102399, 0.0), (2, 64, 5000, 40.0), (1, 8, 3, 0.0)])
@pytest.mark.parametrize("gelu", [True, False])
def test_chnorm_gelu(B, C, L, offset, gelu):
    g = torch.Generator().manual_seed(C + L)
    x = torch.randn(B, C, L, generator=g) * 0.5 + offset  # offset: mean large against the spread
    gm, bt = torch.randn(C, generator=g), torch.randn(C, generator=g)
    out = torch.empty(B, C, L, device=DEV)
    ops.chnorm_gelu(x.to(DEV), gm.to(DEV), bt.to(DEV), out, B, C, L, gelu=gelu)
    ref = F.group_norm(x.double(), C, gm.double(), bt.double(), 1e-5)
    if gelu:
        ref = F.gelu(ref)
    assert (out.cpu().double() - ref).abs().max().item() <= 5e-5 * max(1.0, ref.abs().max().item())
