"""ContentVec linear shapes (K=1 convs, N = 1599 frames of a 30 s clip): the split-operand engine
(rvc_conv1d) vs the vendor f32 GEMM (torch.mm -> hipBLASLt / rocBLAS, TF32 off) on the same device."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rvc-maker_amd"))
import torch
from rvc_amd import ops

torch.backends.cuda.matmul.allow_tf32 = False
dev = "cuda"
N = 1599


def t_of(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


for Co, Ci in ((3072, 768), (768, 3072), (2304, 768), (768, 768), (768, 512)):
    w = torch.randn(Co, Ci, 1) / Ci ** 0.5
    b = torch.randn(Co)
    conv = ops.Conv(w, b, device=dev)
    x = torch.randn(Ci, N, device=dev)
    y = torch.empty(Co, N, device=dev)
    W = w[:, :, 0].to(dev).contiguous()
    bb = b.to(dev)
    te = t_of(lambda: conv(x, out=y))
    tb = t_of(lambda: torch.addmm(bb.view(-1, 1), W, x))
    ref = (W.double() @ x.double() + bb.double().view(-1, 1))
    ee = float(((y.double() - ref).abs().max()))
    eb = float(((torch.addmm(bb.view(-1, 1), W, x).double() - ref).abs().max()))
    fl = 2 * Co * Ci * N
    print(f"{Co}x{Ci}x{N}: engine {te:7.1f} us {fl / te / 1e6:6.1f} TF err {ee:.2e} | blas {tb:7.1f} us "
          f"{fl / tb / 1e6:6.1f} TF err {eb:.2e}", flush=True)
