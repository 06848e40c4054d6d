"""Micro-timings of the non-conv kernels at the bench's 30 s shapes (HIP events, torch stream).

    python scripts/micro.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rvc-maker_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    from rvc_amd import ops
    from rvc_amd.pipeline import AH, BH
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    # filtfilt + reflect pad, 30 s at 16 kHz
    f = ops.FiltFilt(BH, AH)
    for n in (480000, 96000, 16000, 4000):
        x = (torch.randn(n, generator=g) * 0.3).to(dev)
        print(f"filtfilt_pad N={n}: {timeit(lambda: f(x, min(16000, n - 1))):9.1f} us")
    # attention: TextEncoder (2 x 96, rel band W=10), ContentVec (12 x 64)
    for H, D, T, rel in ((2, 96, 3200, True), (12, 64, 1600, False), (2, 96, 3200, False)):
        qkv = torch.randn(3 * H * D, T, generator=g).to(dev)
        o = torch.empty(H * D, T, device=dev)
        kw = {}
        if rel:
            kw = dict(rk=torch.randn(H, 21, T, generator=g).to(dev) * 0.1, ev=torch.randn(21, D, generator=g).to(dev),
                      ml=torch.empty(H, 2, T, device=dev), W=10)
        C = H * D
        fn = lambda: ops.attention(qkv, qkv[C:], qkv[2 * C:], o, B=1, H=H, D=D, T=T, ldc=T, q_hs=D * T,  # noqa: E731
                                   k_hs=D * T, v_hs=D * T, o_hs=D * T, scale=D ** -0.5, **kw)
        us = timeit(fn)
        fl = 4.0 * T * T * D * H
        print(f"attention H={H} D={D} T={T} rel={rel}: {us:9.1f} us  {fl / us / 1e6:6.1f} TFLOP/s")
    # split-K reduce candidates: a flow-sized conv
    for Ci, Co, K, L in ((192, 384, 5, 3200), (192, 192, 1, 3200), (192, 768, 3, 3200), (768, 192, 3, 3200)):
        w = torch.randn(Co, Ci, K, generator=g) / np.sqrt(Ci * K)
        c = ops.Conv(w, torch.zeros(Co), device=dev)
        xi = torch.randn(Ci, L, generator=g).to(dev)
        us = timeit(lambda: c(xi, pad=K // 2))
        print(f"conv Ci={Ci} Co={Co} K={K} L={L}: {us:9.1f} us  {2.0 * Ci * Co * K * L / us / 1e6:6.1f} TFLOP/s")


def branches():
    """Critical-path pieces of one 30 s pipeline step, each timed alone."""
    import bench
    from rvc_amd import synthetic
    vc, hub, net_g = bench.build_models("cuda:0")
    audio = torch.from_numpy(synthetic.synthetic_audio(float(os.environ.get("SECONDS", 30)), seed=1000)).cuda()
    xp, _ = vc.filt(audio, vc.t_pad)
    print(f"filtfilt+pad:      {timeit(lambda: vc.filt(audio, vc.t_pad), 5):9.1f} us")
    print(f"ContentVec feats:  {timeit(lambda: vc.features_device(hub, xp, 'v2'), 5):9.1f} us")
    print(f"RMVPE f0:          {timeit(lambda: vc._rmvpe().f0_device(xp, 0.03, 0.0), 5):9.1f} us")
    feats = vc.features_device(hub, xp, "v2")
    coarse, pitchf, _ = vc._rmvpe().f0_device(xp, 0.03, 0.0)
    p_len = xp.numel() // 160
    fn = lambda: vc.voice_conversion_device(hub, net_g, 0, xp, coarse[:p_len], pitchf[:p_len], "v2", 0.33, 0,  # noqa
                                            feats=feats)
    print(f"synth (enc+flow+gen): {timeit(fn, 3):9.1f} us")
    print(f"full pipeline_device: {timeit(lambda: vc.pipeline_device(hub, net_g, 0, audio, 0, 'v2', 0.33), 3):9.1f} us")


if __name__ == "__main__" and not (len(sys.argv) > 1 and sys.argv[1] in ("retrieval", "synth", "bigru", "norms")):
    if len(sys.argv) > 1 and sys.argv[1] == "branches":
        branches()
        sys.exit(0)
    main()


def retrieval():
    """IVF-Flat search + blend at the cfg-3 index shape (100k x 768, IVF2564, nprobe 1), 1599 queries."""
    import bench
    idx = bench.synthetic_index("cuda")
    q = torch.randn(768, 1599, device="cuda")
    print(f"ivf search: {timeit(lambda: idx.search_cf(q), 5):9.1f} us")
    D, I = idx.search_cf(q)
    print(f"ivf blend:  {timeit(lambda: idx.blend_cf(q, D, I, 0.75), 5):9.1f} us")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "retrieval":
    retrieval()


def synth_stages():
    """The synthesizer's stages at the 30 s shape (T = 3198), each timed alone."""
    import bench
    vc, hub, net_g = bench.build_models("cuda:0")
    T = 3198
    g = torch.Generator().manual_seed(0)
    phone = torch.randn(768, T, generator=g).cuda()
    pitch = torch.randint(1, 255, (T,), generator=g).cuda()
    f0 = (torch.rand(T, generator=g) * 300 + 80).cuda()
    gc = net_g.speaker_cond(0)
    stats = net_g.text_encoder(phone, pitch, T)
    z_p = stats[:net_g.inter].contiguous()
    z = net_g.flow_reverse(z_p, gc, T)
    sn = torch.randn(T * net_g.upp, generator=g).cuda()
    print(f"text encoder: {timeit(lambda: net_g.text_encoder(phone, pitch, T), 5):9.1f} us")
    print(f"flow reverse: {timeit(lambda: net_g.flow_reverse(z_p, gc, T), 5):9.1f} us")
    print(f"generator:    {timeit(lambda: net_g.generator(z, f0, gc[4 * 6 * net_g.hidden:], T, sn), 3):9.1f} us")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "synth":
    synth_stages()


def bigru_bench():
    """The BiGRU recurrence alone at the 30 s shape (Tp = 3232), 1 and 16 sequences."""
    from rvc_amd import ops, synthetic
    from rvc_amd.rmvpe import RMVPEAMD
    rm = RMVPEAMD(synthetic.rmvpe_state_dict(1236), "cuda")
    T = 3232
    g = torch.Generator().manual_seed(0)
    for B in (1, 16):
        gi = (torch.randn(B, 1536, T, generator=g) * 0.5).cuda()
        y = torch.empty(B, 512, T, device="cuda")
        gran = torch.zeros(1024 * B, dtype=torch.int64, device="cuda")
        us = timeit(lambda: ops.bigru_batched(gi, rm.w_hh, rm.b_hh, y, gran, rm.err, B, T), 5)
        print(f"bigru B={B:2d} T={T}: {us:9.1f} us  ({us / T * 1e3:.0f} ns per step)")
    rm.check_error()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "bigru":
    bigru_bench()


def norms():
    """layernorm_cf / chnorm_gelu at the bench's shapes: time and HBM GB/s (bytes: read x (+res), write)."""
    from rvc_amd import ops
    g = torch.Generator().manual_seed(0)
    for C, T, res in ((768, 1599, True), (192, 3198, True), (512, 1599, False)):
        x = torch.randn(C, T, generator=g).cuda()
        r = torch.randn(C, T, generator=g).cuda() if res else None
        gm, bt = torch.ones(C).cuda(), torch.zeros(C).cuda()
        out = torch.empty(C, T, device="cuda")
        us = timeit(lambda: ops.layernorm_cf(x, r, gm, bt, out, 1, C, T), 20)
        nb = 4 * C * T * (3 if res else 2)
        print(f"layernorm_cf C={C} T={T} res={int(res)}: {us:7.1f} us  {nb / us / 1e3:7.1f} GB/s")
    x = torch.randn(512, 102399, generator=g).cuda()
    out = torch.empty_like(x)
    us = timeit(lambda: ops.chnorm_gelu(x, torch.ones(512).cuda(), torch.zeros(512).cuda(), out, 1, 512, 102399), 10)
    nb = 4 * 512 * 102399 * 3
    print(f"chnorm_gelu C=512 L=102399: {us:7.1f} us  {nb / us / 1e3:7.1f} GB/s (2 reads + 1 write)")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "norms":
    norms()
