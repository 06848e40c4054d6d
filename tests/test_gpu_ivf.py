"""FAISS IVF-Flat retrieval on the device (ivf.hip) vs the numpy oracle (oracle/ivf.py): identical
neighbour indices, and the convert.py:349-359 blend; plus VC.pipeline with an index file vs the CPU
oracle pipeline.  faiss is absent here, so faiss's own f32 rounding is "parity unpinned"."""
import numpy as np
import pytest
import torch

import f0check
from oracle import ivf as oivf
from rvc_amd.faiss_index import IVFFlatIndex

pytestmark = pytest.mark.gpu
DEV = "cuda"


def make(n, d, nlist, nprobe=1, seed=0, dups=0):
    rng = np.random.default_rng(seed)
    xb = rng.standard_normal((n, d)).astype(np.float32)
    if dups:
        xb[-dups:] = xb[:dups]  # exact duplicates: distance ties broken by id
    cent = xb[rng.choice(n, nlist, replace=False)] + 0.01
    return IVFFlatIndex.build(cent, xb, nprobe=nprobe), xb


@pytest.mark.parametrize("arithmetic", ["faiss", "exact"])
@pytest.mark.parametrize("n,d,nlist,nprobe,nq", [(6000, 768, 153, 1, 400), (3000, 256, 60, 3, 300),
                                                 (500, 768, 64, 1, 200), (800, 256, 16, 2, 12)])
def test_search_matches_oracle(n, d, nlist, nprobe, nq, arithmetic):
    """Identical neighbour lists and distances, in both arithmetics (the last case has nq < 20: faiss's direct
    coarse distances instead of the BLAS decomposition)."""
    from rvc_amd.retrieval import IVFFlatDevice
    idx, xb = make(n, d, nlist, nprobe, dups=8)
    rng = np.random.default_rng(7)
    nh = min(20, nq // 2)
    q = np.concatenate([xb[:nh] + 0.0, rng.standard_normal((nq - nh, d)).astype(np.float32)])  # exact hits too
    dev = IVFFlatDevice(idx, DEV)
    Dg, Ig = dev.search_cf(torch.from_numpy(np.ascontiguousarray(q.T)).to(DEV), k=8, arithmetic=arithmetic)
    Do, Io = oivf.search(idx, q, k=8, arithmetic=arithmetic)
    np.testing.assert_array_equal(Ig.cpu().numpy(), Io)
    if arithmetic == "faiss":  # the same f32 operations in the same order: bit-identical distances
        np.testing.assert_array_equal(Dg.cpu().numpy(), Do)
    else:
        np.testing.assert_allclose(Dg.cpu().numpy(), Do, rtol=1e-6, atol=1e-6)


def test_blend_matches_oracle():
    from rvc_amd.retrieval import IVFFlatDevice
    idx, xb = make(4000, 768, 100)
    rng = np.random.default_rng(3)
    q = rng.standard_normal((321, 768)).astype(np.float32)
    dev = IVFFlatDevice(idx, DEV)
    qd = torch.from_numpy(np.ascontiguousarray(q.T)).to(DEV)
    D, I = dev.search_cf(qd)
    out = dev.blend_cf(qd, D, I, 0.75).cpu().numpy().T
    ref = oivf.blend(q, D.cpu().numpy(), I.cpu().numpy(), idx.reconstruct_n(0, idx.ntotal), 0.75)
    np.testing.assert_allclose(out, ref, rtol=0, atol=2e-6)


def test_pipeline_with_index_vs_oracle(tmp_path):
    """VC.pipeline(file_index=..., index_rate=0.75) end to end vs the CPU oracle with oracle.ivf."""
    from oracle import contentvec as ocv
    from oracle import pipeline as opl
    from oracle import rmvpe as orm
    from oracle import synth as osy
    from rvc_amd import melbasis, synthetic
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    sr, version, seed = 40000, "v2", 71
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(sr, version, seed=seed), DEV)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(seed + 1), DEV)
    vc = VC(sr, Config(DEV), rmvpe=RMVPEAMD(synthetic.rmvpe_state_dict(seed + 2), DEV))
    audio = synthetic.synthetic_audio(3.0, seed=5)
    # index over "training features": ContentVec outputs of another clip, as create_index.py builds it
    feats = hub.features_cf(torch.from_numpy(synthetic.synthetic_audio(8.0, seed=6)).to(DEV)).t().cpu().numpy()
    rng = np.random.default_rng(0)
    idx = IVFFlatIndex.build(feats[rng.choice(len(feats), 16, replace=False)], feats)
    path = tmp_path / "added_IVF16_Flat_nprobe_1_test_v2.index"
    idx.write(str(path))
    noises = {}

    def noise(seg, kind, shape):
        if (seg, kind) not in noises:
            noises[(seg, kind)] = torch.randn(*shape, generator=torch.Generator().manual_seed(11 * seg + len(kind)))
        return noises[(seg, kind)]

    vc.noise_fn = lambda s, k, sh: noise(s, k, sh).to(DEV)
    out = vc.pipeline(hub, net_g, 0, audio.copy(), 0, "rmvpe", str(path), 0.75, 1, 3, 1, version, 0.33, 64, False, 1,
                      ".pth", ".pt")
    ck = synthetic.make_synth_ckpt(sr, version, seed=seed)
    torch.set_num_threads(16)
    Wc, Ws = ocv.load_weights(synthetic.make_contentvec_ckpt(seed + 1)), osy.load_weights(ck["weight"])
    Wr = orm.load_weights(synthetic.rmvpe_state_dict(seed + 2))
    mb = torch.from_numpy(melbasis.mel_filterbank())
    # f0 decisions vs the exact model (tests/f0check.py), then the waveform within 1e-4 RMS of the oracle
    f0check.assert_pipeline(vc, out, synthetic.rmvpe_state_dict(seed + 2), audio, lambda f0: opl.pipeline(
        Wc, Ws, Wr, mb, ck["config"], 0, audio, 0.0, version, 0.33, noise, index=idx, index_rate=0.75, f0_track=f0))


@pytest.mark.timeout(400)
def test_search_cfg3_index_shape_matches_oracle():
    """BASELINE configs[2]'s benchmarked index (bench.synthetic_ivf: IVF2564,Flat over 100k x 768, nprobe 1) searched
    with 1,599 queries -- one 32 s padded chunk's ContentVec frames, the largest query count the bench issues -- at
    the real [nq][nlist] coarse workspace and list sizes: identical neighbour ids and bit-identical distances to
    oracle/ivf.py.  Half the queries are drawn like the indexed data (close competition between nearby lists and
    neighbours), half are ContentVec features of a synthetic clip (the bench's own queries).
    Reference: create_index.py:63-83 (IVF{n},Flat, nprobe 1), convert.py:349-359 (search k=8)."""
    import importlib.util
    import os
    from rvc_amd import synthetic
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.retrieval import IVFFlatDevice
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    idx = bench.synthetic_ivf(DEV)
    assert idx.nlist == 2564 and idx.ntotal == 100_000
    rng = np.random.default_rng(5)
    near = (idx.centroids[rng.integers(0, idx.nlist, 800)] + 0.35 * rng.standard_normal((800, 768))).astype(np.float32)
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(1235), DEV)
    cv = hub.features_cf(torch.from_numpy(synthetic.synthetic_audio(32.0, seed=1000)).to(DEV)).t().cpu().numpy()
    q = np.ascontiguousarray(np.concatenate([near, cv[: 1599 - 800]]), dtype=np.float32)
    assert q.shape == (1599, 768)
    dev = IVFFlatDevice(idx, DEV)
    Dg, Ig = dev.search_cf(torch.from_numpy(np.ascontiguousarray(q.T)).to(DEV), k=8)
    Do, Io = oivf.search(idx, q, k=8)
    np.testing.assert_array_equal(Ig.cpu().numpy(), Io)
    np.testing.assert_array_equal(Dg.cpu().numpy(), Do)
