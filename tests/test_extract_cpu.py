"""Host side of training-feature extraction and the conversion front end:
coarse quantiser vs the reference's outputs, file list, WAV I/O, and the rank partition of the
extract / batch-convert loops over gloo (world 2) with the device models stubbed out."""
import os
import random
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from rvc_amd import audio_io, extract


def test_coarse_f0_matches_reference(golden):
    g = golden("edges")
    fi = extract.FeatureInputAMD(device="cpu")
    np.testing.assert_array_equal(fi.coarse_f0(g["coarse_in64"]), g["coarse_out64"])
    np.testing.assert_array_equal(fi.coarse_f0(g["coarse_in32"]), g["coarse_out32"])


def test_wav_roundtrip_and_load(tmp_path):
    rng = np.random.Generator(np.random.PCG64(1))
    x = (rng.standard_normal((16000, 2)) * 0.2).astype(np.float32)
    p = str(tmp_path / "a.wav")
    audio_io.write_wav(p, x, 16000)
    y, sr = audio_io.read_wav(p)
    assert sr == 16000 and y.shape == x.shape and y.dtype == np.float32
    assert np.abs(y - np.clip(x, -1, 1)).max() <= 2.0 / 32767  # write x 32767, read / 32768 (libsndfile)
    mono = audio_io.load_audio(" " + p + "\n", 16000)
    np.testing.assert_array_equal(mono, y.mean(axis=1, dtype=np.float32))
    audio_io.write_wav(p, x[:, 0], 48000)
    assert audio_io.load_audio(p, 16000).shape == (-(-16000 // 3),)
    with pytest.raises(FileNotFoundError):
        audio_io.load_audio(str(tmp_path / "missing.wav"))


def _make_exp(root, names, version="v2"):
    for d in ("sliced_audios", "sliced_audios_16k", f"{version}_extracted", "f0", "f0_voiced"):
        os.makedirs(os.path.join(root, d), exist_ok=True)
    for i, n in enumerate(names):
        x = np.sin(np.arange(1600 * (i + 2)) * 0.05).astype(np.float32) * 0.3
        audio_io.write_wav(os.path.join(root, "sliced_audios_16k", n), x, 16000)
        audio_io.write_wav(os.path.join(root, "sliced_audios", n), x, 48000)


def test_generate_filelist(tmp_path):
    root = str(tmp_path)
    _make_exp(root, ["0_0.wav", "0_1.wav", "1_0.wav"])
    for n in ("0_0", "0_1"):  # 1_0 misses its outputs -> dropped (set intersection, extract.py:63)
        np.save(os.path.join(root, "v2_extracted", n + ".npy"), np.zeros((3, 768), np.float32))
        np.save(os.path.join(root, "f0", n + ".wav.npy"), np.zeros(3, np.int64))
        np.save(os.path.join(root, "f0_voiced", n + ".wav.npy"), np.zeros(3))
    opts = extract.generate_filelist(True, root, "v2", 48000, rng=random.Random(0))
    assert len(opts) == 4
    assert sorted(o.split("|")[0].rsplit("/", 1)[1] for o in opts if "mute" not in o) == ["0_0.wav", "0_1.wav"]
    assert all(o.endswith("|0") and o.count("|") == 4 for o in opts)
    assert open(os.path.join(root, "filelist.txt")).read() == "\n".join(opts)
    opts2 = extract.generate_filelist(False, root, "v2", 48000, rng=random.Random(0))
    assert len(opts2) == 4 and all(o.count("|") == 2 for o in opts2)  # 1_0 has no features either


class _FakeF0(extract.FeatureInputAMD):
    def compute_f0(self, np_arr, f0_method, hop_length=160, f0_onnx=False):
        return np.abs(np_arr[::160]).astype(np.float64) * 1000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, root, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        extract.embed_file = lambda model, wav, version, device: np.full((wav.size // 320, 768), wav.size, np.float32)
        extract.run_extract(root, "v2", "rmvpe", None, _FakeF0(device="cpu"), "cpu", dist=dist, sample_rate=48000,
                            write_config=False)
        q.put((rank, "ok"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_extract_two_ranks_gloo(tmp_path):
    root = str(tmp_path)
    names = [f"{i}_0.wav" for i in range(5)]
    _make_exp(root, names)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=100) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == [(0, "ok"), (1, "ok")]
    fi = extract.FeatureInputAMD(device="cpu")
    for i, n in enumerate(names):  # every file done exactly once, outputs as the single-rank path
        x = audio_io.load_audio(os.path.join(root, "sliced_audios_16k", n))
        f0 = np.load(os.path.join(root, "f0_voiced", n + ".npy"))
        np.testing.assert_array_equal(f0, np.abs(x[::160]).astype(np.float64) * 1000)
        np.testing.assert_array_equal(np.load(os.path.join(root, "f0", n + ".npy")), fi.coarse_f0(f0))
        assert np.load(os.path.join(root, "v2_extracted", n.replace("wav", "npy"))).shape == (x.size // 320, 768)
    lines = open(os.path.join(root, "filelist.txt")).read().split("\n")
    assert len(lines) == len(names) + 2


def test_convert_batch_partition(tmp_path):
    from rvc_amd import convert

    class Fake:
        def __init__(self):
            self.done = []

        def convert_audio(self, src, dst, **kw):
            self.done.append(src)

    root = str(tmp_path)
    for i in range(5):
        audio_io.write_wav(os.path.join(root, f"f{i}.wav"), np.zeros(1000 * (i + 1), np.float32), 16000)
    pairs = convert.batch_files(root)
    assert [os.path.basename(o) for _, o in pairs] == [f"f{i}_output.wav" for i in range(5)]
    parts = [convert.convert_batch(Fake(), pairs, r, 2) for r in range(2)]
    assert sorted(p for part in parts for p, _ in part) == sorted(p for p, _ in pairs)
