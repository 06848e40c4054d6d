"""BASELINE configs[3] on the device: a job of utterances sharded over 2 ranks (gloo transport, both ranks on this
GPU) through rvc_amd.shard.convert_utterances -- every utterance arrives at rank 0 exactly once, the bytes
received are the other rank's samples, the gathered waveforms are device tensors (the gather packs and unpacks on
the device, as its "nccl" branch does), and each is **bit-identical** to the 1-rank clip stream of the same job:
utterance i draws seed 17 + i wherever it runs.  Plus ``bench.py --gpus 2 --utterances`` end to end.
Reference: the batch loop /root/reference/main/inference/convert.py:129-135 (one pipeline() call per file)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from rvc_amd import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SECS = [30.0, 30.0, 12.0, 30.0, 30.0]  # four 30 s utterances and one ragged 12 s one


def _models(dev):
    from rvc_amd.contentvec import ContentVecAMD
    from rvc_amd.pipeline import VC, Config
    from rvc_amd.rmvpe import RMVPEAMD
    from rvc_amd.synth import SynthesizerAMD
    hub = ContentVecAMD(synthetic.make_contentvec_ckpt(91), dev)
    rm = RMVPEAMD(synthetic.rmvpe_state_dict(92), dev)
    net_g = SynthesizerAMD(synthetic.make_synth_ckpt(48000, "v2", seed=93), dev)
    return hub, net_g, VC(48000, Config(dev), rmvpe=rm)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _clip(i):
    return torch.from_numpy(synthetic.synthetic_audio(SECS[i], seed=1000 + i)).to(DEV)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from rvc_amd.shard import convert_utterances, shard_utterances
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hub, net_g, vc = _models(DEV)
        shards = shard_utterances([int(s * 16000) for s in SECS], world)
        stats = {}
        got = convert_utterances(vc, hub, net_g, 0, [_clip(i) for i in shards[rank]], shards, dist, seed=17,
                                 stats=stats)
        torch.cuda.synchronize()
        vc.check_errors()
        msg = {"rank": rank, "stats": stats, "shards": shards}
        if rank == 0:
            msg["devices"] = [w.device.type for w in got]
            msg["got"] = [w.cpu().numpy() for w in got]
            # the same job on one rank: one clip stream over every utterance, no gather
            ref = convert_utterances(vc, hub, net_g, 0, [_clip(i) for i in range(len(SECS))], [list(range(len(SECS)))],
                                     None, seed=17)
            torch.cuda.synchronize()
            vc.check_errors()
            msg["ref"] = [w.cpu().numpy() for w in ref]
        q.put(msg)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_two_ranks_bit_identical_to_one_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msgs = {}
    for _ in range(2):
        m = q.get(timeout=350)
        msgs[m["rank"]] = m
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m0, m1 = msgs[0], msgs[1]
    shards = m0["shards"]
    assert sorted(shards[0] + shards[1]) == list(range(len(SECS))) and shards[1]  # both ranks work
    got, ref = m0["got"], m0["ref"]
    assert len(got) == len(SECS) and all(d == "cuda" for d in m0["devices"])
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g.shape == r.shape, (i, g.shape, r.shape)
        if SECS[i] == 30.0:
            assert g.shape == (1439040,), g.shape
        np.testing.assert_array_equal(g, r, err_msg=f"utterance {i}")
    # distinct noise per utterance: the equal-length utterances differ (their inputs and seeds differ)
    assert not np.array_equal(got[0], got[1])
    # bytes moved = exactly rank 1's samples, once
    sent = 4 * sum(ref[i].size for i in shards[1])
    assert m1["stats"]["bytes_sent"] == sent and m0["stats"]["bytes_recv"] == sent
    assert m0["stats"]["bytes_sent"] == 0 and m1["stats"]["bytes_recv"] == 0


@pytest.mark.timeout(420)
def test_bench_utterances_two_ranks():
    """``bench.py --gpus 2 --utterances 4`` (BASELINE configs[3]'s mode, two ranks on one GPU: gloo transport):
    one contract line, every utterance gathered once, rank 1's samples received."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--utterances", "4",
                        "--seconds", "5", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=400, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["value"] > 0
    assert line["waveforms_gathered_per_step"] == 4 and line["utterances_per_rank"] == 2
    out_len = round(line["config"]["output_seconds_per_clip"] * 48000)
    assert line["gather_bytes_recv_per_step"] == 4 * 2 * out_len
