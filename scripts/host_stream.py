"""Host issue time of the clip stream vs its GPU time: per-clip host cost of issue_front / back issue."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rvc-maker_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from rvc_amd import synthetic  # noqa: E402

dev = "cuda:0"
vc, hub, net_g = bench.build_models(dev)
clips = [torch.from_numpy(synthetic.synthetic_audio(30.0, seed=1000 + c)).to(dev) for c in range(8)]
vc.pipeline_device_stream(hub, net_g, 0, clips[:2], 0, "v2", 0.33)
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    outs = vc.pipeline_device_stream(hub, net_g, 0, clips, 0, "v2", 0.33)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"8 clips: host issue {1e3 * (t1 - t0):.1f} ms, total {1e3 * (t2 - t0):.1f} ms "
          f"({1e3 * (t2 - t0) / 8:.1f} ms per clip, host {1e3 * (t1 - t0) / 8:.1f} ms per clip)", flush=True)
# per-call host issue for comparison
t0 = time.perf_counter()
for c in clips:
    vc.pipeline_device(hub, net_g, 0, c, 0, "v2", 0.33)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"per-call 8 clips: host issue {1e3 * (t1 - t0):.1f} ms, total {1e3 * (t2 - t0):.1f} ms")
# stream event timeline: does the back stream wait for the front?
evs = []
vc.pipeline_device_stream(hub, net_g, 0, clips, 0, "v2", 0.33, events=evs)
torch.cuda.synchronize()
t = {(r, g): e for r, g, e in evs}
base = t[("front_start", 0)]
for g in range(len(clips)):
    f = (base.elapsed_time(t[("front_start", g)]), base.elapsed_time(t[("front_end", g)]))
    b = (base.elapsed_time(t[("back_start", g)]), base.elapsed_time(t[("back_end", g)]))
    print(f"clip {g}: front {f[0]:7.1f} -> {f[1]:7.1f} ({f[1] - f[0]:5.1f} ms)  back {b[0]:7.1f} -> {b[1]:7.1f} "
          f"({b[1] - b[0]:5.1f} ms)")
