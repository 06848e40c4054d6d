"""RMVPE alone on one 30 s clip (the headline shape), n passes: for rocprofv3 --kernel-trace --stats.

    rocprofv3 --kernel-trace --stats -d gpurun_out/rmprof -o run -- python3 scripts/rmvpe_prof.py [f64|fp32sa] [n]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rvc-maker_amd")]
from rvc_amd import synthetic  # noqa: E402
from rvc_amd.pipeline import VC, Config  # noqa: E402
from rvc_amd.rmvpe import RMVPEAMD  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "f64"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rm = RMVPEAMD(synthetic.rmvpe_state_dict(203), "cuda", precision=prec)
vc = VC(48000, Config("cuda"), rmvpe=rm)
audio = synthetic.synthetic_audio(30.0, seed=1000)
xp, _ = vc.filt(torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)).cuda(), vc.t_pad)
rm.f0_device(xp)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    rm.f0_device(xp)
e1.record()
torch.cuda.synchronize()
rm.check_error()
print(f"RMVPE {prec}: {e0.elapsed_time(e1) / n:.2f} ms per 30 s clip")
