"""CPU checks of the plain-C hosts (examples/c_host): the safetensors reader they share parses an export of
each checkpoint into the same names, dtypes, shapes and bytes as Python, metadata ints included."""
import os
import subprocess

import numpy as np
import torch

from rvc_amd import synthetic
from rvc_amd.native import export_safetensors, export_synth_safetensors, synth_cfg

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = r'''
#include "safetensors_min.h"
int main(int argc, char** argv) {
    char* keep;
    Model m = load_safetensors(argv[1], argc > 2 ? argv[2] : NULL, &keep);
    printf("cfg");
    for (int i = 0; i < m.ncfg; ++i) printf(" %d", m.cfg[i]);
    printf("\n");
    for (int i = 0; i < m.n; ++i) {
        const rvc_param* p = &m.params[i];
        long long n = 1;
        for (int d = 0; d < p->ndim; ++d) n *= p->shape[d];
        const int es = p->dtype == RVC_DT_F16 ? 2 : (p->dtype == RVC_DT_F64 ? 8 : 4);
        unsigned long long h = 1469598103934665603ull;  /* FNV-1a of the tensor bytes */
        for (long long b = 0; b < n * es; ++b) h = (h ^ ((const unsigned char*)p->data)[b]) * 1099511628211ull;
        printf("%s %d %d", p->name, p->dtype, p->ndim);
        for (int d = 0; d < p->ndim; ++d) printf(" %lld", (long long)p->shape[d]);
        printf(" %llu\n", h);
    }
    return 0;
}
'''


def fnv(b: bytes) -> int:
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def probe(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-O1", "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "examples", "c_host"),
                    str(src), "-o", str(exe)], check=True)
    return exe


def parse(out):
    lines = out.strip().split("\n")
    cfg = [int(v) for v in lines[0].split()[1:]]
    rows = {}
    for ln in lines[1:]:
        f = ln.split()
        nd = int(f[2])
        rows[f[0]] = (int(f[1]), tuple(int(v) for v in f[3:3 + nd]), int(f[3 + nd]))
    return cfg, rows


def test_reader_matches_python_on_synth_export(tmp_path):
    exe = probe(tmp_path)
    ck = synthetic.make_synth_ckpt(32000, "v1", seed=2)
    export_synth_safetensors(ck, str(tmp_path / "m.safetensors"))
    r = subprocess.run([str(exe), str(tmp_path / "m.safetensors"), "rvc_synth_cfg"], capture_output=True, text=True,
                       check=True)
    cfg, rows = parse(r.stdout)
    assert cfg == list(np.frombuffer(bytes(synth_cfg(ck)), dtype=np.int32))
    W = ck["weight"]
    assert set(rows) == set(W)
    for k, v in W.items():
        a = v.detach().cpu().contiguous().numpy()
        dt = {np.dtype(np.float16): 1, np.dtype(np.float32): 0}[a.dtype]
        shape = a.shape if a.ndim else (1,)
        assert rows[k] == (dt, tuple(shape), fnv(a.tobytes())), k


def test_reader_f64_and_metadata(tmp_path):
    exe = probe(tmp_path)
    t = {"a": torch.arange(6, dtype=torch.float64).reshape(2, 3), "b.weight": torch.ones(4, 1, 3)}
    export_safetensors(t, str(tmp_path / "x.safetensors"), rvc_contentvec_cfg=[768, 12, 16, 0])
    r = subprocess.run([str(exe), str(tmp_path / "x.safetensors"), "rvc_contentvec_cfg"], capture_output=True,
                       text=True, check=True)
    cfg, rows = parse(r.stdout)
    assert cfg == [768, 12, 16, 0]
    assert rows["a"] == (2, (2, 3), fnv(t["a"].numpy().tobytes()))
    assert rows["b.weight"] == (0, (4, 1, 3), fnv(t["b.weight"].numpy().tobytes()))
