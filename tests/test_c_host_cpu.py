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


# ---- sanitizer builds of the host C/C++ (SURVEY §5 "sanitizers"): the safetensors reader the plain-C hosts share
# and the f0-file resampling behind rvc_f0_file_resample / rvc_vc_convert_ex (csrc/host_f0file.h), compiled for the
# CPU with AddressSanitizer + UndefinedBehaviorSanitizer and run on well-formed and malformed inputs.  Any report
# aborts the probe (halt_on_error), so a clean exit status is the check.
SAN = ["-fsanitize=address,undefined,float-cast-overflow", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
       "-g", "-O1"]
SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:exitcode=86:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
F0_PROBE = r'''
#include <cstdio>
#include <vector>
#include "host_f0file.h"
int main() {  // stdin: nrows, then nrows "t f0" pairs; stdout: the count, then the values (%.17g)
    long long n;
    if (scanf("%lld", &n) != 1) return 2;
    std::vector<float> rows(2 * (n > 0 ? n : 0));
    for (long long i = 0; i < 2 * n; ++i) if (scanf("%f", &rows[i]) != 1) return 2;
    std::vector<double> rep;
    int rc = rvc_host::f0_file_interp(n > 0 ? rows.data() : nullptr, n, rep);
    printf("%d %zu\n", rc, rep.size());
    for (double v : rep) printf("%.17g\n", v);
    return 0;
}
'''


def san_probe(tmp_path):
    src = tmp_path / "probe_san.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe_san"
    subprocess.run(["gcc", *SAN, "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "examples", "c_host"),
                    str(src), "-o", str(exe)], check=True)
    return exe


def test_reader_sanitized_wellformed_and_malformed(tmp_path):
    exe = san_probe(tmp_path)
    ck = synthetic.make_synth_ckpt(32000, "v1", seed=2)
    good = tmp_path / "m.safetensors"
    export_synth_safetensors(ck, str(good))
    r = subprocess.run([str(exe), str(good), "rvc_synth_cfg"], capture_output=True, text=True, env=SAN_ENV)
    assert r.returncode == 0, r.stderr[-3000:]
    assert set(parse(r.stdout)[1]) == set(ck["weight"])
    raw = good.read_bytes()
    hlen = int.from_bytes(raw[:8], "little")
    header = raw[8:8 + hlen]
    bad = {
        "empty": b"",
        "short": raw[:5],
        "hlen_past_end": (len(raw) * 4).to_bytes(8, "little") + raw[8:],
        "truncated_data": raw[: 8 + hlen + 16],
        "header_cut": (hlen // 2).to_bytes(8, "little") + header[: hlen // 2],
        "not_object": (4).to_bytes(8, "little") + b"[1] ",
        "no_colon": (9).to_bytes(8, "little") + b'{"a" 1}  ',
        "bad_dtype": _hdr({"a": {"dtype": "I8", "shape": [1], "data_offsets": [0, 1]}}, 1),
        "dtype_not_str": _hdr({"a": {"dtype": 5, "shape": [1], "data_offsets": [0, 4]}}, 4),
        "shape_not_list": _hdr({"a": {"dtype": "F32", "shape": 7, "data_offsets": [0, 4]}}, 4),
        "shape_junk": _hdr({"a": {"dtype": "F32", "shape": ["x"], "data_offsets": [0, 4]}}, 4),
        "five_dims": _hdr({"a": {"dtype": "F32", "shape": [1, 1, 1, 1, 1], "data_offsets": [0, 4]}}, 4),
        "huge_shape": _hdr({"a": {"dtype": "F32", "shape": [1 << 30, 1 << 30], "data_offsets": [0, 4]}}, 4),
        "neg_shape": _hdr({"a": {"dtype": "F32", "shape": [-1], "data_offsets": [0, 4]}}, 4),
        "offsets_outside": _hdr({"a": {"dtype": "F32", "shape": [2], "data_offsets": [0, 8]}}, 4),
        "offsets_reversed": _hdr({"a": {"dtype": "F32", "shape": [1], "data_offsets": [4, 0]}}, 4),
        "span_mismatch": _hdr({"a": {"dtype": "F32", "shape": [2], "data_offsets": [0, 4]}}, 8),
        "meta_not_ints": _hdr({"__metadata__": {"rvc_synth_cfg": "1,2"}}, 0),
        "meta_no_colon": (40).to_bytes(8, "little") + b'{"__metadata__":{"rvc_synth_cfg"}}      ',
    }
    for name, blob in bad.items():
        f = tmp_path / f"{name}.safetensors"
        f.write_bytes(blob)
        r = subprocess.run([str(exe), str(f), "rvc_synth_cfg"], capture_output=True, text=True, env=SAN_ENV,
                           timeout=30)
        # a clean refusal: exit 1 with a message, never a sanitizer report or a signal
        assert r.returncode == 1, (name, r.returncode, r.stderr[-2000:])
        assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, (name, r.stderr[-2000:])


def _hdr(obj, ndata):
    import json
    h = json.dumps(obj).encode()
    return len(h).to_bytes(8, "little") + h + b"\0" * ndata


def test_f0_file_resample_sanitized(tmp_path):
    """host_f0file.h under ASan + UBSan (float-cast-overflow included) vs the reference's numpy steps
    (convert.py:316-318, rvc_amd.pipeline.f0_override): bit-identical values; non-finite times refused."""
    from rvc_amd.pipeline import f0_override
    src = tmp_path / "f0.cpp"
    src.write_text(F0_PROBE)
    exe = tmp_path / "f0_san"
    subprocess.run(["g++", *SAN, "-ffp-contract=off", "-I", os.path.join(REPO, "rvc-maker_amd", "csrc"), str(src),
                    "-o", str(exe)], check=True)
    rng = np.random.default_rng(4)
    cases = [np.array([[0.0, 200.0], [0.4, 260.5], [0.9, 150.0], [1.6, 0.0], [2.0, 310.0]], np.float32),
             np.array([[0.25, 100.0]], np.float32), np.array([[3.0, 1.0], [3.0, 2.0]], np.float32)]
    for _ in range(12):
        n = int(rng.integers(2, 60))
        t = np.sort(rng.uniform(0, 9, n)).astype(np.float32)
        cases.append(np.stack([t, rng.uniform(0, 900, n).astype(np.float32)], 1))

    def run(rows):
        txt = f"{len(rows)}\n" + "\n".join(f"{a!r} {b!r}" for a, b in rows.tolist()) + "\n"
        r = subprocess.run([str(exe)], input=txt, capture_output=True, text=True, env=SAN_ENV, timeout=30)
        assert r.returncode == 0, r.stderr[-3000:]
        lines = r.stdout.split()
        return int(lines[0]), np.array([float(v) for v in lines[2:]], np.float64)

    for rows in cases:
        rc, got = run(rows)
        want, _ = f0_override(rows, 1)
        assert rc == 0
        np.testing.assert_array_equal(got, np.asarray(want, np.float64))
    for rows in (np.array([[np.nan, 1.0], [1.0, 2.0]], np.float32), np.array([[0.0, 1.0], [np.inf, 2.0]], np.float32),
                 np.array([[0.0, 1.0], [3e7, 2.0]], np.float32)):
        rc, got = run(rows)
        assert rc == -1 and got.size == 0
