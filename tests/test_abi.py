"""CPU-side checks of the C ABI: the library loads and exports every symbol include/rvc_amd.h declares."""
import ctypes
import os
import re

from rvc_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(REPO, "include", "rvc_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rvc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 10
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(declared_symbols()) <= set(_lib.SIGNATURES), set(declared_symbols()) - set(_lib.SIGNATURES)


def test_struct_layouts_match_header():
    # sizes of the POD structs as the C compiler lays them out (checked by a tiny host probe below)
    assert ctypes.sizeof(_lib.Conv1dArgs) == 6 * 8 + 10 * 8 + 12 * 4 + 4 * 4 + 18 * 4 + 8 + 2 * 4 + 2 * 8 + 3 * 8 + 4 * 4 + 2 * 8
    assert ctypes.sizeof(_lib.AttnArgs) == 7 * 8 + 13 * 8 + 4 * 4


def test_errors_are_reported_without_gpu():
    lib = _lib.load()
    a = _lib.Conv1dArgs()  # all-null -> EINVAL, no device touched
    rc = lib.rvc_conv1d(ctypes.byref(a), None, 0, None)
    assert rc == -22
    assert b"null" in lib.rvc_last_error()
    assert lib.rvc_version() >= 1


def test_model_api_rejects_bad_arguments_without_gpu():
    import ctypes as C
    lib = _lib.load()
    cfg = _lib.SynthCfg()
    assert lib.rvc_load_synth(None, None, 0, C.byref(cfg)) == -22
    assert b"null" in lib.rvc_last_error()
    assert lib.rvc_synth_infer(None, None, None, None, 1, 1, None, None, None, 0, None, None) == -22
    assert b"no synthesizer" in lib.rvc_last_error()
    assert lib.rvc_synth_out_len(None, 10) == -1
    assert lib.rvc_ctx_set_precision(None, 0) == -22
    lib.rvc_ctx_destroy(None)  # no-op
    assert lib.rvc_load_contentvec(None, None, 0, None) == -22
    assert lib.rvc_contentvec_forward(None, None, 1, 16000, 12, 0, None, None) == -22
    assert lib.rvc_load_rmvpe(None, None, 0) == -22
    assert lib.rvc_rmvpe_forward(None, None, 1, 16000, None, None) == -22
    assert lib.rvc_rmvpe_check(None) == -22
    assert lib.rvc_load_crepe(None, None, 0) == -22
    assert lib.rvc_crepe_f0(None, None, 16000, None, 0, 0.0, None, None, None, None, None) == -22


def test_model_api_size_queries():
    from rvc_amd import contentvec
    lib = _lib.load()
    for n in (400, 16000, 160000 + 37, 480000):
        assert lib.rvc_contentvec_frames(n) == contentvec.frames(n)
        F = 1 + n // 160
        assert lib.rvc_rmvpe_frames(n) == F
        assert lib.rvc_rmvpe_salience_ld(n) == 32 * ((F - 1) // 32 + 1)
    assert lib.rvc_contentvec_frames(100) == 0


def test_synth_cfg_from_checkpoint_config():
    from rvc_amd import synthetic
    from rvc_amd.native import synth_cfg
    ck = synthetic.make_synth_ckpt(48000, "v2", seed=1)
    c = synth_cfg(ck)
    cfg = ck["config"]
    assert (c.inter_channels, c.hidden_channels, c.filter_channels, c.n_heads, c.n_layers, c.kernel_size) == \
        tuple(cfg[2:8])
    assert [c.upsample_rates[i] for i in range(c.n_upsamples)] == list(cfg[12])
    assert [c.upsample_kernel_sizes[i] for i in range(c.n_upsamples)] == list(cfg[14])
    assert [c.resblock_kernel_sizes[j] for j in range(c.n_resblocks)] == list(cfg[10])
    assert [[c.resblock_dilation_sizes[j][m] for m in range(c.n_dilations)] for j in range(c.n_resblocks)] == \
        [list(d) for d in cfg[11]]
    assert (c.upsample_initial_channel, c.gin_channels, c.sr) == (cfg[13], cfg[16], cfg[17])
    assert c.spk_embed_dim == ck["weight"]["emb_g.weight"].shape[0]


def test_struct_layouts_match_c_compiler(tmp_path):
    import subprocess
    fields = {"rvc_conv1d_args": [f[0] for f in _lib.Conv1dArgs._fields_],
              "rvc_attn_args": [f[0] for f in _lib.AttnArgs._fields_],
              "rvc_f0_post": [f[0] for f in _lib.F0Post._fields_],
              "rvc_denoise_args": [f[0] for f in _lib.DenoiseArgs._fields_],
              "rvc_param": [f[0] for f in _lib.Param._fields_],
              "rvc_synth_cfg": [f[0] for f in _lib.SynthCfg._fields_],
              "rvc_contentvec_cfg": [f[0] for f in _lib.ContentVecCfg._fields_],
              "rvc_vc_args": [f[0] for f in _lib.VcArgs._fields_],
              "rvc_ivf_index": [f[0] for f in _lib.IvfIndex._fields_],
              "rvc_conv64_args": [f[0] for f in _lib.Conv64Args._fields_],
              "rvc_wino64_args": [f[0] for f in _lib.Wino64Args._fields_]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rvc_amd.h"', "int main(void){"]
    for st, fs in fields.items():
        lines.append(f'printf("%zu\\n", sizeof({st}));')
        for f in fs:
            lines.append(f'printf("%zu\\n", offsetof({st}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = []
    for cls in (_lib.Conv1dArgs, _lib.AttnArgs, _lib.F0Post, _lib.DenoiseArgs, _lib.Param, _lib.SynthCfg, _lib.ContentVecCfg,
                _lib.VcArgs, _lib.IvfIndex, _lib.Conv64Args, _lib.Wino64Args):
        want.append(ctypes.sizeof(cls))
        want += [getattr(cls, f[0]).offset for f in cls._fields_]
    assert got == want


def test_f0_file_resample_matches_reference_numpy():
    """rvc_f0_file_resample (the f0-file values rvc_vc_convert_ex writes) vs the reference's own numpy steps
    (convert.py:316-318, restated in rvc_amd.pipeline.f0_override): bit-identical, including rows starting after
    0 s (np.interp's left value), exact grid hits and rounding of the frame count."""
    import numpy as np
    from rvc_amd.pipeline import f0_override
    lib = _lib.load()
    rng = np.random.default_rng(3)
    cases = [np.array([[0.0, 200.0], [0.4, 260.5], [0.9, 150.0], [1.6, 0.0], [2.0, 310.0]], np.float32),
             np.array([[0.25, 100.0]], np.float32),
             np.array([[0.013, 80.0], [0.505, 400.0], [3.3333, 123.456]], np.float32)]
    for _ in range(20):
        n = int(rng.integers(2, 40))
        t = np.sort(rng.uniform(0, 8, n)).astype(np.float32)
        cases.append(np.stack([t, rng.uniform(0, 900, n).astype(np.float32)], 1))
    for rows in cases:
        want, off = f0_override(rows, 1)
        out = np.zeros(max(len(want), 1), np.float64)
        n = lib.rvc_f0_file_resample(ctypes.c_void_p(rows.ctypes.data), rows.shape[0], ctypes.c_void_p(out.ctypes.data),
                                     out.size)
        assert n == len(want) and off == 100
        np.testing.assert_array_equal(out[:n], np.asarray(want, np.float64))


def test_bench_pass_set_parser():
    """bench.py reads each split-operand kernel's pass set from its template arguments (torch.profiler names)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench._pass_set("conv_x6_kernel<2, 8, 4, 2, 6, 3, true, false>") == 16
    assert bench._pass_set("conv_x6_kernel<2, 4, 4, 2, 3, 6, false, true>") == 7
    assert bench._pass_set("conv_x6_kernel<2, 4, 4, 2, 3, 6, false, false>") == 6
    assert bench._pass_set("conv_x6_kernel<2, 2, 1, 4, 3, 1, false, false>") == 1
    assert bench._pass_set("resblock_x6_kernel<64, 6, false>") == 6
    assert bench._pass_set("resblock_x6_kernel<32, 3, true>") == 16
