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
    assert ctypes.sizeof(_lib.Conv1dArgs) == 6 * 8 + 10 * 8 + 12 * 4 + 4 * 4 + 18 * 4 + 8 + 2 * 4
    assert ctypes.sizeof(_lib.AttnArgs) == 7 * 8 + 13 * 8 + 4 * 4


def test_errors_are_reported_without_gpu():
    lib = _lib.load()
    a = _lib.Conv1dArgs()  # all-null -> EINVAL, no device touched
    rc = lib.rvc_conv1d(ctypes.byref(a), None, 0, None)
    assert rc == -22
    assert b"null" in lib.rvc_last_error()
    assert lib.rvc_version() >= 1


def test_struct_layouts_match_c_compiler(tmp_path):
    import subprocess
    fields = {"rvc_conv1d_args": [f[0] for f in _lib.Conv1dArgs._fields_],
              "rvc_attn_args": [f[0] for f in _lib.AttnArgs._fields_],
              "rvc_f0_post": [f[0] for f in _lib.F0Post._fields_],
              "rvc_denoise_args": [f[0] for f in _lib.DenoiseArgs._fields_]}
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
    for cls in (_lib.Conv1dArgs, _lib.AttnArgs, _lib.F0Post, _lib.DenoiseArgs):
        want.append(ctypes.sizeof(cls))
        want += [getattr(cls, f[0]).offset for f in cls._fields_]
    assert got == want
