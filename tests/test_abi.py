"""The drop-in boundary: libpinot_gpu.so loads and exports every entry point include/pinot_gpu.h declares, and the
ctypes mirror (pinot_amd/abi.py, what a JNI / ctypes binding sees) has the same struct layouts as the C header.
No compute calls: this runs without a GPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

from pinot_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include")))
           if h.endswith(".h")]
LIB = os.path.join(ROOT, "pinot_amd", "libpinot_gpu.so")


def header_functions():
    """Every entry point declared by include/*.h (pinot_gpu.h: the query path; pinot_codec.h: the chunk codecs)."""
    names = set()
    for h in HEADERS:
        with open(h) as f:
            names |= set(re.findall(r"^(?:int|uint32_t)\s+(pg_\w+)\s*\(", f.read(), flags=re.M))
    return sorted(names)


def test_header_and_mirror_agree():
    assert header_functions() == sorted(abi.EXPORTED)


def test_library_exports_every_symbol():
    assert os.path.exists(LIB), "build first: python -c 'import __graft_entry__ as g; g.build()'"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s+(pg_\w+)$", out, flags=re.M))
    missing = set(header_functions()) - exported
    assert not missing, missing
    lib = C.CDLL(LIB)
    abi.declare(lib)
    assert lib.pg_abi_version() == abi.PG_ABI_VERSION
    # error path without touching the device: pg_last_error on a fresh thread is empty
    buf = C.create_string_buffer(64)
    assert lib.pg_last_error(buf, 64) >= 0


def test_library_is_gfx950_only():
    with open(LIB, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"gfx1100", b"sm_"):
        assert b"amdhsa--" + other not in blob


STRUCTS = ["pg_col_desc", "pg_leaf", "pg_agg", "pg_key", "pg_segment_ref", "pg_order", "pg_plan", "pg_stats",
           "pg_result", "pg_partials", "pg_timing"]


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "sz.c"
    header = os.path.join(ROOT, "include", "pinot_gpu.h")
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{header}"', "int main(void){"]
    for s in STRUCTS:
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for name, _ in getattr(abi, s)._fields_:
            lines.append(f'printf("{s}.{name} %zu\\n", offsetof({s}, {name}));')
    lines.append("return 0;}")
    src.write_text("\n".join(lines))
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    for s in STRUCTS:
        t = getattr(abi, s)
        assert int(got[s]) == C.sizeof(t), s
        for name, _ in t._fields_:
            assert int(got[f"{s}.{name}"]) == getattr(t, name).offset, (s, name)


def test_oracle_is_not_linked_into_product():
    out = subprocess.run(["nm", "-D", LIB], capture_output=True, text=True, check=True).stdout
    assert "orc_" not in out
    ldd = subprocess.run(["ldd", LIB], capture_output=True, text=True).stdout
    assert "pinot_oracle" not in ldd
    import pinot_amd.gpu as g
    with open(g.__file__) as f:
        assert "oracle" not in f.read().replace("no fallback", "")
