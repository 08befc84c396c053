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
           "pg_result", "pg_partials", "pg_timing", "pg_image_header", "pg_image_segment", "pg_image_leaf", "pg_trace"]


def test_struct_layouts_match_header(tmp_path):
    src = tmp_path / "sz.c"
    lines = ["#include <stdio.h>", "#include <stddef.h>"] + [f'#include "{h}"' for h in HEADERS] + ["int main(void){"]
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


# ------------------------------------------------------------------ the relocatable plan image (pg_execute_image)

def image_from_bytes(**over):
    """A one-segment plan image written with struct.pack alone -- offsets, no pointers -- as a Java GpuPlanMaker fills a
    direct ByteBuffer with putInt / putLong: SELECT COUNT(*) WHERE col0 IN (dictIds 1, 3) over segment key 7.
    header @0 (120 B) | segment @120 (24 B) | leaf @144 (88 B) | ops @232 | agg @240 (48 B) | ids @288 (2 x int32)."""
    import struct
    f = dict(magic=abi.PG_IMAGE_MAGIC, abi=abi.PG_ABI_VERSION, n=296, segments_off=120, leaves_off=144, ops_off=232,
             aggs_off=240, ids_off=288, num_ids=2, num_segments=1)
    f.update(over)
    b = struct.pack("<IIQ8I4Q5Q", f["magic"], f["abi"], f["n"], f["num_segments"], 1, 1, 1, 0, 0, 0, 0,
                    0, 0, 0, 0, f["segments_off"], f["ops_off"], f["aggs_off"], 0, 0)
    b += struct.pack("<QIIQ", 7, 1000, 0, f["leaves_off"])
    b += struct.pack("<4I2iQ2q2d2IQ2I", abi.PG_LEAF_SV_SCAN, 0, 0, f["num_ids"], 0, 0, f["ids_off"], 0, 0, 0.0, 0.0,
                     0, 0, 0, 0, 0)
    b += struct.pack("<i", 0) + bytes(4)
    b += struct.pack("<6IqiIiI", abi.PG_AGG_COUNT, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
    b += struct.pack("<2i", 1, 3)
    assert len(b) == 296
    return b


def _run_image(lib, b, shift=0):
    import numpy as np
    arr = np.zeros(len(b) // 8 + 2, dtype=np.uint64).view(np.uint8)
    arr[shift:shift + len(b)] = np.frombuffer(b, dtype=np.uint8)
    res = C.POINTER(abi.pg_result)()
    rc = lib.pg_execute_image(arr.ctypes.data + shift, len(b), C.byref(res))
    buf = C.create_string_buffer(512)
    lib.pg_last_error(buf, 512)
    return rc, buf.value.decode()


def test_plan_image_from_python_bytes():
    """The image parser accepts a well-formed image built from bytes alone (it then stops at the device: no pg_init
    here -> PG_E_STATE) and names the first bad field of a malformed one (PG_E_INVALID) before touching a device."""
    lib = abi.declare(C.CDLL(LIB))
    rc, msg = _run_image(lib, image_from_bytes())
    assert rc == abi.PG_E_STATE, msg
    bad = [dict(magic=0x1234), dict(abi=abi.PG_ABI_VERSION - 1), dict(n=304), dict(segments_off=280),
           dict(segments_off=121), dict(leaves_off=250), dict(ids_off=290), dict(ids_off=292),
           dict(num_ids=0), dict(ops_off=4), dict(aggs_off=256), dict(num_segments=2)]
    for over in bad:
        b = image_from_bytes(**over)
        if "n" in over:
            b = b + bytes(over["n"] - len(b))
            b = b[:len(b) - 8]  # header says 304, the buffer holds 296
        rc, msg = _run_image(lib, b)
        assert rc == abi.PG_E_INVALID and msg.startswith("image"), (over, rc, msg)
    rc, msg = _run_image(lib, image_from_bytes(), shift=4)
    assert rc == abi.PG_E_INVALID and "aligned" in msg
    rc, msg = _run_image(lib, image_from_bytes()[:100])
    assert rc == abi.PG_E_INVALID


def test_plan_image_of_a_lowered_plan(sv_segment):
    """CPlan.image(): the lowered config-style plan as an image (values-mode IN literals shared by the segments are
    stored once) that the library's parser accepts."""
    import numpy as np
    from pinot_amd.plan import CPlan, Table
    from pinot_amd.query import parse
    t = Table("t", [sv_segment] * 3)
    vals = sv_segment.columns["column9"].dictionary.values
    lits = ", ".join(str(int(vals[i])) for i in (3, 7, 40, 41, 900))
    q = parse(f"SELECT column11, SUM(column1) FROM t WHERE column9 IN ({lits}) AND column3 > 5 "
              "GROUP BY column11 ORDER BY SUM(column1) DESC LIMIT 3")
    ids = {}

    def id_sets(col_id, dt, lit, keys):  # per-segment dictIds as the device lookup returns them
        from pinot_amd.plan import dict_id_set
        d = sv_segment.columns["column9"].dictionary
        row = dict_id_set(d, list(lit))
        out = np.zeros((len(keys), len(lit)), dtype=np.int32)
        out[:, :len(row)] = row
        return out, np.full(len(keys), len(row), dtype=np.uint32)
    cp = CPlan(t, q, t.segments, [11, 12, 13], trim="server", id_sets=id_sets)
    im, _ = cp.image()
    h = abi.pg_image_header.from_buffer_copy(im.tobytes()[:C.sizeof(abi.pg_image_header)])
    assert (h.magic, h.num_segments, h.num_leaves, h.image_bytes) == (abi.PG_IMAGE_MAGIC, 3, 2, im.size)
    assert h.flags & abi.PG_PLAN_EXACT_LIMIT and h.limit == 5000 and h.num_order == 1
    segs = (abi.pg_image_segment * 3).from_buffer_copy(im.tobytes()[h.segments_off:h.segments_off + 72])
    leaf_sets = [(abi.pg_image_leaf * 2).from_buffer_copy(im.tobytes()[s.leaves_off:s.leaves_off + 176]) for s in segs]
    assert [s.seg_key for s in segs] == [11, 12, 13]
    vo = {ls[0].values_off for ls in leaf_sets}
    assert len(vo) == 1 and 0 not in vo   # one literal array for every segment
    lib = abi.declare(C.CDLL(LIB))
    rc, msg = _run_image(lib, im.tobytes())
    assert rc == abi.PG_E_STATE, msg


def _decode_image_leaves(im):
    """(seg_key, num_docs, [(leaf fields..., ids tuple, values tuple)]) per segment of an image, offsets resolved."""
    import numpy as np
    b = im.tobytes()
    h = abi.pg_image_header.from_buffer_copy(b[:C.sizeof(abi.pg_image_header)])
    segs = (abi.pg_image_segment * h.num_segments).from_buffer_copy(
        b[h.segments_off:h.segments_off + C.sizeof(abi.pg_image_segment) * h.num_segments])
    out = []
    for s in segs:
        leaves = (abi.pg_image_leaf * h.num_leaves).from_buffer_copy(
            b[s.leaves_off:s.leaves_off + C.sizeof(abi.pg_image_leaf) * h.num_leaves]) if h.num_leaves else []
        row = []
        for x in leaves:
            ids = tuple(np.frombuffer(b, np.int32, x.num_ids, x.ids_off)) if x.ids_off else ()
            nv = x.num_values or x.num_ids
            vals = tuple(np.frombuffer(b, np.int64, nv, x.values_off)) if x.values_off else ()
            row.append((x.kind, x.col_id, x.exclusive, x.num_ids, x.lo, x.hi, x.ilo, x.ihi, x.dlo, x.dhi,
                        x.lo_inclusive, x.hi_inclusive, x.num_values, ids, vals))
        out.append((s.seg_key, s.num_docs, row))
    return h, out


def test_vectorized_image_matches_the_per_segment_writer(sv_segment):
    """The leaf table image (one copy of the [segment][leaf] table, pointers translated by region) holds exactly the
    plan the per-segment writer produces -- every leaf's fields, dictId lists and literals."""
    import numpy as np
    from pinot_amd.plan import CPlan, Table, dict_id_set
    from pinot_amd.query import parse
    t = Table("t", [sv_segment] * 3)
    vals = sv_segment.columns["column9"].dictionary.values
    lits = ", ".join(str(int(vals[i])) for i in (3, 7, 40, 41, 900))
    sql = (f"SELECT column11, SUM(column1) FROM t WHERE column9 IN ({lits}) AND column3 > 5 AND column1 <> 3 "
           "AND column5 = 'gFuH' GROUP BY column11 ORDER BY SUM(column1) DESC LIMIT 3")

    def id_sets(col_id, dt, lit, keys):
        row = dict_id_set(sv_segment.columns["column9"].dictionary, list(lit))
        out = np.zeros((len(keys), len(lit)), dtype=np.int32)
        out[:, :len(row)] = row
        return out, np.full(len(keys), len(row), dtype=np.uint32)
    cp = CPlan(t, parse(sql), t.segments, [11, 12, 13], trim="server", id_sets=id_sets)
    fast, _ = cp.image()
    slow = abi.build_image(cp.plan)
    hf, lf = _decode_image_leaves(fast)
    hs, ls = _decode_image_leaves(slow)
    assert lf == ls
    assert (hf.num_segments, hf.num_leaves, hf.flags, hf.limit) == (hs.num_segments, hs.num_leaves, hs.flags, hs.limit)


def test_one_hip_runtime_per_process():
    """The library and torch share one HIP runtime in a Python process (gpu.load_library loads torch first; both
    libamdhip64 builds have the SONAME libamdhip64.so.7): no second runtime mapped, whichever is imported first."""
    import subprocess
    import sys
    code = ("import pinot_amd.gpu as g; g.load_library(); import torch; "
            "print(len({l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}))")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == "1", out.stdout + out.stderr
