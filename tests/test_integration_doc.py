"""INTEGRATION.md's ctypes binding cannot drift from the ABI: every
``ctypes.Structure`` in its code blocks is executed and compared field by
field (names, C types, offsets, sizeof) with include/aa.h's struct and with
aa_amd/_lib.py's binding of it."""
import ctypes as C
import re
from pathlib import Path

import pytest

from aa_amd import _lib

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "aa.h"
DOC = ROOT / "INTEGRATION.md"

# header struct -> the Python class name used by _lib.py and INTEGRATION.md
NAMES = {"aa_window": "Window", "aa_fe_config": "FeConfig", "aa_layer": "Layer",
         "aa_sn_config": "SnConfig", "aa_sn_component": "SnComponent", "aa_flac_stream_info": "FlacInfo",
         "aa_vorbis_stream_info": "VorbisInfo"}
CTYPES = {"int32_t": C.c_int32, "int64_t": C.c_int64, "float": C.c_float, "double": C.c_double}


def header_structs():
    """{struct name: [(field, ctype), ...]} parsed from include/aa.h."""
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = {}
    for name, body in re.findall(r"typedef struct (\w+) \{(.*?)\}", text, re.S):
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            ty, rest = decl.split(None, 1)
            for item in rest.split(","):
                item = item.strip()
                m = re.fullmatch(r"(\w+)(?:\[(\d+)\])?", item)
                assert m, (name, item)
                ct = CTYPES[ty]
                fields.append((m.group(1), ct * int(m.group(2)) if m.group(2) else ct))
        out[name] = fields
    return out


def doc_structs():
    """Every ctypes.Structure defined in INTEGRATION.md's python blocks."""
    ns = {"C": C}
    for block in re.findall(r"```python\n(.*?)```", DOC.read_text(), re.S):
        for cls in re.findall(r"^class \w+\(C\.Structure\):\n(?:    .*\n?)+", block, re.M):
            exec(cls, ns)
    return {k: v for k, v in ns.items() if isinstance(v, type) and issubclass(v, C.Structure)}


def _layout(cls):
    return [(f, t, getattr(cls, f).offset) for f, t in cls._fields_], C.sizeof(cls)


def _same_type(a, b):
    if issubclass(a, C.Array) or issubclass(b, C.Array):
        return issubclass(a, C.Array) and issubclass(b, C.Array) and a._type_ == b._type_ and a._length_ == b._length_
    return a == b


def test_header_parses():
    hs = header_structs()
    assert set(NAMES) <= set(hs)
    assert len(hs["aa_fe_config"]) == 12 and hs["aa_fe_config"][-1][0] == "out_f16"


@pytest.mark.parametrize("cname", sorted(NAMES))
def test_lib_binding_matches_header(cname):
    want = header_structs()[cname]
    py = getattr(_lib, NAMES[cname])
    assert [f for f, _ in py._fields_] == [f for f, _ in want]
    for (_, a), (_, b) in zip(py._fields_, want):
        assert _same_type(a, b), cname

    class Ref(C.Structure):
        _fields_ = want
    assert _layout(py)[1] == C.sizeof(Ref)
    assert [o for _, _, o in _layout(py)[0]] == [getattr(Ref, f).offset for f, _ in want]


def test_documented_structs_match_the_binding():
    docs = doc_structs()
    assert {"Window", "FeConfig", "SnConfig"} <= set(docs)
    hs = header_structs()
    inv = {v: k for k, v in NAMES.items()}
    for name, cls in docs.items():
        lib_cls = getattr(_lib, name)
        assert [f for f, _ in cls._fields_] == [f for f, _ in lib_cls._fields_], name
        for (_, a), (_, b) in zip(cls._fields_, lib_cls._fields_):
            assert _same_type(a, b), name
        assert C.sizeof(cls) == C.sizeof(lib_cls), name
        assert [f for f, _ in cls._fields_] == [f for f, _ in hs[inv[name]]], name
