"""libaa.so loads (CPU host, no GPU calls) and exports exactly the C ABI that
include/aa.h declares; argument validation fails loudly before any HIP call."""
import ctypes as C
import re
from pathlib import Path

import numpy as np

from aa_amd import _lib

HEADER = Path(__file__).resolve().parent.parent / "include" / "aa.h"


def declared():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|size_t|const char\*)\s+(aa_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    names = declared()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), n
    assert sorted(_lib.EXPORTED) == names


def test_abi_version_and_struct_sizes():
    assert _lib.lib().aa_abi_version() == _lib.ABI_VERSION
    assert C.sizeof(_lib.Window) == 16
    assert C.sizeof(_lib.Layer) == 6 * 4 + 4 * 8
    assert C.sizeof(_lib.FeConfig) == 12 * 4
    assert C.sizeof(_lib.SnConfig) == 32 and C.sizeof(_lib.SnComponent) == 24


def test_invalid_arguments_fail_without_gpu():
    L = _lib.lib()
    h = C.c_void_p()
    cfg = _lib.FeConfig(win_len=144000, n_fft=1000, hop=640, n_mels=160, normalize=1,
                        db_scale=1, power=2.0, amin=1e-10, top_db=80.0, mean_sub=0, channels=1)
    fb = np.zeros((160, 501), np.float32)
    rc = L.aa_fe_create(C.byref(cfg), fb.ctypes.data, C.byref(h))
    assert rc == 3 and b"n_fft" in L.aa_last_error()
    assert L.aa_model_create(None, 0, None, 0, 1, 1, 1, 0, C.byref(h)) == 1
    assert L.aa_fe_run(None, None, 0, None, 0, None, None, None, 0, None) == 1
    sc = _lib.SnConfig(sr=48000, n_fft=2048, hop_length=281, signal_width=0.25, freq_range=100.0)
    assert L.aa_sn_create(C.byref(sc), C.byref(h)) == 3 and b"n_fft" in L.aa_last_error()
    assert L.aa_sn_run(None, None, 0, None, 0, None, 0, None, None, None) == 1


def test_signal_geometry_matches_reference_arithmetic():
    """width / height / filter thresholds of src/identify_tracks.py:673-691
    (host-side plan values; no GPU call)."""
    from oracle.signal_oracle import signal_geometry
    L = _lib.lib()
    for sr, hop in [(48000, 281), (44100, 281), (16000, 281), (96000, 281), (48000, 640)]:
        sc = _lib.SnConfig(sr=sr, n_fft=4096, hop_length=hop, signal_width=0.25, freq_range=100.0)
        g = (C.c_int32 * 6)()
        assert L.aa_sn_geometry(C.byref(sc), g) == 0
        width, height, _ = signal_geometry(sr, hop)
        dh, dw = (height, width) if height and width else (3, 3)
        eh, ew = (height // 10, width) if height // 10 and width else (3, 3)
        assert tuple(g) == (dh, dw, eh, ew, int(0.65 * width) + 1, height - height // 10 + 1)


def test_read_file(tmp_path):
    """aa_read_file: the whole file in one call; AA_ERR_WORKSPACE (nothing
    read) past the buffer; AA_ERR_INVALID with the reason for a missing file."""
    import ctypes as C
    from aa_amd import _lib
    L = _lib.lib()
    data = bytes(range(256)) * 40 + b"tail"
    p = tmp_path / "f.bin"
    p.write_bytes(data)
    buf = C.create_string_buffer(len(data) + 7)
    got = C.c_int64(-1)
    assert L.aa_read_file(str(p).encode(), buf, len(data) + 7, C.byref(got)) == _lib.AA_OK
    assert got.value == len(data) and buf.raw[:len(data)] == data
    small = C.create_string_buffer(16)
    assert L.aa_read_file(str(p).encode(), small, 16, C.byref(got)) == _lib.AA_ERR_WORKSPACE
    assert got.value == len(data) and small.raw == b"\0" * 16
    empty = tmp_path / "empty.bin"
    empty.write_bytes(b"")
    assert L.aa_read_file(str(empty).encode(), small, 16, C.byref(got)) == _lib.AA_OK and got.value == 0
    assert L.aa_read_file(str(tmp_path / "missing.wav").encode(), small, 16, C.byref(got)) == _lib.AA_ERR_INVALID
    assert b"missing.wav" in L.aa_last_error()
