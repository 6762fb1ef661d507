"""ctypes binding of libaa.so (include/aa.h).

torch is imported first on purpose: the library's DT_NEEDED libamdhip64.so.7
then resolves to the HIP runtime torch already loaded, so device pointers from
torch tensors and the library's launches live in one runtime.  There is no
fallback: if the shared object is missing or does not load, every compute call
raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must precede loading libaa.so, see above)

# AA_LIB: an alternative build of the same library (tools/ab_build.py variants)
LIB_PATH = Path(os.environ.get("AA_LIB") or Path(__file__).resolve().parent / "libaa.so")
ABI_VERSION = 2

AA_PREC_F32 = 0
AA_PREC_BF16 = 1
AA_PREC_FP8 = 2
AA_PREC_BF16X3 = 3

AA_OP = {
    "conv2d": 1,
    "batchnorm": 2,
    "leakyrelu": 3,
    "maxpool2d": 4,
    "globalmaxpool2d": 5,
    "sigmoid": 6,
    "magtransform": 7,
    "relu": 8,
    "dense": 9,
}

# aa_status (include/aa.h)
AA_OK = 0
AA_ERR_INVALID = 1
AA_ERR_HIP = 2
AA_ERR_UNSUPPORTED = 3
AA_ERR_WORKSPACE = 4

AA_WIN_OK = 0
AA_WIN_NONFINITE = 1

AA_SN_NONFINITE = 1
AA_SN_RUN_OVERFLOW = 2


class AAError(RuntimeError):
    pass


class Window(C.Structure):
    _fields_ = [("src", C.c_int64), ("n_valid", C.c_int32), ("pad_left", C.c_int32)]


class FeConfig(C.Structure):
    _fields_ = [
        ("win_len", C.c_int32), ("n_fft", C.c_int32), ("hop", C.c_int32), ("n_mels", C.c_int32),
        ("normalize", C.c_int32), ("db_scale", C.c_int32), ("power", C.c_float),
        ("amin", C.c_float), ("top_db", C.c_float), ("mean_sub", C.c_int32),
        ("channels", C.c_int32), ("out_f16", C.c_int32),
    ]


class Layer(C.Structure):
    _fields_ = [
        ("op", C.c_int32), ("kh", C.c_int32), ("kw", C.c_int32), ("filters", C.c_int32),
        ("alpha", C.c_float), ("eps", C.c_float), ("off", C.c_int64 * 4),
    ]


class Node(C.Structure):
    _fields_ = [
        ("op", C.c_int32), ("in0", C.c_int32), ("in1", C.c_int32), ("kh", C.c_int32), ("kw", C.c_int32),
        ("sh", C.c_int32), ("sw", C.c_int32), ("pt", C.c_int32), ("pb", C.c_int32), ("pl", C.c_int32),
        ("pr", C.c_int32), ("filters", C.c_int32), ("act", C.c_int32), ("alpha", C.c_float),
        ("off", C.c_int64 * 2),
    ]


AA_G = {"conv": 1, "dwconv": 2, "maxpool": 3, "avgpool": 4, "gmaxpool": 5, "gavgpool": 6, "add": 7, "mul": 8,
        "affine": 9, "dense": 10, "pow": 11}
AA_GACT = {None: 0, "linear": 0, "relu": 1, "leaky": 2, "sigmoid": 3, "swish": 4}


class SnConfig(C.Structure):
    _fields_ = [("sr", C.c_int32), ("n_fft", C.c_int32), ("hop_length", C.c_int32),
                ("signal_width", C.c_double), ("freq_range", C.c_double)]


class SnComponent(C.Structure):
    _fields_ = [("left", C.c_int32), ("top", C.c_int32), ("width", C.c_int32), ("height", C.c_int32),
                ("area", C.c_int32), ("order", C.c_int32)]


class FlacInfo(C.Structure):
    _fields_ = [("sample_rate", C.c_int32), ("channels", C.c_int32), ("bits_per_sample", C.c_int32),
                ("total_frames", C.c_int64)]


class VorbisInfo(C.Structure):
    _fields_ = [("sample_rate", C.c_int32), ("channels", C.c_int32), ("blocksize_0", C.c_int32),
                ("blocksize_1", C.c_int32), ("total_frames", C.c_int64)]


_lib = None

_SIGS = {
    "aa_abi_version": (C.c_int, []),
    "aa_last_error": (C.c_char_p, []),
    "aa_fe_create": (C.c_int, [C.POINTER(FeConfig), C.c_void_p, C.POINTER(C.c_void_p)]),
    "aa_fe_destroy": (C.c_int, [C.c_void_p]),
    "aa_fe_n_frames": (C.c_int, [C.c_void_p]),
    "aa_fe_workspace_bytes": (C.c_size_t, [C.c_void_p, C.c_int32]),
    "aa_fe_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int32, C.c_void_p,
                            C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "aa_fe_n_stages": (C.c_int, [C.c_void_p]),
    "aa_fe_stage_info": (C.c_int, [C.c_void_p, C.c_int32, C.c_char_p, C.c_int32,
                                   C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "aa_fe_set_timing": (C.c_int, [C.c_void_p, C.c_uint32]),
    "aa_fe_stage_time": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_double),
                                   C.POINTER(C.c_int64)]),
    "aa_model_create": (C.c_int, [C.POINTER(Layer), C.c_int32, C.c_void_p, C.c_int64, C.c_int32,
                                  C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "aa_model_destroy": (C.c_int, [C.c_void_p]),
    "aa_model_n_outputs": (C.c_int, [C.c_void_p]),
    "aa_model_workspace_bytes": (C.c_size_t, [C.c_void_p, C.c_int32]),
    "aa_model_forward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_size_t, C.c_void_p]),
    "aa_model_n_stages": (C.c_int, [C.c_void_p]),
    "aa_model_stage_info": (C.c_int, [C.c_void_p, C.c_int32, C.c_char_p, C.c_int32,
                                      C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "aa_model_set_timing": (C.c_int, [C.c_void_p, C.c_uint32]),
    "aa_model_set_input_f16": (C.c_int, [C.c_void_p, C.c_int32]),
    "aa_model_stage_time": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_double),
                                      C.POINTER(C.c_int64)]),
    "aa_graph_create": (C.c_int, [C.POINTER(Node), C.c_int32, C.c_void_p, C.c_int64, C.c_int32, C.c_int32,
                                  C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "aa_graph_destroy": (C.c_int, [C.c_void_p]),
    "aa_graph_n_outputs": (C.c_int, [C.c_void_p]),
    "aa_graph_workspace_bytes": (C.c_size_t, [C.c_void_p, C.c_int32]),
    "aa_graph_forward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_size_t, C.c_void_p]),
    "aa_graph_n_stages": (C.c_int, [C.c_void_p]),
    "aa_graph_set_timing": (C.c_int, [C.c_void_p, C.c_uint32]),
    "aa_graph_time_stage": (C.c_int, [C.c_void_p, C.c_int32]),
    "aa_graph_stage_time": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "aa_graph_stage_info": (C.c_int, [C.c_void_p, C.c_int32, C.c_char_p, C.c_int32, C.POINTER(C.c_double),
                                      C.POINTER(C.c_double)]),
    "aa_track_mean": (C.c_int, [C.c_void_p, C.c_int32, C.c_int64, C.c_int32, C.c_void_p,
                                C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "aa_span_nonzero": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int32, C.c_void_p,
                                  C.c_void_p]),
    "aa_pcm_s16_to_f32": (C.c_int, [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p]),
    "aa_resample_poly": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                   C.c_int32, C.c_void_p, C.c_int64, C.c_void_p]),
    "aa_sn_create": (C.c_int, [C.POINTER(SnConfig), C.POINTER(C.c_void_p)]),
    "aa_sn_destroy": (C.c_int, [C.c_void_p]),
    "aa_sn_geometry": (C.c_int, [C.POINTER(SnConfig), C.POINTER(C.c_int32)]),
    "aa_sn_n_frames": (C.c_int64, [C.c_void_p, C.c_int64]),
    "aa_sn_workspace_bytes": (C.c_size_t, [C.c_void_p, C.c_int64]),
    "aa_sn_batch_workspace_bytes": (C.c_size_t, [C.c_void_p, C.c_int64, C.c_int32]),
    "aa_sn_run_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_int32,
                                  C.c_void_p, C.c_size_t, C.c_void_p, C.c_int32, C.c_int64, C.c_void_p, C.c_int32,
                                  C.c_void_p]),
    "aa_sn_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_size_t, C.c_void_p,
                            C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "aa_sn_spectrogram": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p]),
    "aa_sn_n_stages": (C.c_int, [C.c_void_p]),
    "aa_sn_stage_info": (C.c_int, [C.c_void_p, C.c_int32, C.c_char_p, C.c_int32, C.POINTER(C.c_double),
                                   C.POINTER(C.c_double)]),
    "aa_sn_set_timing": (C.c_int, [C.c_void_p, C.c_uint32]),
    "aa_sn_stage_time": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "aa_sn_components_from_mask": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_size_t,
                                             C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "aa_flac_info": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(FlacInfo)]),
    "aa_flac_decode": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]),
    "aa_vorbis_info": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(VorbisInfo)]),
    "aa_vorbis_decode": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]),
    "aa_read_file": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]),
    "aa_tracks_from_signals": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_double, C.c_int32, C.c_void_p,
                                         C.c_int64, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64)]),
}

EXPORTED = tuple(_SIGS)


def lib():
    """Load libaa.so once; raises if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise AAError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc gfx950)")
        h = C.CDLL(str(LIB_PATH))
        for name, (res, args) in _SIGS.items():
            try:
                f = getattr(h, name)
            except AttributeError:
                if os.environ.get("AA_LIB_AB"):
                    continue  # an older A/B build (tools/ab_head.py) lacks newer entry points
                raise AAError(f"{LIB_PATH} lacks {name}: a stale libaa.so (rebuild with __graft_entry__.build())")
            f.restype = res
            f.argtypes = args
        v = h.aa_abi_version()
        if v != ABI_VERSION:
            raise AAError(f"libaa.so ABI {v} != {ABI_VERSION}")
        _lib = h
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().aa_last_error().decode(errors="replace")
        raise AAError(f"{what or 'libaa'} failed ({rc}): {msg}")


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def dptr(t) -> int:
    if t is None:
        return 0
    if not t.is_cuda:
        raise AAError("libaa needs device tensors")
    if not t.is_contiguous():
        raise AAError("libaa needs contiguous tensors")
    return int(t.data_ptr())


class StageTiming:
    """Per-launch HIP-event timing of a plan/model handle (aa_fe_stage_* /
    aa_model_stage_*); subclasses set ``_timing_prefix`` and ``_h``."""
    _timing_prefix = ""

    def _fn(self, what):
        return getattr(lib(), f"{self._timing_prefix}_{what}")

    def n_stages(self) -> int:
        return self._fn("n_stages")(self._h)

    def stage_info(self, i: int):
        """(name, algorithmic flops per window, algorithmic bytes per window)"""
        name = C.create_string_buffer(96)
        fl, by = C.c_double(), C.c_double()
        check(self._fn("stage_info")(self._h, i, name, 96, C.byref(fl), C.byref(by)),
              f"{self._timing_prefix}_stage_info")
        return name.value.decode(), fl.value, by.value

    def set_timing(self, on=True, stages=None) -> None:
        """Time every stage (``on``) or only the stage indices in ``stages``
        (graphs: one stage, or every one)."""
        if self._timing_prefix == "aa_graph" and on and stages is not None:
            st = list(stages)
            if len(st) != 1:
                raise ValueError("graph models time one node or every node (stages=None), "
                                 f"not a subset of {len(st)}")
            check(lib().aa_graph_time_stage(self._h, int(st[0])), "aa_graph_time_stage")
            return
        mask = 0
        if on:
            mask = 0xFFFFFFFF if stages is None else sum(1 << int(i) for i in stages)
        check(self._fn("set_timing")(self._h, mask), f"{self._timing_prefix}_set_timing")

    def stage_time(self, i: int):
        """(total ms, launches) recorded for stage i since the last call"""
        ms, cnt = C.c_double(), C.c_int64()
        check(self._fn("stage_time")(self._h, i, C.byref(ms), C.byref(cnt)),
              f"{self._timing_prefix}_stage_time")
        return ms.value, cnt.value
