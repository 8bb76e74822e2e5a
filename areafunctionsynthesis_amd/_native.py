"""ctypes binding of libafs.so (include/afs.h).

The library is built in-tree by ``areafunctionsynthesis_amd.build``.  There is no
fallback: if the library or a HIP device is missing, the calls raise.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# (AFS_LIB: another in-tree build of the same library, for A/B timing of kernel variants)
LIB_PATH = os.environ.get("AFS_LIB") or os.path.join(HERE, "libafs.so")

AFS_OK = 0
STATUS = {0: "ok", 1: "invalid argument", 2: "no HIP device", 3: "HIP runtime error",
          4: "out of device memory", 5: "unsupported configuration"}
AFS_SOLVER_CHOLESKY = 0
AFS_SOLVER_TREE = 1
AFS_SOLVER_SOR = 2
AFS_PLAN_WORDS = 16  # afs.h
AFS_PLAN_HOP_BYTES = 544  # afs.h
AFS_PLAN_HOP_MIN = 32  # afs.h
AFS_FP64 = 0
AFS_ASYNC = 0x1
AFS_PROFILE = 0x2
AFS_LANES_16 = 0x4
AFS_LANES_64 = 0x8
AFS_COMM_ID_BYTES = 128

# Every symbol include/afs.h declares.
EXPORTED = (
    "afs_abi_version", "afs_config_default", "afs_status_string", "afs_create", "afs_destroy",
    "afs_last_error", "afs_set_stream", "afs_lanes_per_utterance", "afs_synthesis_kernel", "afs_synchronize", "afs_synthesize",
    "afs_session_create", "afs_session_synthesize", "afs_session_reset", "afs_session_destroy",
    "afs_af_to_frames", "afs_to_int16", "afs_target_sequence_default", "afs_target_sequence_samples",
    "afs_play_target_sequences", "afs_rng_draws", "afs_noise_plans", "afs_noise_plan_hops", "afs_plan_hop_words", "afs_tube_interpolate", "afs_session_rng_draws", "afs_kernel_times",
    "afs_kernel_times_ex",
    "afs_shard_range", "afs_comm_unique_id", "afs_comm_create", "afs_comm_create_all", "afs_comm_destroy",
    "afs_gather_pcm", "afs_comm_fence", "afs_comm_synchronize", "afs_comm_gather_times", "afs_multi_synthesize",
)


class AfsOptions(ctypes.Structure):
    _fields_ = [("turbulence_losses", ctypes.c_int32), ("soft_walls", ctypes.c_int32),
                ("generate_noise_sources", ctypes.c_int32), ("radiation_from_skin", ctypes.c_int32),
                ("piriform_fossa", ctypes.c_int32), ("inner_length_corrections", ctypes.c_int32),
                ("transvelar_coupling", ctypes.c_int32), ("glottis_loss", ctypes.c_int32),
                ("glottis_model", ctypes.c_int32), ("flow_separation_area_ratio", ctypes.c_double)]


class AfsTargetSequence(ctypes.Structure):
    _fields_ = [("stationary_s", ctypes.c_double * 4), ("transition_s", ctypes.c_double * 3),
                ("f0_hz", ctypes.c_double * 4), ("lung_pressure_dpa", ctypes.c_double),
                ("glottis", ctypes.c_double * 6)]


class AfsConfig(ctypes.Structure):
    _fields_ = [("sampling_rate_hz", ctypes.c_double), ("precision", ctypes.c_int32),
                ("solver", ctypes.c_int32), ("device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("options", AfsOptions)]


class AfsReport(ctypes.Structure):
    _fields_ = [("device_ms", ctypes.c_double), ("samples", ctypes.c_int64),
                ("nonfinite_utterances", ctypes.c_int32), ("kernel", ctypes.c_int32)]


class AfsKernelTiming(ctypes.Structure):
    _fields_ = [("synth_ms", ctypes.c_double), ("synth_launches", ctypes.c_int32),
                ("plan_ms", ctypes.c_double), ("plan_launches", ctypes.c_int32),
                ("output_ms", ctypes.c_double), ("output_launches", ctypes.c_int32)]


class AfsError(RuntimeError):
    pass


_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libafs.so, building it first when it is absent (never a CPU substitute)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        from . import build as _build
        _build.build()
    if not os.path.exists(path):
        raise AfsError(f"libafs.so not found at {path}; run python -m areafunctionsynthesis_amd.build")
    lib = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    lib.afs_abi_version.restype = ctypes.c_int32
    lib.afs_config_default.argtypes = [ctypes.POINTER(AfsConfig)]
    lib.afs_status_string.restype = ctypes.c_char_p
    lib.afs_status_string.argtypes = [ctypes.c_int]
    lib.afs_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(AfsConfig)]
    lib.afs_destroy.argtypes = [vp]
    lib.afs_last_error.restype = ctypes.c_char_p
    lib.afs_last_error.argtypes = [vp]
    lib.afs_set_stream.argtypes = [vp, vp]
    lib.afs_lanes_per_utterance.argtypes = [vp, ctypes.c_int32]
    lib.afs_lanes_per_utterance.restype = ctypes.c_int32
    lib.afs_synthesis_kernel.argtypes = [vp, ctypes.c_int32]
    lib.afs_synthesis_kernel.restype = ctypes.c_char_p
    lib.afs_synchronize.argtypes = [vp]
    lib.afs_synthesize.argtypes = [vp, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp,
                                   ctypes.POINTER(AfsReport)]
    lib.afs_rng_draws.argtypes = [vp, ctypes.c_int32, vp]
    lib.afs_tube_interpolate.argtypes = [vp, vp, vp, vp, ctypes.c_int32, vp, vp]
    lib.afs_noise_plans.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                    ctypes.c_int64, vp]
    lib.afs_noise_plan_hops.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                        ctypes.c_int64, vp, vp]
    lib.afs_plan_hop_words.argtypes = [vp, vp, vp, ctypes.c_int32, vp]
    lib.afs_session_rng_draws.argtypes = [vp, vp]
    lib.afs_session_create.argtypes = [vp, ctypes.c_int32, vp, ctypes.POINTER(vp)]
    lib.afs_session_synthesize.argtypes = [vp, vp, ctypes.c_int32, vp, vp, ctypes.POINTER(ctypes.c_int32),
                                           ctypes.POINTER(AfsReport)]
    lib.afs_session_reset.argtypes = [vp, vp]
    lib.afs_session_destroy.argtypes = [vp]
    lib.afs_af_to_frames.argtypes = [vp, vp, ctypes.c_int64, vp]
    lib.afs_to_int16.argtypes = [vp, vp, ctypes.c_int64, vp]
    lib.afs_target_sequence_default.argtypes = [ctypes.POINTER(AfsTargetSequence)]
    lib.afs_target_sequence_default.restype = None
    lib.afs_target_sequence_samples.argtypes = [ctypes.POINTER(AfsTargetSequence), ctypes.c_double]
    lib.afs_target_sequence_samples.restype = ctypes.c_int64
    lib.afs_play_target_sequences.argtypes = [vp, vp, ctypes.c_int32, vp, ctypes.POINTER(AfsTargetSequence), vp,
                                              ctypes.c_int32, vp, vp, ctypes.POINTER(AfsReport)]
    i32p, i64p, dp = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)
    lib.afs_kernel_times.argtypes = [vp, dp, i32p, dp, i32p]
    lib.afs_kernel_times_ex.argtypes = [vp, ctypes.POINTER(AfsKernelTiming)]
    lib.afs_shard_range.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, i64p, i64p]
    lib.afs_shard_range.restype = None
    lib.afs_comm_unique_id.argtypes = [vp]
    lib.afs_comm_create.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(vp)]
    lib.afs_comm_create_all.argtypes = [vp, ctypes.c_int32, vp]
    lib.afs_comm_destroy.argtypes = [vp]
    lib.afs_comm_destroy.restype = None
    lib.afs_gather_pcm.argtypes = [vp, vp, ctypes.c_int64, vp, vp]
    lib.afs_comm_fence.argtypes = [vp]
    lib.afs_comm_synchronize.argtypes = [vp]
    lib.afs_comm_gather_times.argtypes = [vp, dp, i32p]
    lib.afs_multi_synthesize.argtypes = [vp, vp, ctypes.c_int32, vp, vp, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, vp, vp, ctypes.POINTER(AfsReport)]
    for name in ("afs_create", "afs_set_stream", "afs_synchronize", "afs_synthesize",
                 "afs_session_create", "afs_session_synthesize", "afs_session_reset", "afs_af_to_frames",
                 "afs_to_int16", "afs_play_target_sequences", "afs_rng_draws", "afs_session_rng_draws", "afs_plan_hop_words",
                 "afs_kernel_times", "afs_kernel_times_ex", "afs_comm_unique_id", "afs_comm_create", "afs_comm_create_all",
                 "afs_gather_pcm", "afs_comm_fence", "afs_comm_synchronize", "afs_comm_gather_times",
                 "afs_multi_synthesize"):
        getattr(lib, name).restype = ctypes.c_int
    _lib = lib
    return lib


def check(status: int, ctx=None, what: str = "") -> None:
    if status != AFS_OK:
        msg = STATUS.get(status, str(status))
        detail = ""
        if ctx is not None:
            raw = load().afs_last_error(ctx)
            detail = raw.decode() if raw else ""
        raise AfsError(f"{what}: {msg}" + (f" ({detail})" if detail else ""))
