"""Loader for libhwy.so (the HIP/gfx950 C ABI of include/hwy.h).

The product path always runs through this library: there is no CPU fallback.  If the library is
missing or cannot be loaded, every compute entry point raises ``HwyNativeError``.
torch is imported first so that libhwy.so binds to the HIP runtime torch already loaded
(same soname, libamdhip64.so.7) and shares its streams.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

from ._abi import HWY_ABI_VERSION, HwyConfig

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libhwy.so")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

HWY_OK, HWY_EINVAL, HWY_EDEVICE, HWY_ENOMEM = 0, -1, -2, -3


class HwyNativeError(RuntimeError):
    """libhwy.so is unavailable or a device call failed."""


_lib = None


class HwyStepIO(ctypes.Structure):
    """hwy_step_io (include/hwy.h): one handle's buffers for a grouped step."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("actions", "obs", "reward", "terminated",
                                               "truncated", "ep_return", "ep_length")]


class HwyStepGroupPlan(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("blocks", ctypes.c_int32), ("big", ctypes.c_int32)]


def build(jobs: int = 4) -> str:
    """Compile libhwy.so for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", CSRC], check=True)
    return LIB_PATH


def lib():
    """The loaded libhwy.so (raises HwyNativeError when it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (load torch's HIP runtime first; see module docstring)

    if not os.path.exists(LIB_PATH):
        raise HwyNativeError(
            f"{LIB_PATH} not found: build it with `make -C {CSRC}` "
            "(or __graft_entry__.build()); there is no CPU fallback"
        )
    try:
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on the box
        raise HwyNativeError(f"cannot load {LIB_PATH}: {e}") from e
    vp, i32, f32, f64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_double
    cfgp = ctypes.POINTER(HwyConfig)
    L.hwy_abi_version.restype = i32
    L.hwy_last_error.restype = ctypes.c_char_p
    L.hwy_create.argtypes = [cfgp, i32, ctypes.POINTER(vp)]
    L.hwy_destroy.argtypes = [vp]
    L.hwy_destroy.restype = None
    L.hwy_obs_features.argtypes = [vp]
    L.hwy_set_pe_table.argtypes = [vp, vp, i32]
    L.hwy_set_seed_schedule.argtypes = [vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64]
    L.hwy_reset.argtypes = [vp, vp, vp, vp, vp]
    L.hwy_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.hwy_export_state.argtypes = [vp, vp, vp]
    L.hwy_import_state.argtypes = [vp, vp, vp]
    L.hwy_obs_pe.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, f32, vp, vp, vp]
    L.hwy_gae.argtypes = [vp, vp, vp, vp, f64, f64, i32, i32, vp, vp, vp]
    L.hwy_math_selftest.argtypes = [i32, vp, vp, vp, i32, vp]
    L.hwy_set_seed_groups.argtypes = [vp, vp, i32, i32]
    L.hwy_step_group_table_bytes.argtypes = [i32]
    L.hwy_step_group_table_bytes.restype = ctypes.c_int64
    L.hwy_step_group_prepare.argtypes = [vp, vp, i32, vp, ctypes.POINTER(HwyStepGroupPlan), vp]
    L.hwy_step_group.argtypes = [ctypes.POINTER(HwyStepGroupPlan), vp, vp]
    for name in ("hwy_create", "hwy_obs_features", "hwy_set_pe_table", "hwy_set_seed_schedule",
                 "hwy_set_seed_groups", "hwy_reset", "hwy_step", "hwy_step_group_prepare",
                 "hwy_step_group",
                 "hwy_export_state", "hwy_import_state", "hwy_obs_pe", "hwy_gae",
                 "hwy_math_selftest"):
        getattr(L, name).restype = i32
    if L.hwy_abi_version() != HWY_ABI_VERSION:
        raise HwyNativeError(
            f"libhwy.so ABI {L.hwy_abi_version()} != python ABI {HWY_ABI_VERSION}; rebuild"
        )
    _lib = L
    return L


def last_error() -> str:
    msg = lib().hwy_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc == HWY_OK:
        return
    msg = f"{what}: {last_error()}"
    if rc == HWY_EINVAL:
        raise ValueError(msg)
    raise HwyNativeError(msg)


def ptr(t) -> Optional[int]:
    """Device pointer of a torch tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(stream=None) -> Optional[int]:
    import torch

    s = torch.cuda.current_stream() if stream is None else stream
    return s.cuda_stream


def require_device(t, name: str) -> None:
    if not t.is_cuda:
        raise HwyNativeError(f"{name} must be a HIP device tensor (got {t.device}); no CPU path")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
