"""C ABI boundary: libhwy.so loads (no GPU needed), exports every function include/*.h
declares, and agrees with the Python/ctypes mirror on the config and PPO parameter layouts."""

import ctypes
import os
import re

import pytest

from hwy import _abi
from hwy.native import LIB_PATH

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include")))
           if h.endswith(".h")]


def declared_functions():
    names = set()
    for header in HEADERS:
        src = open(header).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names.update(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s+(hwy_[a-z_0-9]+)\s*\(", src,
                                flags=re.M))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    assert os.path.exists(LIB_PATH), "run __graft_entry__.build() first"
    return ctypes.CDLL(LIB_PATH)


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["hwy_create", "hwy_destroy", "hwy_reset", "hwy_step", "hwy_obs_pe", "hwy_gae",
                 "hwy_set_pe_table", "hwy_export_state", "hwy_import_state", "hwy_last_error"]:
        assert must in names
    for must in ["hwy_ppo_param_layout", "hwy_ppo_workspace_bytes", "hwy_ppo_forward_backward",
                 "hwy_ppo_optimizer", "hwy_ppo_sync_params", "hwy_ppo_act"]:
        assert must in names
    assert len(names) >= 20


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"libhwy.so lacks {missing}"


def test_abi_version_and_config_layout(lib):
    assert lib.hwy_abi_version() == _abi.HWY_ABI_VERSION
    assert lib.hwy_config_size() == ctypes.sizeof(_abi.HwyConfig)


def test_oracle_config_layout_matches():
    from oracle import oracle

    assert oracle.lib().hwyo_config_size() == ctypes.sizeof(_abi.HwyConfig)


def test_validation_errors_without_gpu(lib):
    """Configuration errors are reported before any device work (-> ValueError in Python)."""
    lib.hwy_last_error.restype = ctypes.c_char_p
    cfg = _abi.config_from_dict({"observation": {"vehicles_count": 15, "features": ["x", "y"]}},
                                num_envs=4, pe_kind=_abi.PE_ROPE, d_embed=3)
    h = ctypes.c_void_p()
    rc = lib.hwy_create(ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc == -1 and b"rotate_dim" in lib.hwy_last_error()
    cfg = _abi.config_from_dict({"vehicles_count": 80}, num_envs=4)
    assert lib.hwy_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == -1
    assert b"vehicles_count" in lib.hwy_last_error()


def test_no_cpu_fallback_in_product_path():
    """The product modules never import the oracle."""
    pkg = os.path.join(ROOT, "highway-rope-ppo_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                text = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", text, flags=re.M), f


def test_ppo_param_layout_matches_actor_critic():
    """hwy_ppo_param_layout (host-only) equals nn.Module.parameters() sizes in _PARAM_ORDER."""
    import torch

    from hwy.ppo_native import _PARAM_ORDER, param_layout
    from ppo.agent import ActorCritic

    for S, H in [(60, 256), (120, 64), (136, 512)]:
        ac = ActorCritic(S, 2, H)
        named = dict(ac.named_parameters())
        offs, numel = param_layout(S, H)
        sizes = [named[n].numel() for n in _PARAM_ORDER]
        assert offs == [sum(sizes[:i]) for i in range(13)]
        assert numel == sum(sizes) == sum(p.numel() for p in ac.parameters())
    with pytest.raises(ValueError):
        param_layout(60, 100)  # hidden_dim not a multiple of 64


def test_product_library_reads_no_development_knobs(lib):
    """The shipped libhwy.so is a product build: the development knobs that change the PPO
    partitions (HWY_WG_BAL / HWY_ROWS_RT / HWY_WG_FILL) and the section clocks are compiled out
    (hwy_ppo_build_flags() == 0), so no environment variable changes a gradient's summation
    order."""
    lib.hwy_ppo_build_flags.restype = ctypes.c_int
    assert lib.hwy_ppo_build_flags() == 0
    src = open(os.path.join(ROOT, "highway-rope-ppo_amd", "csrc", "ppo_kernels.hip")).read()
    # every getenv of the PPO kernels sits inside the HWY_DEV_KNOBS block
    dev = src[src.index("#ifdef HWY_DEV_KNOBS"):src.index("#endif", src.index("#ifdef HWY_DEV_KNOBS"))]
    assert src.count("getenv(") == dev.count("getenv(")


def test_product_library_holds_only_reachable_row_kernels():
    """Kernels no product launch selects are not built into libhwy.so (the
    transposed ppo_rowsT row kernel was compiled in but reachable only through a dev knob)."""
    blob = open(LIB_PATH, "rb").read()
    assert b"ppo_rowsT" not in blob
    # mangled names (length-prefixed), so that ppo_rows_c64 does not also satisfy ppo_rows_c
    # (ADVICE r4): the 32-row compact tile and the 64-row tile are separate kernels
    for name in (b"10ppo_rows_cILi4ELi8ELi32E", b"12ppo_rows_c64ILi4ELi8E", b"ppo_wgrad",
                 b"ppo_wsum", b"ppo_adam", b"ppo_act_c", b"hwy_step_kernel"):
        assert name in blob, name
    # H = 256's 32-row tiles always run the compact kernel: the plain one is not built
    assert b"8ppo_rowsILi4ELi8ELi32E" not in blob


def test_kernel_sources_carry_no_ab_knob_forest():
    """the measured-and-rejected A/B alternatives are gone from the product
    kernel sources; what remains for development sits behind HWY_DEV_KNOBS (the partition knobs
    of ppo_kernels.hip's dev block, the timing-only pricing masks of hwy_dev_knobs.h)."""
    import glob
    import re

    csrc = os.path.join(ROOT, "highway-rope-ppo_amd", "csrc")
    n = 0
    for path in glob.glob(os.path.join(csrc, "*.hip")):
        src = open(path).read()
        n += len(re.findall(r"^#ifndef HWY_", src, flags=re.M))
        # timing-only (wrong-result) builds are reachable only through the dev header
        assert "HWY_SKIP" not in src, path
        assert "HWY_WG_EXP" not in src and "HWY_WG_TEAMS" not in src, path
    assert n <= 3
    dev = open(os.path.join(csrc, "hwy_dev_knobs.h")).read()
    assert "HWY_SKIP" in dev


def test_group_table_geometry_without_gpu(lib):
    """hwy_ppo_group_table_bytes (include/hwy_ppo.h): the grouped step covers the fused path's
    16-row tiles (a sweep experiment's 64-row minibatches), not the 32- / 64-row tiles of large
    minibatches; the table grows with the learner count."""
    from hwy.ppo_native import PpoDims

    f = lib.hwy_ppo_group_table_bytes
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.POINTER(PpoDims), ctypes.c_int]
    one = f(ctypes.byref(PpoDims(64, 60, 256, 2)), 1)
    ten = f(ctypes.byref(PpoDims(64, 60, 256, 2)), 10)
    assert 0 < one < ten and ten % 256 == 0
    assert f(ctypes.byref(PpoDims(64, 120, 512, 2)), 10) > 0
    assert f(ctypes.byref(PpoDims(16384, 60, 256, 2)), 10) == -1  # 32-row tiles
    assert f(ctypes.byref(PpoDims(64, 62, 256, 2)), 10) == -1     # S % 4 != 0: general path
    assert f(ctypes.byref(PpoDims(64, 60, 256, 2)), 0) == -1
    g = lib.hwy_ppo_group_act_table_bytes
    g.restype = ctypes.c_int64
    assert g(10) > g(1) > 0 and g(0) == -1


def test_step_group_table_and_argument_checks_without_gpu(lib):
    """hwy_step_group (include/hwy.h): the table holds one launch-parameter record per handle,
    and a prepare or launch with missing arguments is refused before any device call."""
    from hwy.native import HwyStepGroupPlan, HwyStepIO

    f = lib.hwy_step_group_table_bytes
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_int]
    one = f(1)
    assert one > 0 and f(4) == 4 * one and f(0) == -1
    p = lib.hwy_step_group_prepare
    p.restype = ctypes.c_int
    p.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                  ctypes.POINTER(HwyStepGroupPlan), ctypes.c_void_p]
    plan = HwyStepGroupPlan()
    io = (HwyStepIO * 1)()
    assert p(None, io, 1, None, ctypes.byref(plan), None) == -1
    handles = (ctypes.c_void_p * 1)(None)
    assert p(handles, io, 1, ctypes.c_void_p(16), ctypes.byref(plan), None) == -1  # NULL handle
    lib.hwy_last_error.restype = ctypes.c_char_p
    assert b"NULL" in lib.hwy_last_error()
    s = lib.hwy_step_group
    s.restype = ctypes.c_int
    s.argtypes = [ctypes.POINTER(HwyStepGroupPlan), ctypes.c_void_p, ctypes.c_void_p]
    assert s(ctypes.byref(HwyStepGroupPlan(0, 0, 0)), ctypes.c_void_p(16), None) == -1
