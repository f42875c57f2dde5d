"""ctypes binding of the amx C ABI (include/amx_hip.h).

The product path goes through these bindings only: there is no CPU or eager-PyTorch
fallback for any hot-path op.  If the library is missing or cannot be loaded, every op
raises `AmxNativeError` — loudly, on purpose.
"""
from __future__ import annotations

import ctypes as C
import os
import re

from . import _build

_HEADER = os.path.join(_build.INCLUDE, "amx_hip.h")
# AMX_ABI_VERSION of include/amx_hip.h (2: RFF column partials per 32 rows, AMX_RFF_PART_ROWS;
# the measured-slower A/B entry points removed)
ABI_VERSION = 2

c_int, c_ll, c_dbl, c_flt, c_u64, c_u32, vp = C.c_int, C.c_longlong, C.c_double, C.c_float, C.c_uint64, C.c_uint32, C.c_void_p
ip = C.POINTER(C.c_int)


class ResetNoise(C.Structure):
    """amx_reset_noise: SimEnv reset_args' AddNoise options (run.py:113-117)."""
    _fields_ = [("noise_bef_rot", C.c_int), ("noise_min", C.c_double), ("noise_max", C.c_double),
                ("radian", C.c_double), ("rot_vel_w_pose", C.c_int), ("vel_noise", C.c_int),
                ("interp", C.c_double), ("knee_rot", C.c_int)]

    @classmethod
    def from_reset_args(cls, ra: dict) -> "ResetNoise | None":
        """None when reset_args add no noise (radian 0 and noise_min = noise_max = 0)."""
        if float(ra["radian"]) == 0 and float(ra["noise_min"]) == 0 and float(ra["noise_max"]) == 0:
            return None
        return cls(int(bool(ra["noise_bef_rot"])), float(ra["noise_min"]), float(ra["noise_max"]),
                   float(ra["radian"]), int(bool(ra["rot_vel_w_pose"])), int(bool(ra["vel_noise"])),
                   float(ra["interp"]), int(bool(ra["knee_rot"])))


AMX_NOISE_ROT_SLOTS = 48
RFF_PART_ROWS = 32  # AMX_RFF_PART_ROWS: rows per fp64 column partial of the RFF features

# name -> (restype, argtypes); must match include/amx_hip.h exactly.
SIGNATURES = {
    "amx_create": (vp, [c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    "amx_destroy": (c_int, [vp]),
    "amx_last_error": (C.c_char_p, []),
    "amx_abi_version": (c_int, []),
    "amx_layout": (c_int, [vp, ip, ip, ip, ip]),
    "amx_set_normalizers": (c_int, [vp, vp, vp, vp, vp, vp, vp]),
    "amx_set_termination": (c_int, [vp, c_int, vp, vp, vp, vp, c_int, c_int, c_int, c_int, c_int,
                                    c_int, c_int, c_dbl, c_int, c_dbl]),
    "amx_assemble_input": (c_int, [vp, vp, vp, c_int, vp, c_ll, c_int, c_int, vp]),
    "amx_assemble_input_rexp": (c_int, [vp, vp, vp, c_int, vp, c_ll, c_int, c_int, vp, c_ll, c_ll, c_int, vp]),
    "amx_gemm_bias_act": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, c_ll, vp, c_int, c_ll,
                                  vp, c_ll, vp, c_int, c_ll, c_int, c_int, vp]),
    "amx_gemm_out_unnorm": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, c_ll, vp, c_int, c_ll,
                                    vp, c_ll, vp, c_int, c_ll, vp]),
    "amx_split_bf16x3": (c_int, [vp, c_int, c_int, c_int, vp, c_int, c_ll, vp, c_ll, vp]),
    "amx_gemm_bias_act_x6": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, c_ll, vp, c_ll,
                                     vp, c_ll, vp, c_int, c_ll, c_int, c_int, vp]),
    "amx_gemm_out_unnorm_x6": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, c_ll, vp, c_ll,
                                       vp, c_ll, vp, c_int, c_ll, vp]),
    "amx_rff_features_x6": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, vp, vp, c_flt, vp, c_int,
                                    vp, vp, vp]),
    "amx_split_f16x2": (c_int, [vp, c_int, c_int, c_int, vp, c_int, c_ll, vp, c_ll, vp, c_ll, vp]),
    "amx_row_exponents": (c_int, [vp, c_int, c_int, c_int, vp, c_int, c_ll, vp, c_ll, c_int, vp]),
    "amx_gemm_bias_act_h3": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, c_ll, vp, c_ll, vp, c_ll,
                                     vp, c_ll, vp, c_int, c_ll, c_int, c_int, vp, c_ll, c_int, vp, c_int, vp]),
    "amx_gemm_out_unnorm_h3": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, c_ll, vp, c_ll, vp, c_ll,
                                       vp, c_ll, vp, c_int, c_ll, vp, c_ll, c_int, c_int, vp]),
    "amx_set_motion": (c_int, [vp, vp, c_ll]),
    "amx_motion_duration": (c_dbl, [vp]),
    "amx_motion_states": (c_int, [vp, vp, c_int, c_int, vp, c_ll, vp]),
    "amx_motion_states_noise": (c_int, [vp, vp, c_int, c_int, vp, vp, c_ll, c_u64, vp, c_ll, vp]),
    "amx_reset_lanes_motion_noise": (c_int, [vp, vp, vp, c_u64, c_dbl, c_int, vp, vp, c_ll, vp, vp, vp, vp, vp, vp,
                                             c_int, vp]),
    "amx_reset_lanes_motion": (c_int, [vp, vp, vp, c_u64, c_dbl, c_int, vp, vp, vp, vp, vp, vp, c_int, vp]),
    "amx_amp_obs_size": (c_int, [vp]),
    "amx_state_amp_obs": (c_int, [vp, vp, vp, c_ll, c_int, c_int, vp, c_ll, vp]),
    "amx_motion_amp_obs": (c_int, [vp, vp, c_dbl, c_int, c_int, vp, c_ll, vp]),
    "amx_state_amp_rows": (c_int, [vp, vp, vp, c_ll, c_int, c_int, vp, c_ll, vp]),
    "amx_npg_param_count": (c_ll, [c_int, c_int]),
    "amx_npg_pass": (c_int, [vp, c_int, c_int, vp, c_int, c_ll, vp, c_int, c_ll, vp, vp, vp, c_int, vp, vp]),
    "amx_npg_reduce": (c_int, [vp, vp, c_int, c_int, vp, vp]),
    "amx_npg_pass_gated": (c_int, [vp, c_int, c_int, vp, c_int, c_ll, vp, c_int, c_ll, vp, vp, vp, c_int, vp, vp, vp]),
    "amx_npg_reduce_gated": (c_int, [vp, vp, c_int, c_int, vp, vp, vp]),
    "amx_npg_curvature": (c_int, [vp, vp, c_int, c_int, vp, vp]),
    "amx_npg_cg_tail_work": (c_ll, [c_int]),
    "amx_npg_cg_tail": (c_int, [vp, vp, c_int, c_int, c_int, vp, c_dbl, c_dbl, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "amx_npg_cg_reduce": (c_int, [vp, vp, c_int, c_int, c_int, vp, c_dbl, vp, vp, vp, vp, vp]),
    "amx_npg_cg_xrp": (c_int, [vp, c_int, c_dbl, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "amx_npg_pass_cg": (c_int, [vp, c_int, vp, c_int, c_ll, vp, c_int, vp, vp, c_dbl, vp, vp, vp, vp, vp, vp, vp, vp,
                                vp, vp]),
    "amx_npg_apply_step": (c_int, [vp, c_int, c_int, vp, vp, vp, c_int, c_dbl, c_dbl, c_flt, vp, vp, vp]),
    "amx_npg_pass_ex": (c_int, [vp, c_int, c_int, vp, c_int, c_ll, vp, c_int, c_ll, vp, vp, vp, c_int, vp, vp, vp, vp]),
    "amx_npg_cg_init": (c_int, [vp, c_int, vp, vp, vp, vp, vp, vp, vp]),
    "amx_npg_cg_init_ls": (c_int, [vp, c_int, c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "amx_npg_cg_step": (c_int, [vp, c_int, c_int, vp, vp, c_dbl, c_dbl, vp, vp, vp, vp, vp, vp]),
    "amx_step": (c_int, [vp, vp, c_int, c_ll, vp, vp, vp, vp, vp, vp, vp, c_int, vp, c_int, vp]),
    "amx_step_rexp": (c_int, [vp, vp, c_int, c_ll, vp, vp, vp, vp, vp, vp, vp, c_int, vp, vp, c_int, vp]),
    "amx_step_reset": (c_int, [vp, vp, c_int, c_ll, vp, vp, vp, vp, vp, vp, vp, c_int, vp, vp, vp, c_int, vp,
                               c_u64, vp, vp, vp, vp, vp, c_ll, vp, c_int, vp]),
    "amx_step_reset_act": (c_int, [vp, vp, c_int, c_ll, vp, vp, vp, vp, vp, vp, vp, c_int, vp, vp, vp, c_int, vp,
                                   c_u64, vp, vp, vp, vp, vp, vp, c_int, c_int, vp, c_u64, c_u64, vp, c_int, vp, vp,
                                   vp, c_ll, c_int, vp, c_ll, c_ll, c_int, c_int, vp]),
    "amx_set_step_act_occupancy": (c_int, [vp, c_int]),
    "amx_rff_features_h3": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, vp, vp, vp, vp, c_flt, vp, c_int,
                                    vp, vp, vp]),
    "amx_disagreement": (c_int, [vp, vp, c_int, c_ll, vp, c_int, vp]),
    "amx_reset_lanes": (c_int, [vp, vp, vp, c_int, vp, c_u64, vp, vp, vp, vp, vp, vp, c_int, vp]),
    "amx_policy_act": (c_int, [vp, vp, c_int, vp, c_int, c_int, vp, vp, c_u64, c_u64, c_int, vp, vp, vp, c_ll,
                               c_int, vp, c_ll, c_ll, c_int, vp]),
    "amx_policy_act_dev": (c_int, [vp, vp, c_int, vp, c_int, c_int, vp, vp, c_u64, vp, c_u64, c_int, vp, vp, vp,
                                   c_ll, c_int, vp, c_ll, c_ll, c_int, vp]),
    "amx_counter_add": (c_int, [vp, vp, c_ll, vp]),
    "amx_set_gemm_timer": (c_int, [vp, vp]),
    "amx_split_workspace_floats": (c_ll, [vp, c_int, c_int, ip]),
    "amx_set_split_workspace": (c_int, [vp, vp, c_ll, vp, c_int]),
    "amx_policy_blob_floats": (c_ll, [vp, c_int, c_int]),
    "amx_policy_pack": (c_int, [vp, vp, vp, c_int, vp, vp, c_int, vp, vp, vp, vp]),
    "amx_rff_features": (c_int, [vp, c_int, c_int, c_int, c_int, vp, c_int, vp, c_int, vp, c_flt, vp, c_int,
                                 vp, vp, vp]),
    "amx_sum_partials": (c_int, [vp, vp, c_int, c_int, vp, vp]),
    "amx_mmd_fit": (c_int, [vp, vp, c_dbl, vp, c_int, vp, vp, vp]),
    "amx_mmd_reward": (c_int, [vp, vp, c_int, vp, c_int, vp, c_flt, c_dbl, c_flt, c_flt, vp, vp, vp, c_int, vp]),
    "amx_mmd_reward_raw": (c_int, [vp, vp, c_int, vp, c_int, vp, c_dbl, vp, vp, vp, c_int, vp]),
    "amx_expert_cost": (c_int, [vp, vp, c_int, vp, c_int, c_int, c_flt, c_flt, vp, vp, c_dbl, vp]),
    "amx_feature_message": (c_int, [vp, vp, c_int, c_int, c_dbl, vp, vp]),
    "amx_mmd_relabel": (c_int, [vp, vp, c_dbl, vp, c_int, vp, vp, vp, c_int, vp, c_flt, c_dbl, c_int, c_flt, c_flt,
                                vp, vp, vp, c_int, vp, c_int, c_int, vp, vp, vp, vp]),
    "amx_amp_reward": (c_int, [vp, vp, c_int, c_int, vp, c_flt, vp, c_dbl, vp, vp, c_int, vp]),
    "amx_disc_reward": (c_int, [vp, c_int, vp, c_int, c_int, vp, c_flt, vp, c_dbl, vp, vp, c_int, vp]),
    "amx_cost_rows": (c_int, [vp, vp, c_ll, c_int, vp, c_ll, c_int, vp, c_ll, c_int, c_int, vp, c_int, vp]),
    "amx_value_features": (c_int, [vp, c_int, c_int, vp, vp, vp, c_ll, vp, vp, c_int, vp, c_int, vp]),
    "amx_value_head": (c_int, [vp, c_int, vp, c_int, c_int, vp, vp, vp, vp]),
    "amx_gae": (c_int, [vp, c_int, c_int, vp, vp, c_ll, vp, vp, vp, c_ll, vp, c_dbl, c_dbl, vp, vp, vp]),
    "amx_adv_whiten": (c_int, [vp, c_int, c_int, vp, vp, c_ll, vp, c_dbl, vp, vp, vp]),
    "amx_philox": (c_int, [vp, c_u64, c_u32, c_u32, c_u32, vp, c_int, vp]),
    "amx_mt_seed": (c_int, [vp, c_int, vp, vp, c_int]),
    "amx_mt_policy_noise": (c_int, [vp, c_int, vp, c_int, c_int, c_int, vp, c_ll, c_ll]),
}
AMX_MT_STATE_BYTES = 2512

AMX_ROW_TILE = 128
AMX_K_TILE = 32
AMX_SHAPE_SPHERE, AMX_SHAPE_CAPSULE, AMX_SHAPE_BOX = 0, 1, 2
AMX_ACT_NONE, AMX_ACT_RELU = 0, 1
AMX_IN_F64, AMX_IN_F32 = 0, 1
AMX_DISC_LEAST_SQUARES, AMX_DISC_LOG_LIKELIHOOD = 0, 1


class AmxNativeError(RuntimeError):
    pass


def header_symbols(path: str = _HEADER) -> list[str]:
    """Every function the public header declares (used by the export test)."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(amx_[a-z0-9_]+)\s*\(", txt)))


_LIB = None


def load(path: str | None = None, build_if_missing: bool = False):
    """Load libamx_hip.so and bind signatures.  Never falls back to anything else."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    path = path or _build.LIB_PATH
    if not os.path.exists(path):
        if build_if_missing:
            _build.build()
        else:
            raise AmxNativeError(
                f"{path} is missing: build it with `python -m amp_extensions_amd._build` "
                "(there is no CPU fallback for the rollout hot path)")
    try:
        lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    except OSError as e:
        raise AmxNativeError(f"cannot load {path}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.amx_abi_version() != ABI_VERSION:
        raise AmxNativeError("libamx_hip ABI version mismatch")
    if path == _build.LIB_PATH:
        _LIB = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = _LIB.amx_last_error().decode() if _LIB is not None else "?"
        raise AmxNativeError(f"{what or 'amx call'} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream
