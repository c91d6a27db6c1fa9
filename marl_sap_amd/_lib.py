"""ctypes binding of the C-ABI in include/asg.h (libmarl_sap_amd.so, built in-tree).

There is no fallback: if the HIP library is missing or fails to load, every entry point
raises.  Status codes map to Python exceptions the way the reference's own failures
surface (ValueError for bad input / scipy LSA errors, RuntimeError for HIP failures).
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ASG_LIB_PATH") or os.path.join(HERE, "libmarl_sap_amd.so")

ASG_OK = 0
ASG_E_INVALID_ARG = -1
ASG_E_HIP = -2
ASG_E_STATE = -3
ASG_E_LSA_INVALID = -4
ASG_E_LSA_INFEASIBLE = -5
ASG_E_ACTION_RANGE = -6

ASG_F32, ASG_F64, ASG_I64, ASG_I32, ASG_BOOL, ASG_F16, ASG_I16 = 0, 1, 2, 3, 4, 5, 6
ASG_RNG_PHILOX, ASG_RNG_MT19937 = 0, 1
ASG_BENEFIT_BUMP, ASG_BENEFIT_DENSE, ASG_BENEFIT_INJECTED = 0, 1, 2
ASG_QUIRK_PREV_ASSIGNS_ZERO = 0x1
ASG_QUIRK_PARALLEL_TERMINATED = 0x2
ASG_QUIRK_REPLICATE_STREAM = 0x4
ASG_STEP_USE_SELECTED_BIDS = 0x1

_DTYPES = {torch.float32: ASG_F32, torch.float64: ASG_F64, torch.int64: ASG_I64,
           torch.int32: ASG_I32, torch.bool: ASG_BOOL, torch.float16: ASG_F16, torch.int16: ASG_I16}

# every symbol include/asg.h declares (checked by tests/test_abi.py)
EXPORTS = ["asg_abi_version", "asg_last_error", "asg_create", "asg_destroy", "asg_set_stream",
           "asg_reset", "asg_step", "asg_random_actions", "asg_sync_status", "asg_set_benefits",
           "asg_export_benefits", "asg_export_bump_params", "asg_export_prev_assigns", "asg_get_returns", "asg_get_step",
           "asg_advance_stream", "asg_beta_hat", "asg_lsa_batched", "asg_haa_select", "asg_sap_select", "asg_epsilon_greedy",
           "asg_rnn_agent_packed_size", "asg_rnn_agent_mfma_mode", "asg_rnn_agent_mode", "asg_rnn_agent_pack", "asg_rnn_agent_forward",
           "asg_rnn_agent_select", "asg_real_create", "asg_real_destroy", "asg_real_set_stream",
           "asg_real_set_benefits", "asg_real_set_initial_assignments", "asg_real_reset", "asg_real_step", "asg_real_sync_status",
           "asg_real_get_returns", "asg_real_get_step", "asg_real_obs_size", "asg_filtered_topm",
           "asg_filtered_benefits", "asg_filtered_epsilon_greedy", "asg_filtered_soft_map", "asg_real_haal_select",
           "asg_real_haal_num_sequences", "asg_step_select", "asg_step_select_l2_slices", "asg_rollout",
           "asg_rollout_l2_slices", "asg_reset_rollout", "asg_sap_select_into", "asg_step_forward",
           "asg_sap_noise", "asg_random_rollout", "asg_sap_select_warm", "asg_bids_select",
           "asg_reset_forward", "asg_step_ex", "asg_step_forward_ex", "asg_bids_select_count"]


class AsgField(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("dtype", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("stride", ctypes.c_int64 * 4)]


_VIEW_FIELDS = ["obs", "actions", "avail_actions", "rewards", "terminated", "prev_assigns", "beta",
                "actions_onehot", "filled"]


class AsgBatchView(ctypes.Structure):
    _fields_ = [(f, AsgField) for f in _VIEW_FIELDS]


class AsgConfig(ctypes.Structure):
    _fields_ = [("num_envs", ctypes.c_int64), ("n", ctypes.c_int32), ("m", ctypes.c_int32),
                ("T", ctypes.c_int32), ("L", ctypes.c_int32), ("lambda_", ctypes.c_double),
                ("bids_as_actions", ctypes.c_int32), ("rng_mode", ctypes.c_int32),
                ("benefit_mode", ctypes.c_int32), ("quirks", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("env_index_base", ctypes.c_int64),
                ("T_trans", ctypes.POINTER(ctypes.c_double))]


class AsgRealConfig(ctypes.Structure):
    _fields_ = [("num_envs", ctypes.c_int64), ("n", ctypes.c_int32), ("m", ctypes.c_int32),
                ("T", ctypes.c_int32), ("L", ctypes.c_int32), ("N", ctypes.c_int32), ("M", ctypes.c_int32),
                ("lambda_", ctypes.c_double), ("T_trans", ctypes.POINTER(ctypes.c_double)),
                ("task_prios", ctypes.POINTER(ctypes.c_double)), ("variant", ctypes.c_int32),
                ("bids_as_actions", ctypes.c_int32), ("seed", ctypes.c_uint64), ("env_index_base", ctypes.c_int64),
                ("sat_freq_bands", ctypes.POINTER(ctypes.c_int32)),
                ("neighbor_matrix", ctypes.POINTER(ctypes.c_double))]


class AsgRealBatchView(ctypes.Structure):
    _fields_ = [("base", AsgBatchView), ("power_states", AsgField)]


ASG_REAL_PLAIN, ASG_REAL_POWER, ASG_REAL_INTERFERENCE = 0, 1, 2


_lib = None


def lib():
    """Load the HIP library (after torch, so both share torch's HIP runtime)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"marl_sap_amd HIP library not built ({LIB_PATH} missing): run "
                "`python -m marl_sap_amd.build` (hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        vp, i64, i32, dbl = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.asg_abi_version.restype = i32
        L.asg_last_error.argtypes = [vp]
        L.asg_last_error.restype = ctypes.c_char_p
        L.asg_create.argtypes = [ctypes.POINTER(AsgConfig), i32, vp, ctypes.POINTER(vp)]
        L.asg_destroy.argtypes = [vp]
        L.asg_set_stream.argtypes = [vp, vp]
        for f in ("asg_reset", "asg_step", "asg_random_actions"):
            getattr(L, f).argtypes = [vp, ctypes.POINTER(AsgBatchView), i32]
        if hasattr(L, "asg_random_rollout"):  # absent from older A/B builds (tools/build_rev.sh)
            L.asg_random_rollout.argtypes = [vp, ctypes.POINTER(AsgBatchView), i32, i32, i32]
        L.asg_sync_status.argtypes = [vp]
        L.asg_set_benefits.argtypes = [vp, vp, i64, i32]
        L.asg_export_benefits.argtypes = [vp, vp]
        L.asg_export_bump_params.argtypes = [vp, vp]
        L.asg_export_prev_assigns.argtypes = [vp, vp]
        L.asg_get_returns.argtypes = [vp, vp]
        L.asg_get_step.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
        L.asg_advance_stream.argtypes = [vp, i64]
        L.asg_beta_hat.argtypes = [vp, i32, i64p, vp, i64p, i64, i32, i32, vp, dbl, vp, vp]
        L.asg_lsa_batched.argtypes = [vp, i32, i64p, i64, i32, i32, i32, vp, vp, vp, vp]
        L.asg_haa_select.argtypes = [vp, i64p, vp, i64p, i64, i32, i32, vp, dbl, vp, vp, vp]
        L.asg_sap_select.argtypes = [vp, i64p, i64, i32, i32, dbl, ctypes.c_uint64, ctypes.c_uint64, i64, vp, vp, vp,
                                     vp]
        L.asg_epsilon_greedy.argtypes = [vp, i64p, vp, i64p, i64, i32, i32, dbl, ctypes.c_uint64, ctypes.c_uint64,
                                         i64, vp, i64p, vp, vp]
        L.asg_rnn_agent_packed_size.argtypes = [i32, i32, i32, i32]
        L.asg_rnn_agent_mfma_mode.restype = i32
        L.asg_rnn_agent_mode.argtypes = [i32, i32, i32, i32]
        L.asg_rnn_agent_mode.restype = i32
        L.asg_rnn_agent_pack.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, vp, vp]
        L.asg_rnn_agent_forward.argtypes = [vp, i64, i64, i32, vp, i64] + [vp] * 5 + [i32, i32, i32, vp, vp, vp]
        L.asg_rnn_agent_select.argtypes = [vp, i64, i64, i32, vp, i64] + [vp] * 5 + [i32, i32, i32, vp, vp, vp, i64p,
                                                                                 i32, dbl, ctypes.c_uint64,
                                                                                 ctypes.c_uint64, i64, vp, i64p, vp,
                                                                                 vp]
        L.asg_real_create.argtypes = [ctypes.POINTER(AsgRealConfig), i32, vp, ctypes.POINTER(vp)]
        L.asg_real_destroy.argtypes = [vp]
        L.asg_real_destroy.restype = None
        L.asg_real_set_stream.argtypes = [vp, vp]
        L.asg_real_set_benefits.argtypes = [vp, vp, i64, i32]
        L.asg_real_set_initial_assignments.argtypes = [vp, vp, i64, i32]
        L.asg_real_reset.argtypes = [vp, ctypes.POINTER(AsgRealBatchView), i32]
        L.asg_real_step.argtypes = [vp, ctypes.POINTER(AsgRealBatchView), i32]
        L.asg_real_sync_status.argtypes = [vp]
        L.asg_real_get_returns.argtypes = [vp, vp]
        L.asg_real_get_step.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
        L.asg_real_obs_size.argtypes = [i32, i32, i32]
        u64 = ctypes.c_uint64
        L.asg_filtered_topm.argtypes = [vp, i32, i64p, i64, i32, i32, i32, i32, vp, vp]
        L.asg_filtered_benefits.argtypes = [vp, i64p, vp, i64, i32, i32, i32, vp, dbl, vp, u64, u64, i64, vp, vp]
        L.asg_filtered_epsilon_greedy.argtypes = [vp, i64p, vp, i64p, i64, i32, i32, dbl, u64, u64, i64, vp, i64p,
                                                  vp, vp]
        L.asg_filtered_soft_map.argtypes = [vp, vp, i64, i32, i32, i32, u64, u64, i64, vp, vp, vp]
        L.asg_real_haal_select.argtypes = [vp, vp, vp, vp, vp]
        L.asg_real_haal_num_sequences.argtypes = [vp]
        L.asg_step_select.argtypes = [vp, ctypes.POINTER(AsgBatchView), i32, vp, vp, vp, vp, vp, i32, i32, vp, i64, vp,
                                      dbl, u64, u64, vp, vp]
        L.asg_step_select_l2_slices.argtypes = [i32, i32, i32]
        L.asg_rollout.argtypes = [vp, ctypes.POINTER(AsgBatchView), i32, i32, i32, i32, vp, vp, vp, vp, vp, i32, i32,
                                  i32, vp, i64, vp, dbl, u64, u64, vp, vp]
        L.asg_rollout_l2_slices.argtypes = [i32, i32, i32, i32]
        L.asg_reset_rollout.argtypes = [vp, ctypes.POINTER(AsgBatchView), i32, i32, i32, vp, vp, vp, vp, vp, i32, i32,
                                        i32, vp, i64, vp, dbl, u64, u64, vp, vp]
        L.asg_sap_select_into.argtypes = [vp, i64p, i64, i32, i32, dbl, u64, u64, i64, vp, vp, vp, vp]
        L.asg_sap_noise.argtypes = [vp, i64p, i64, i32, i32, dbl, u64, u64, i64, vp, vp, vp]
        if hasattr(L, "asg_sap_select_warm"):  # absent from older A/B builds
            L.asg_sap_select_warm.argtypes = [vp, i64p, i64, i32, i32, dbl, u64, u64, i64, vp, vp, vp, vp, i32, vp]
        if hasattr(L, "asg_bids_select"):  # absent from older A/B builds
            L.asg_bids_select.argtypes = [vp, vp, i64p, vp, i64p, i32, i32, dbl, u64, u64, vp]
        if hasattr(L, "asg_bids_select_count"):
            L.asg_bids_select_count.argtypes = [vp, vp, i64p, vp, i64p, i32, i32, dbl, u64, u64, vp, vp]
        if hasattr(L, "asg_reset_forward"):
            L.asg_reset_forward.argtypes = [vp, ctypes.POINTER(AsgBatchView), i32, vp, vp, vp, vp, vp, i32, i32, i32,
                                            vp, i64, vp, vp, vp]
        L.asg_step_forward.argtypes = [vp, ctypes.POINTER(AsgBatchView), i32, vp, vp, vp, vp, vp, i32, i32, i32, vp,
                                       i64, vp, vp, vp]
        if hasattr(L, "asg_step_ex"):  # absent from older A/B builds
            L.asg_step_ex.argtypes = [vp, ctypes.POINTER(AsgBatchView), i32, i32]
            L.asg_step_forward_ex.argtypes = [vp, ctypes.POINTER(AsgBatchView), i32, vp, vp, vp, vp, vp, i32, i32,
                                              i32, vp, i64, vp, vp, i32, vp]
        for f in EXPORTS:
            if f not in ("asg_last_error", "asg_real_destroy") and hasattr(L, f):
                getattr(L, f).restype = i32
        L.asg_rnn_agent_packed_size.restype = i64
        if L.asg_abi_version() != 1:
            raise RuntimeError("libmarl_sap_amd.so ABI version mismatch")
        _lib = L
    return _lib


def last_error(handle=None):
    msg = lib().asg_last_error(handle)
    return msg.decode() if msg else ""


def check(rc, handle=None):
    """Map an ASG status code to the exception the reference would raise."""
    if rc == ASG_OK:
        return
    msg = last_error(handle)
    if rc in (ASG_E_INVALID_ARG, ASG_E_LSA_INVALID, ASG_E_LSA_INFEASIBLE, ASG_E_ACTION_RANGE):
        raise ValueError(msg)
    raise RuntimeError(f"asg error {rc}: {msg}")


def i64arr(vals):
    return (ctypes.c_int64 * len(vals))(*[int(v) for v in vals])


def field(t):
    """asg_field of a tensor of up to 4 dims ([B, T+1, d2, d3]), or 5 dims with a
    contiguous last dim (the real env's beta [B, T+1, n, m, L]); None -> absent."""
    f = AsgField()
    if t is None:
        f.ptr = None
        return f
    if not t.is_cuda:
        raise ValueError("EpisodeBatch tensors handed to the HIP env must live on the GPU")
    if t.dim() == 5 and t.stride(-1) == 1:
        t = t.select(-1, 0)
    if t.dim() > 4:
        raise ValueError("batch fields have at most 4 dims (or 5 with a contiguous last dim)")
    f.ptr = t.data_ptr()
    f.dtype = _DTYPES[t.dtype]
    st = list(t.stride()) + [1] * (4 - t.dim())
    for i in range(4):
        f.stride[i] = st[i]
    return f


def dtype_code(dt):
    return _DTYPES[dt]


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
