"""Loader and build recipe of libdoko_amd.so (HIP, gfx950).

There is no CPU fallback: if the shared library is missing or no gfx950 device
is usable, the product API raises.
"""
import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "libdoko_amd.so")
# profiling builds (-DDK_PHASE_PROF) are loaded by setting DK_LIB to their path
PROF_LIB_PATH = os.path.join(PKG_DIR, "libdoko_amd_prof.so")
SRC = os.path.join(PKG_DIR, "csrc", "doko_amd.hip")
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared"]


def build(verbose=False, profiling=False):
    """Compile csrc/doko_amd.hip for gfx950 into the package directory (in-tree).
    profiling=True builds the phase-timer variant libdoko_amd_prof.so."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    out = PROF_LIB_PATH if profiling else LIB_PATH
    cmd = [hipcc] + HIPCC_FLAGS + (["-DDK_PHASE_PROF"] if profiling else []) + ["-o", out, SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True, cwd=PKG_DIR)
    return out


class dk_config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("max_roots", ctypes.c_uint32),
                ("max_iterations", ctypes.c_uint32), ("slot_capacity", ctypes.c_uint32)]


_lib = None
vp = ctypes.c_void_p
u32 = ctypes.c_uint32
u64 = ctypes.c_uint64


def lib():
    """Load libdoko_amd.so (importing torch first when available so that the
    process uses a single HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("DK_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError("libdoko_amd.so not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:
        import torch  # noqa: F401  (shares libamdhip64 with the extension)
    except Exception:
        pass
    L = ctypes.CDLL(path)
    sigs = {
        "dk_abi_version": (ctypes.c_int, []),
        "dk_status_string": (ctypes.c_char_p, [ctypes.c_int]),
        "dk_create": (vp, [ctypes.POINTER(dk_config)]),
        "dk_destroy": (None, [vp]),
        "dk_last_error": (ctypes.c_int, [vp]),
        "dk_pool_bytes": (u64, [vp]),
        "dk_pool_high_water": (ctypes.c_int, [vp, vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]),
        "dk_sync": (ctypes.c_int, [vp, vp]),
        "dk_last_search_ms": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_float)]),
        "dk_last_search_waves": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
        "dk_last_search_clocks": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
        "dk_new_game_batch": (ctypes.c_int, [vp, ctypes.c_int, vp, u32, vp]),
        "dk_new_game_batch_async": (ctypes.c_int, [vp, ctypes.c_int, vp, u32, vp, vp]),
        "dk_env_allowed_batch": (ctypes.c_int, [vp, vp, u32, ctypes.c_int, vp]),
        "dk_env_step_batch": (ctypes.c_int, [vp, vp, vp, u32]),
        "dk_env_rewards_batch": (ctypes.c_int, [vp, vp, u32, vp, vp]),
        "dk_env_rollout_batch": (ctypes.c_int, [vp, vp, vp, u32, vp]),
        "dk_env_rollout_batch_async": (ctypes.c_int, [vp, vp, vp, u32, vp, vp]),
        "dk_env_random_plies_batch": (ctypes.c_int, [vp, vp, vp, vp, u32]),
        "dk_search_batch": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, u32, u32, ctypes.c_double, vp, vp, vp]),
        "dk_search_batch_async": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, u32, u32, ctypes.c_double, vp, vp, vp, vp]),
        "dk_search_batch_rng": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, u32, u32, ctypes.c_double, vp, vp, vp]),
        "dk_search_batch_rng_async": (ctypes.c_int, [vp, ctypes.c_int, vp, vp, u32, u32, ctypes.c_double, vp, vp, vp, vp]),
        "dk_determinize_batch": (ctypes.c_int, [vp, vp, u32, u32, vp, vp]),
        "dk_determinize_batch_async": (ctypes.c_int, [vp, vp, u32, u32, vp, vp, vp]),
        "dk_fuse": (ctypes.c_int, [vp, vp, u32, u32, vp, ctypes.c_int, vp]),
        "dk_fuse_accumulate_async": (ctypes.c_int, [vp, vp, u32, u32, vp, ctypes.c_int, vp, vp, vp]),
        "dk_fuse_select_async": (ctypes.c_int, [vp, u32, ctypes.c_int, vp, vp, vp, vp, vp]),
        "dk_legal_actions_async": (ctypes.c_int, [vp, vp, u32, vp, vp]),
        "dk_env_step_batch_async": (ctypes.c_int, [vp, vp, vp, u32, vp]),
        "dk_env_random_plies_batch_async": (ctypes.c_int, [vp, vp, vp, vp, u32, vp]),
        "dk_decide_batch": (ctypes.c_int, [vp, vp, u32, u32, vp, u32, ctypes.c_double, ctypes.c_int, vp, vp]),
        "dk_az_begin_async": (ctypes.c_int, [vp, vp, vp, u32, u32, ctypes.c_int, vp, vp]),
        "dk_az_root_async": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_float, ctypes.c_float, vp]),
        "dk_az_rng_async": (ctypes.c_int, [vp, vp, ctypes.c_int, vp]),
        "dk_f32_libm_async": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, vp, vp]),
        "dk_az_select_async": (ctypes.c_int, [vp, ctypes.c_float, vp, vp, vp]),
        "dk_az_backup_async": (ctypes.c_int, [vp, vp, vp, vp]),
        "dk_az_finish_async": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_float, vp, vp, vp]),
        "dk_az_records_async": (ctypes.c_int, [vp, vp, u32, vp, vp]),
        "dk_az_step_async": (ctypes.c_int, [vp, vp, vp, u32, vp]),
        "dk_az_encode_async": (ctypes.c_int, [vp, vp, u32, vp, vp]),
        "dk_ar_begin_async": (ctypes.c_int, [vp, vp, u32, u32, vp, ctypes.c_float, vp, vp]),
        "dk_ar_guesses_async": (ctypes.c_int, [vp, vp, u32, vp, vp]),
        "dk_ar_prepare_async": (ctypes.c_int, [vp, vp, vp]),
        "dk_ar_choose_async": (ctypes.c_int, [vp, vp, ctypes.c_float, vp]),
        "dk_ar_output_async": (ctypes.c_int, [vp, vp, vp, vp, vp]),
        "dk_ar_fallback_async": (ctypes.c_int, [vp, u32, u32, vp, vp, vp, vp, vp, vp]),
        "dk_fuse_accumulate_masked_async": (ctypes.c_int, [vp, vp, u32, u32, vp, vp, ctypes.c_int, vp, vp, vp]),
        "dk_fdo_from_fields": (ctypes.c_int, [vp, vp]),
        "dk_is_consistent_batch": (ctypes.c_int, [vp, vp, vp, vp, u32, vp]),
        "dk_fdo_to_fields": (ctypes.c_int, [vp, vp]),
        "dk_do_from_fields": (ctypes.c_int, [vp, vp]),
        "dk_do_to_fields": (ctypes.c_int, [vp, vp]),
        "dk_net_embed_ln_bf16_async": (ctypes.c_int, [vp, u32, ctypes.POINTER(vp), u32, vp, vp, ctypes.c_float, vp, vp, vp]),
        "dk_net_add_ln_bf16_async": (ctypes.c_int, [vp, vp, u32, u32, vp, vp, ctypes.c_float, vp, vp]),
        "dk_net_attn62_bf16_async": (ctypes.c_int, [vp, vp, u32, u32, u32, vp]),
        "dk_net_fc_gelu_bf16_async": (ctypes.c_int, [vp, vp, vp, u32, u32, u32, vp, vp]),
        "dk_net_mlp_ln_bf16_async": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, u32, u32, u32, vp, vp, ctypes.c_float, vp, vp]),
        "dk_net_mlp_ln_f32x3_async": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, vp, vp, ctypes.c_float,
                                                     vp, vp]),
        "dk_net_qkv_attn_ln_f32x3_async": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, u32, u32, u32, vp, vp,
                                                          ctypes.c_float, vp, vp]),
        "dk_net_qkv_attn_ln_f32x3_ex_async": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_float, vp, vp, vp, vp, vp, vp, u32, u32,
                                                             u32, vp, vp, ctypes.c_float, vp, vp, vp, vp, vp]),
        "dk_net_mlp_ln_f32x3_ex_async": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_float, vp, vp, vp, vp, vp, vp, u32, u32, u32,
                                                        vp, vp, ctypes.c_float, vp, vp, vp, vp]),
        "dk_net_class_pool_ln_f32_async": (ctypes.c_int, [vp, u32, u32, vp, u32, ctypes.c_float, vp, vp, ctypes.c_float,
                                                          vp, vp]),
        "dk_net_class_mlp_f32x3_async": (ctypes.c_int, [vp, u32, u32, u32, vp, vp, vp, vp, vp, vp, vp]),
        "dk_net_class_mlp_bf16_async": (ctypes.c_int, [vp, u32, u32, u32, vp, vp, vp, vp, vp, vp]),
        "dk_net_attn_ln_bf16_async": (ctypes.c_int, [vp, vp, vp, vp, u32, u32, u32, vp, vp, ctypes.c_float, vp, vp]),
        "dk_net_qkv_attn_ln_bf16_async": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, u32, u32, u32, vp, vp, ctypes.c_float, vp, vp]),
        "dk_net_class_pool_ln_bf16_async": (ctypes.c_int, [vp, u32, u32, vp, u32, ctypes.c_float, vp, vp, ctypes.c_float, vp, vp]),
        "dk_net_embed_ln_f32_async": (ctypes.c_int, [vp, u32, ctypes.POINTER(vp), u32, vp, vp, ctypes.c_float, vp, vp, vp]),
        "dk_net_add_ln_f32_async": (ctypes.c_int, [vp, vp, u32, u32, vp, vp, ctypes.c_float, vp, vp]),
        "dk_net_attn62_f32_async": (ctypes.c_int, [vp, vp, u32, u32, u32, vp]),
        "dk_net_gelu_f32_async": (ctypes.c_int, [vp, u64, vp]),
        "dk_net_add_bias_ln_f32_async": (ctypes.c_int, [vp, vp, vp, u32, u32, vp, vp, ctypes.c_float, vp, vp]),
        "dk_net_gelu_bias_f32_async": (ctypes.c_int, [vp, vp, u64, u32, vp]),
        "dk_net_attn62_bias_f32_async": (ctypes.c_int, [vp, vp, vp, u32, u32, u32, vp]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


# every symbol include/doko_amd.h declares (checked by the CPU test suite)
EXPORTED = [
    "dk_create", "dk_destroy", "dk_last_error", "dk_status_string", "dk_abi_version", "dk_new_game_batch",
    "dk_new_game_batch_async", "dk_env_allowed_batch", "dk_env_step_batch", "dk_env_rewards_batch",
    "dk_env_rollout_batch", "dk_env_rollout_batch_async", "dk_env_random_plies_batch", "dk_search_batch",
    "dk_search_batch_async", "dk_search_batch_rng", "dk_search_batch_rng_async", "dk_determinize_batch", "dk_determinize_batch_async", "dk_fuse",
    "dk_fuse_accumulate_async", "dk_fuse_select_async", "dk_decide_batch", "dk_sync", "dk_last_search_ms", "dk_last_search_waves", "dk_last_search_clocks",
    "dk_pool_bytes", "dk_legal_actions_async", "dk_env_step_batch_async", "dk_env_random_plies_batch_async",
    "dk_az_begin_async", "dk_az_root_async", "dk_az_rng_async", "dk_f32_libm_async", "dk_az_select_async", "dk_az_backup_async", "dk_az_finish_async",
    "dk_az_records_async", "dk_az_step_async", "dk_az_encode_async", "dk_net_embed_ln_bf16_async",
    "dk_net_add_ln_bf16_async", "dk_net_attn62_bf16_async", "dk_net_fc_gelu_bf16_async", "dk_net_mlp_ln_bf16_async", "dk_net_mlp_ln_f32x3_async", "dk_net_qkv_attn_ln_f32x3_async", "dk_net_qkv_attn_ln_f32x3_ex_async", "dk_net_mlp_ln_f32x3_ex_async", "dk_net_class_pool_ln_f32_async", "dk_net_class_mlp_f32x3_async", "dk_net_class_mlp_bf16_async", "dk_net_attn_ln_bf16_async", "dk_net_qkv_attn_ln_bf16_async", "dk_net_class_pool_ln_bf16_async",
    "dk_net_embed_ln_f32_async", "dk_net_add_ln_f32_async", "dk_net_attn62_f32_async", "dk_net_gelu_f32_async", "dk_net_add_bias_ln_f32_async", "dk_net_gelu_bias_f32_async", "dk_net_attn62_bias_f32_async", "dk_ar_begin_async", "dk_ar_guesses_async", "dk_ar_prepare_async",
    "dk_ar_choose_async", "dk_ar_output_async", "dk_ar_fallback_async", "dk_fuse_accumulate_masked_async",
    "dk_fdo_from_fields", "dk_fdo_to_fields", "dk_do_from_fields", "dk_do_to_fields", "dk_is_consistent_batch",
    "dk_pool_high_water",
]
