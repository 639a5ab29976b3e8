"""ctypes binding of libreidmi.so (the C ABI in include/reidmi.h).

This is the product's only route to compute: there is no CPU or PyTorch fallback.
If the library is missing or no GPU is present, calls raise loudly.
"""
import ctypes
import os

import torch

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libreidmi.so")
TOOLS_LIB_PATH = os.path.join(PKG, "libreidmi_tools.so")  # tests / A-B tools only (reidmi_tools.h)

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f32 = ctypes.c_float
_u16 = ctypes.c_uint16

# name -> argtypes (all return int status)
# entry points returning int64 besides the *_bytes sizes
INT64_RESULT = {"reidmi_rr_rank_rows_f16_pass_rows"}

SIGNATURES = {
    "reidmi_row_sqnorm_f32": [_vp, _i64, _i64, _i64, _vp, _vp],
    "reidmi_l2norm_f32": [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp],
    "reidmi_distmat_f32": [_vp, _i64, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp],
    "reidmi_cosine_f32": [_vp, _i64, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _vp],
    "reidmi_distmat_f16_workspace_bytes": [_i64, _i64, _i64],
    "reidmi_distmat_f16": [_vp, _i64, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp],
    "reidmi_topk_rows_f32": [_vp, _i64, _i64, _i64, _vp, _i32, _vp, _vp, _i64, _vp],
    "reidmi_eval_rows": [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp],
    "reidmi_eval_rows_workspace_bytes": [_i64],
    "reidmi_gemm_f16": [_i32, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp],
    "reidmi_rerank_workspace_bytes": [_i64, _i64, _i32, _i32, _i32, _i32],
    "reidmi_rerank": [_vp, _i64, _i64, _i64, _i64, _i32, _i32, _u16, _f32, _vp, _i64, _vp, _i64, _vp, _vp],
    "reidmi_rerank_from_dist": [_vp, _vp, _i64, _i64, _i32, _i32, _i32, _u16, _f32, _vp, _i64, _vp, _i64, _vp,
                                _vp],
    "reidmi_rr_caps": [_i64, _i32, _i32, _vp, _vp, _vp, _vp],
    "reidmi_rr_rank_rows": [_vp, _i64, _i64, _i64, _vp, _i64, _i64, _i32, _vp, _vp, _vp, _i64, _vp],
    "reidmi_rr_feat16": [_vp, _i64, _i64, _i64, _vp, _i64, _i64, _vp, _vp],
    "reidmi_rr_norm_max": [_vp, _vp, _i64, _vp, _vp],
    "reidmi_rr_rank_rows_f16": [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _vp, _vp, _vp,
                                _vp, _i64, _vp],
    "reidmi_rr_rank_rows_f16_ex": [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _vp, _vp,
                                   _vp, _vp, _i64, _i32, _vp],
    "reidmi_rr_rank_rows_f16_pass_rows": [_i64, _i64, _i64, _i32, _i32],
    "reidmi_rr_tri_plan": [_i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp],
    "reidmi_rr_tri_init": [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp],
    "reidmi_rr_tri_sample": [_vp, _i64, _i64, _vp, _vp, _vp, _i64, _i64, _i32, _vp, _vp, _i64, _i64, _i64, _vp, _i64,
                             _vp, _vp, _vp, _i32, _vp],
    "reidmi_rr_tri_survivors": [_vp, _i64, _i64, _vp, _vp, _i64, _i64, _vp, _vp, _i64, _i64, _vp, _vp, _i32, _vp],
    "reidmi_rr_sv_select": [_vp, _vp, _i32, _vp, _vp, _i64, _i64, _vp, _i64, _i64, _i32, _vp, _vp, _vp, _vp],
    "reidmi_rr_sv_pack": [_vp, _vp, _i32, _i64, _vp, _vp, _vp],
    "reidmi_rr_sv_merge": [_vp, _vp, _i32, _i64, _vp, _vp, _vp, _vp],
    "reidmi_rr_v_rows": [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _i32, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _i64, _vp,
                         _vp],
    "reidmi_rr_row_offsets": [_vp, _i64, _vp, _vp],
    "reidmi_rr_pack": [_vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp],
    "reidmi_rr_qe_rows": [_vp, _i32, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "reidmi_rr_qe_deferred": [_vp, _i32, _i32, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp,
                              _vp, _i64, _vp, _vp],
    "reidmi_rr_csc_workspace_bytes": [_i64, _i64],
    "reidmi_rr_csc": [_i64, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _i64, _vp],
    "reidmi_rr_jaccard_rows": [_vp, _i64, _i64, _i64, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                               _u16, _f32, _vp, _i64, _vp, _i64, _vp, _i64, _vp],
    "reidmi_rr_jaccard_bounds_bytes": [_i64, _i64],
    "reidmi_rowmax_f32": [_vp, _i64, _i64, _i64, _vp, _vp],
    "reidmi_nonzero_i32": [_vp, _i64, _vp, _vp, _vp],
    "reidmi_gather_rows_f32": [_vp, _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp],
    "reidmi_attn_lpad": [_i32],
    "reidmi_prof_enable": [_i32],
    "reidmi_prof_collect": [_i32, _vp, _vp, _vp],
    "reidmi_prof_collect_min": [_i32, ctypes.c_double, _vp, _vp, _vp],
    "reidmi_mhsa_f16": [_vp, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp],
    "reidmi_layernorm": [_vp, _i64, _i64, _vp, _i64, _vp, _vp, _f32, _vp, _i64, _vp, _i64, _vp],
    "reidmi_row_stats_f16": [_vp, _i64, _i64, _i64, _vp, _vp, _vp],
    "reidmi_gemm_f16_resid_partials": [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _i64, _vp, _vp],
    "reidmi_feature_tta_avg": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _i64, _vp],
    "reidmi_feature_tta_mm": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _vp, _i64, _vp],
    "reidmi_class_mean_normalize": [_vp, _vp, _i64, _i64, _vp, _vp],
    "reidmi_prompt_build": [_vp, _i32, _vp, _i32, _vp, _i64, _vp, _i32, _i64, _i32, _vp, _vp, _vp],
    "reidmi_preprocess_u8": [_vp, _vp, _i64, _i32, _i32, _i32, _i32, _vp, _vp, _i32, _vp, _vp],
    "reidmi_preprocess_lds_size": [_i32, _i32, _i32, _i32, _vp],
    "reidmi_jpeg_plan": [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp],
    "reidmi_jpeg_decode": [_vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp],
    "reidmi_files_size": [_vp, _i64, _vp, _i32],
    "reidmi_files_read": [_vp, _i64, _vp, _vp, _vp, _i32],
    "reidmi_bytes_gather": [_vp, _i64, _vp, _vp, _i32],
    "reidmi_comm_unique_id": [_vp],
    "reidmi_comm_init": [_vp, _i32, _i32, _vp, _i32],
    "reidmi_comm_destroy": [_vp],
    "reidmi_comm_rank": [_vp, _vp, _vp],
    "reidmi_comm_allgather_rows_scratch_bytes": [_i32, _i64, _i64],
    "reidmi_comm_allgather_rows": [_vp, _vp, _i64, _i64, _vp, _vp, _i64, _vp],
    "reidmi_comm_allreduce": [_vp, _vp, _vp, _i64, _i32, _vp],
}
# libreidmi_tools.so only (include/reidmi_tools.h): forced kernel variants for tests / A-B timing
TOOLS_SIGNATURES = {
    "reidmi_distmat_f32_variant": [_vp, _i64, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _vp, _i32, _vp],
    "reidmi_gemm_f16_tiled": [_i32, _vp, _i64, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp],
    "reidmi_qkv_attention_f16": [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32,
                                 _vp],
    "reidmi_gemm_f16_w4": [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _vp, _vp, _i64, _i32, _vp],
    "reidmi_gemm_f16_qkv": [_vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "reidmi_mhsa_f16_rr": [_vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp],
}
# entry points with struct arguments are typed in model.py (reidmi_vit_*, reidmi_text_*)
STRUCT_ENTRY_POINTS = ("reidmi_vit_workspace_bytes", "reidmi_vit_forward", "reidmi_text_workspace_bytes",
                       "reidmi_text_forward", "reidmi_vit_pack_bytes", "reidmi_vit_weights_pack",
                       "reidmi_text_pack_bytes", "reidmi_text_weights_pack")

_LIB = None
_TOOLS = None


class ReidmiError(RuntimeError):
    pass


def _open(path, tools):
    if not os.path.exists(path):
        raise ReidmiError(f"{path} is not built: run `python __graft_entry__.py build` "
                          "(there is no CPU fallback)")
    from . import build_lib
    if not build_lib.manifest_matches(tools):
        raise ReidmiError(f"{path} was not built from the sources next to it (its manifest differs): "
                          "run `python __graft_entry__.py build`")
    L = ctypes.CDLL(path)
    L.reidmi_last_error.restype = ctypes.c_char_p
    L.reidmi_abi_version.restype = _i32
    table = dict(SIGNATURES, **TOOLS_SIGNATURES) if tools else SIGNATURES
    for name, args in table.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = _i64 if name.endswith("_bytes") or name in INT64_RESULT else _i32
    return L


def load():
    """Load libreidmi.so (torch's HIP runtime is already loaded by `import torch`, so the
    library's libamdhip64.so.7 dependency resolves to that same runtime)."""
    global _LIB
    if _LIB is None:
        _LIB = _open(LIB_PATH, False)
    return _LIB


def load_tools():
    """libreidmi_tools.so: the product entry points plus reidmi_tools.h's forced variants (tests
    and A/B tools only; its static state — errors, timing hooks — is its own)."""
    global _TOOLS
    if _TOOLS is None:
        _TOOLS = _open(TOOLS_LIB_PATH, True)
    return _TOOLS


def call(name, *args):
    L = load()
    rc = getattr(L, name)(*args)
    if rc != 0:
        raise ReidmiError(f"{name} failed ({rc}): {L.reidmi_last_error().decode()}")


def call_tools(name, *args):
    L = load_tools()
    rc = getattr(L, name)(*args)
    if rc != 0:
        raise ReidmiError(f"{name} failed ({rc}): {L.reidmi_last_error().decode()}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_cuda(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise ReidmiError("libreidmi operates on device tensors (got a CPU tensor)")
