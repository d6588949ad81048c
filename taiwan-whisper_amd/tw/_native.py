"""ctypes binding of libtw_hip.so (include/tw_hip.h).

The library is built in-tree (`make -C taiwan-whisper_amd` / `__graft_entry__.build()`)
into `tw/_lib/libtw_hip.so`.  There is NO fallback: if the library is missing or a call
returns a non-zero status, this module raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TW_HIP_LIB", os.path.join(_HERE, "_lib", "libtw_hip.so"))

P, I64, I32, F32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float

# name -> argtypes (return type is always int status)
SIGNATURES = {
    "tw_gemm_bf16": [P, I64, I32, P, I64, I32, P, I64, I32, I32, I32, I32, I32, I64, I64, I64, F32, P,
                     P, I64, I64, I32, I32, P, I64, I64, I32, P],
    "tw_flac_info": [P, I64, P],
    "tw_flac_decode": [P, I64, P, I64, P],
    "tw_gemv_bf16": [P, I64, P, P, F32, P, I64, P, I64, I32, I32, I32, I32, P, P, I64, I32, P, I64, I32,
                     P, I64, I64, I32, P, P],
    "tw_layernorm_fwd": [P, I32, P, P, P, I32, P, P, I32, I32, F32, P],
    "tw_layernorm_bwd": [P, I32, P, P, P, P, I32, P, I32, P, P, I32, I32, P, I64, P],
    "tw_layernorm_bwd_ex": [P, I32, P, P, P, P, I32, P, I32, P, P, I32, I32, P, I64, P, I32, P],
    "tw_add_layernorm_fwd": [P, I32, P, P, P, P, P, P, P, I32, I32, F32, P],
    "tw_attn_fwd": [P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32, I32, F32, P],
    "tw_attn_bwd": [P, I64, P, I64, P, I64, P, I64, P, I64, P, P, I64, P, I64, P, I64, I32, I32, I32, I32,
                    I32, I32, F32, P, P],
    "tw_kl_ce": [P, P, I64, I32, P, I64, I32, F32, F32, F32, P, F32, P, P, P, P],
    "tw_logmel": [P, I32, P, P, P, P, P, P, P],
    "tw_logmel_len": [P, I32, I64, P, P, P, P, P, P, P],
    "tw_mel_to_conv_input": [P, P, I32, I32, I32, P],
    "tw_embed_fwd": [P, P, I32, P, I32, P, I32, I32, I32, I32, I32, P],
    "tw_embed_bwd": [P, P, P, I32, I32, I64, P],
    "tw_cast_f32_bf16": [P, P, I64, P],
    "tw_transpose_bf16": [P, I64, I32, I32, P, I64, P],
    "tw_colsum": [P, I32, I64, I32, I32, P, I32, I32, P, I64, P],
    "tw_l2norm": [P, I64, P, P, P],
    "tw_adamw": [P, P, P, P, P, I64, F32, F32, F32, F32, F32, I32, P, F32, P],
    "tw_clip_scale": [P, I64, P, F32, P],
    "tw_im2col3": [P, I64, P, I32, I32, I32, I32, P],
    "tw_col2im_s2": [P, P, I32, I32, I32, I32, P],
    "tw_gelu_bwd": [P, I32, P, P, I64, P],
    "tw_shift_tokens_right": [P, P, I32, I32, I64, I64, P],
    "tw_count_valid": [P, I64, P, P],
    "tw_decode_attn": [P, I64, P, I64, I64, P, I64, I64, P, I64, I32, I32, I32, P, I32, F32, I32, P],
    "tw_decode_attn_hs": [P, I64, P, I64, I64, I64, P, I64, I64, I64, P, I64, I32, I32, I32, P, I32, F32, I32, P],
    "tw_greedy_select": [P, I64, I32, I32, I32, P, P, I32, I64, P, P, I64, I32, P, P, I32, P],
    "tw_greedy_select_ts": [P, I64, I32, I32, I32, P, P, I64, P, P, I64, I32, P, P, I32, I32, I32, I32, P, P],
    "tw_select_sample": [P, I64, I32, I32, I32, P, P, I32, I64, P, P, I64, I32, P, P, I32, P, P, P],
    "tw_select_sample_ts": [P, I64, I32, I32, I32, P, P, I64, P, P, I64, I32, P, P, I32, I32, I32, I32, P, P, P, P],
    "tw_token_logprob": [P, I64, I32, I32, I32, I32, P, P],
    "tw_embed_step": [P, P, I32, P, I32, P, I32, I32, I32, P, P],
    "tw_kv_append": [P, I64, P, I64, I64, I32, I32, I32, P, P],
    "tw_kv_head_major": [P, I64, P, I32, I32, I32, I32, P],
    "tw_step_advance": [P, I32, P],
    # fp16 arithmetic path (torch_dtype=float16 decode: run_eval.py:99, run_pseudo_labelling.py:461-463)
    "tw_gemm_f16": [P, I64, I32, P, I64, I32, P, I64, I32, I32, I32, I32, I32, I64, I64, I64, F32, P,
                    P, I64, I64, I32, I32, P, I64, I64, I32, P],
    "tw_gemv_f16": [P, I64, P, P, F32, P, I64, P, I64, I32, I32, I32, I32, P, P, I64, I32, P, I64, I32,
                    P, I64, I64, I32, P, P],
    "tw_attn_fwd_f16": [P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32, I32, F32, P],
    "tw_mel_to_conv_input_f16": [P, P, I32, I32, I32, P],
    # fp16-autocast training (run_distillation.py:815-817 --dtype float16)
    "tw_attn_bwd_f16": [P, I64, P, I64, P, I64, P, I64, P, I64, P, P, I64, P, I64, P, I64, I32, I32, I32, I32,
                        I32, I32, F32, P, P],
    "tw_gelu_bwd_f16": [P, I32, P, P, I64, P],
    "tw_cast_f32_f16": [P, P, I64, P],
    "tw_add_layernorm_fwd_f16": [P, I32, P, P, P, P, P, P, P, I32, I32, F32, P],
    "tw_adamw_ex": [P, P, P, P, P, I32, I64, F32, F32, F32, F32, F32, I32, P, F32, F32, P],
    # fp32 arithmetic path
    "tw_gemm_f32": [P, I64, I32, P, I64, I32, P, I64, I32, I32, I32, I32, I64, I64, I64, I32, I64, I64, I64, F32,
                    P, P, I64, I64, I32, P, I64, I64, I32, P],
    "tw_attn_fwd_f32": [P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32, I32, F32, P, I64, P],
    "tw_attn_bwd_f32": [P, I64, P, I64, P, I64, P, I64, P, I64, P, P, I64, P, I64, P, I64, I32, I32, I32, I32, I32,
                        I32, F32, P, I64, P],
    "tw_mel_to_conv_input_f32": [P, P, I32, I32, I32, P],
    "tw_im2col3_f32": [P, I64, P, I32, I32, I32, I32, P],
    "tw_gelu_bwd_f32": [P, P, P, I64, P],
}

STATUS = {1: "invalid argument / shape", 2: "unsupported configuration", 3: "HIP launch error"}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"tw: HIP library not built: {LIB_PATH} (run `make -C taiwan-whisper_amd` "
                               "or __graft_entry__.build()); there is no CPU fallback")
        l = ctypes.CDLL(LIB_PATH)
        for name, argt in SIGNATURES.items():
            f = getattr(l, name)
            f.argtypes = argt
            f.restype = ctypes.c_int
        _lib = l
    return _lib


def call(name: str, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"tw: {name} failed with status {rc} ({STATUS.get(rc, 'unknown')})")
    return rc
