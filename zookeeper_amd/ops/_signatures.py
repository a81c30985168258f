"""ctypes signatures of the C ABI exported by ``_zkamd.so``.

Kept next to the loader so the Python and C++ sides can be checked against
each other (``tests/test_native_abi.py`` compares this table with the symbols
of the built library)."""

import ctypes as C

P = C.c_void_p
I32 = C.c_int
I64 = C.c_int64
F32 = C.c_float

U64 = C.c_uint64
FP = C.POINTER(C.c_float)
IP = C.POINTER(C.c_int)

SIGNATURES = {
    # build provenance (csrc/build.py embeds the source digest)
    "zk_build_digest": (C.c_char_p, []),
    # host runtime
    "zk_gather_rows": (I32, [P, I64, P, I64, P, I32]),
    # native RCCL communicator (runtime/comm.cpp; parallel/rccl.py)
    "zk_comm_load": (I32, [C.c_char_p]),
    "zk_comm_loaded": (I32, []),
    "zk_comm_unique_id": (I32, [P]),
    "zk_comm_init": (I32, [P, I32, I32, P]),
    "zk_comm_count": (I32, [P, P]),
    "zk_comm_all_reduce": (I32, [P, P, P, I64, I32, I32, P]),
    "zk_comm_broadcast": (I32, [P, P, P, I64, I32, I32, P]),
    "zk_comm_group_start": (I32, []),
    "zk_comm_group_end": (I32, []),
    "zk_comm_destroy": (I32, [P, I32]),
    "zk_comm_async_error": (I32, [P, IP]),
    # preprocessing
    "zk_normalize_flip_c3": (I32, [P, P, I32, I32, I32, FP, FP, I32, U64, P]),
    "zk_normalize_flip_pack_c3": (I32, [P, P, P] + [I32] * 7 + [FP, FP, I32, U64, P]),
    # binary convolution
    "zk_sign_pack": (I32, [P, P, P, P, P, I64, F32, P]),
    "zk_weight_pack": (I32, [P, P, P, P, P, P, I32, I32, I32, P]),
    "zk_unpack_sign": (I32, [P, P, I64, P]),
    "zk_bconv_fwd": (I32, [P, P, P, P, P] + [I32] * 14 + [P]),
    "zk_bconv_dgrad": (I32, [P, P, P, P, P] + [I32] * 13 + [P]),
    "zk_igemm_dgrad": (I32, [P, P, P, P, P] + [I32] * 13 + [P]),
    "zk_igemm_dgrad_bnsum": (I32, [P] * 9 + [I32] * 15 + [P]),
    "zk_igemm_dgrad_fstats": (I32, [P] * 4 + [I32] * 14 + [P]),
    "zk_igemm_dgrad_ex": (I32, [P] * 8 + [I32, P] + [I32] * 14 + [P]),
    "zk_bn_bwd_tiles_reduce": (I32, [P, I32, I32, P, P]),
    "zk_igemm_fwd": (I32, [P, P, P, P] + [I32] * 16 + [P]),
    "zk_igemm_fwd_fp4": (I32, [P, P, P, P] + [I32] * 16 + [P]),
    "zk_bfwd_supported": (I32, [I32] * 10),
    "zk_bfwd_fp4": (I32, [P, P, P, P] + [I32] * 8 + [P]),
    "zk_igemm_wgrad": (I32, [P, P, P, P] + [I32] * 13 + [F32, I32, I32, P, I64, P]),
    "zk_igemm_wgrad_ws_bytes": (I64, [I32] * 14),
    "zk_wgrad_slab_reduce": (I32, [P, I32, I64, P, F32, P, P]),
    # row-streaming 3x3 weight gradient (wgrad_rows.hip)
    "zk_wgrad_rows_plan": (I32, [I32] * 6 + [P, P]),
    "zk_wgrad_rows_lab": (I32, [I32, P]),
    "zk_wgrad_rows": (I32, [P] * 5 + [I64, P, I64] + [I32] * 7 + [F32, I32, P]),
    "zk_igemm_dgrad_supported": (I32, [I32] * 13),
    "zk_set_option": (I32, [I32, I32]),
    "zk_bn_bwd_reduce_blocks": (I32, []),
    "zk_bn_stats_bf16_parts": (I32, [P, P, I64, I32, IP, P]),
    "zk_bn_finalize_f64_parts": (I32, [P, I32, I32, C.c_double, P, P, F32, F32, P, P, P, P]),
    "zk_bn_finalize_f64_stripes": (I32, [P, I32, I32, C.c_double, P, P, F32, F32, P, P, P, P]),
    "zk_bn_bwd_reduce_relu_bf16_parts": (I32, [P, P, P, P, I64, I32, IP, P]),
    "zk_get_option": (I32, [I32]),
    "zk_igemm_fwd_bf16": (I32, [P, P, P] + [I32] * 14 + [P]),
    "zk_igemm_fwd_bf16_supported": (I32, [I32] * 13),
    "zk_igemm_fwd_supported": (I32, [I32] * 15),
    "zk_bconv_wgrad": (I32, [P, P, P, P] + [I32] * 13 + [F32, I32, I32, P]),
    "zk_bn_apply_res_bf16": (I32, [P, P, P, P, P, I64, I32, I32, P]),
    "zk_bn_bwd_dx_res_bf16": (I32, [P, P, P, P, P, P, I64, I32, P]),
    # small-K convolutions (smallconv.hip)
    "zk_smallk_conv_fwd": (I32, [P, P, P] + [I32] * 12 + [P]),
    "zk_smallk_pack": (I32, [P, P] + [I32] * 5 + [I64] * 4 + [I32, P]),
    "zk_smallk_conv_wgrad": (I32, [P, P, P, P, P] + [I32] * 12 + [F32, I32, P]),
    "zk_smallk_conv_wgrad_blocks": (I32, [I32] * 4),
    "zk_band_conv_ok": (I32, [I32] * 10),
    "zk_band_conv_fwd": (I32, [P, P, P] + [I32] * 12 + [P]),
    "zk_band_conv_wgrad_parts": (I32, [I32] * 4),
    "zk_band_conv_wgrad": (I32, [P] * 5 + [I32] * 12 + [F32, I32, P]),
    # batch norm
    "zk_bn_finalize": (I32, [P, I32, I32, C.c_double, P, P, F32, F32, P, P, P, P, P, P, P]),
    "zk_bn_apply": (I32, [P, P, P, P, P, I64, I32, P]),
    "zk_bn_apply_sign": (I32, [P, P, P, P, P, P, P, P, F32, I64, I32, P]),
    "zk_bn_apply_sign_pool": (I32, [P, P, P, P, P, P, P, P, F32, P, I32, I32, I32, I32, P]),
    "zk_bn_bwd_reduce": (I32, [P, P, P, P, P, I64, I32, I32, P]),
    "zk_bn_bwd_dx": (I32, [P, P, P, P, I64, I32, I32, P]),
    "zk_ste_combine": (I32, [P, P, P, P, I64, P]),
    "zk_bn_bwd_coef": (I32, [P, P, P, P, C.c_double, I32, I32, I32, P, P, P, P]),
    # batch norm (bf16) and pooling
    "zk_bn_stats_bf16": (I32, [P, P, I64, I32, P]),
    "zk_bn_finalize_f64": (I32, [P, I32, C.c_double, P, P, F32, F32, P, P, P, P]),
    "zk_bn_apply_bf16": (I32, [P, P, P, I64, I32, I32, P]),
    "zk_bn_apply_bf16_sign": (I32, [P, P, P, P, P, P, F32, I64, I32, I32, P]),
    "zk_bn_bwd_reduce_bf16": (I32, [P, P, P, P, P, I64, I32, P]),
    "zk_bn_bwd_dx_bf16": (I32, [P, P, P, P, P, I64, I32, P]),
    "zk_bn_bwd_reduce_relu_bf16": (I32, [P, P, P, P, I64, I32, P]),
    "zk_bn_bwd_dx_relu_bf16": (I32, [P, P, P, P, P, I64, I32, P]),
    "zk_bn_bwd_parts_max": (I32, []),
    "zk_bn_bwd_reduce_bf16_parts": (I32, [P, P, P, P, P, I64, I32, IP, P]),
    # depthwise convolution
    "zk_dw_fwd": (I32, [P, P, P] + [I32] * 10 + [P]),
    "zk_dw_dgrad": (I32, [P, P, P] + [I32] * 10 + [P]),
    "zk_dw_wgrad": (I32, [P, P, P, P] + [I32] * 10 + [P]),
    "zk_dw_wgrad_blocks": (I32, [I32] * 4),
    # softmax cross-entropy
    "zk_xent_fwd": (I32, [P, P, P, P, P, I32, I32, F32, P, P]),
    "zk_xent_bwd": (I32, [P, P, P, P, P, I32, I32, F32, P]),
    # classifier head: (ReLU) + global average pool + fp32 dense layer
    "zk_head_fwd": (I32, [P, P, P, P, P] + [I32] * 5 + [P]),
    "zk_head_bwd": (I32, [P] * 8 + [I32] * 5 + [P]),
    "zk_gap_fwd": (I32, [P, P] + [I32] * 5 + [P]),
    "zk_gap_bwd": (I32, [P, P, P] + [I32] * 4 + [P]),
    # fused ImageNet stem
    "zk_stem_pack_input": (I32, [P, P] + [I32] * 8 + [P]),
    "zk_stem_pack_weight": (I32, [P, P] + [I32] * 4 + [P]),
    "zk_stem_conv_fwd": (I32, [P, P, P, P] + [I32] * 11 + [IP, P]),
    "zk_stem_max_parts": (I32, [I32, I32, I32]),
    "zk_stem_max_pool_parts": (I32, []),
    "zk_bn_finalize_partials": (I32, [P, I32, I32, C.c_double, P, P, F32, F32, P, P, P, P]),
    "zk_bn_finalize_partials_ws": (I32, [P, I32, I32, C.c_double, P, P, F32, F32, P, P, P, P,
                                         P]),
    "zk_bn_finalize_ws_bytes": (I64, [I32]),
    "zk_reduce_partials": (I32, [P, I32, I32, P, P]),
    "zk_stem_pool_fwd": (I32, [P, P, P, P, P] + [I32] * 10 + [IP, P]),
    "zk_stem_pool_bwd_sums": (I32, [P, P, P, P, P, P] + [I32] * 10 + [IP, P]),
    "zk_stem_dy1": (I32, [P, P, P, P, P, P] + [I32] * 10 + [P]),
    "zk_stem_wgrad": (I32, [P, P, P, P] + [I32] * 11 + [P]),
    "zk_stem_wgrad_splits": (I32, [I32] * 4),
    # recompute-fused stem (stem_fused.hip)
    "zk_stem_fused_blocks": (I32, [I32] * 6),
    "zk_stem_fused_slab_floats": (I32, []),
    "zk_stem_fused_slab_extra": (I32, []),
    "zk_stem_fwd_fused": (I32, [P] * 6 + [I32] * 11 + [IP, P]),
    "zk_stem_pool_relu": (I32, [P, P, P, P, I64, IP, P]),
    "zk_stem_pool_bwd_sums_ya": (I32, [P, P, P, P, I64, IP, P]),
    "zk_stem_bn2_bwd_sums": (I32, [P] * 7 + [I64, IP, P]),
    "zk_stem_bwd_fused": (I32, [P] * 8 + [I32] * 11 + [P]),
    "zk_maxpool_fwd": (I32, [P, P, P] + [I32] * 11 + [P]),
    "zk_maxpool_bwd": (I32, [P, P, P] + [I32] * 10 + [P]),
    "zk_avgpool2_fwd": (I32, [P, P] + [I32] * 6 + [P]),
    "zk_avgpool2_bwd": (I32, [P, P] + [I32] * 6 + [P]),
    "zk_avgpool2_bwd_add": (I32, [P, P, P] + [I32] * 6 + [P]),
    # optimizers
    "zk_adam_step": (I32, [P, P, P, P, P, I32, F32, F32, F32, F32, F32, F32, F32, F32, P, P]),
    "zk_sgd_step": (I32, [P, P, P, P, I32, F32, F32, F32, F32, I32, P, P]),
    "zk_weight_images": (I32, [P, P, I32, I64, P]),
    "zk_zero": (I32, [P, I64, P]),
    "zk_xent_finalize": (I32, [P, P, P, I32, P]),
}
