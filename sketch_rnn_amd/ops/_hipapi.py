"""ctypes bindings for ``libskrnn_hip.so`` (C ABI, raw device pointers).

The argument structs mirror ``FwdArgs`` / ``BwdArgs`` in
``csrc/lstm_cell.hip`` field for field; :func:`bind` checks their sizes
against the library so a layout drift fails at load time, not in a kernel.
"""
from __future__ import annotations

import ctypes as C

_p = C.c_void_p
_i64 = C.c_int64
_f = C.c_float
_u32 = C.c_uint32
_i = C.c_int


class LstmFwdArgs(C.Structure):
    _fields_ = [
        ("B", _i), ("H", _i),
        ("grp_rows", _i),
        ("xp", _p), ("ld_xp", _i64),
        ("R", _p), ("ld_R", _i64),
        ("R_nslab", _i), ("R_slab", _i64),
        ("vec", _p), ("vec_gs", _i64), ("vec_ld", _i64),
        ("vec_bias", _p),
        ("bias", _p),
        ("c_prev", _p),
        ("ln_g", _p), ("ln_b", _p), ("lnc_g", _p), ("lnc_b", _p),
        ("reset", _p),
        ("init_h", _p), ("init_c", _p),
        ("forget_bias", _f), ("keep", _f),
        ("seed", _p), ("stream", _u32), ("step", _u32),
        ("h_out", _p), ("c_out", _p), ("act", _p), ("xhat", _p), ("rstd", _p), ("chat", _p),
        ("h_carry", _p),
        ("h_lp", _p), ("ld_lp", _i64), ("lp_kind", _i),
        ("c_carry", _p),
        ("cluster", _i), ("part", _p), ("err", _p),
        ("r_lp", _p),
        ("gpre", _p), ("gstats", _p), ("gstat_tiles", _i),
        ("save_lp", _i),
        ("h_q8", _p), ("ld_q8", _i64), ("h_qs", _p),
    ]


class LstmBwdArgs(C.Structure):
    _fields_ = [
        ("B", _i), ("H", _i),
        ("grp_rows", _i),
        ("dh_out", _p),
        ("dho_nslab", _i), ("dho_slab", _i64),
        ("dh_rec", _p), ("ld_dh_rec", _i64),
        ("dhr_nslab", _i), ("dhr_slab", _i64),
        ("dh_rec2", _p), ("ld_dh_rec2", _i64),
        ("dhr2_nslab", _i), ("dhr2_slab", _i64),
        ("dc_rec", _p),
        ("act", _p), ("c_new", _p), ("c_prev", _p),
        ("xhat", _p), ("rstd", _p), ("chat", _p),
        ("ln_g", _p), ("lnc_g", _p), ("lnc_b", _p),
        ("xp", _p), ("ld_xp", _i64),
        ("R", _p), ("ld_R", _i64),
        ("R_nslab", _i), ("R_slab", _i64),
        ("vec", _p), ("vec_gs", _i64), ("vec_ld", _i64),
        ("vec_bias", _p),
        ("reset", _p),
        ("keep", _f), ("seed", _p), ("stream", _u32), ("step", _u32),
        ("dG", _p), ("ld_dG", _i64),
        ("dG_lp", _p), ("ld_dG_lp", _i64), ("dG_lp_kind", _i),
        ("dxp", _p), ("ld_dxp", _i64), ("dxp_kind", _i),
        ("dvec", _p), ("dvec_kind", _i),
        ("dlny", _p), ("dlncy", _p),
        ("dinit_h", _p), ("dinit_c", _p),
        ("cluster", _i), ("part", _p), ("err", _p),
        ("ln_b", _p), ("forget_bias", _f),
        ("r_lp", _p),
        ("save_lp", _i),
        ("xp_lp", _i),
    ]


class GruFwdArgs(C.Structure):
    """Mirror of ``GruFwdArgs`` in csrc/gru_cell.hip."""
    _fields_ = [
        ("B", _i), ("H", _i),
        ("xg", _p), ("ld_xg", _i64),
        ("Rg", _p), ("ld_Rg", _i64), ("Rg_nslab", _i), ("Rg_slab", _i64),
        ("xc", _p), ("ld_xc", _i64),
        ("Rc", _p), ("ld_Rc", _i64), ("Rc_nslab", _i), ("Rc_slab", _i64),
        ("h_prev", _p),
        ("reset", _p), ("init_h", _p),
        ("ru", _p),
        ("rh_lp", _p), ("ld_rh", _i64), ("rh_kind", _i),
        ("cand", _p),
        ("h_out", _p),
        ("h_carry", _p),
        ("h_lp", _p), ("ld_lp", _i64), ("lp_kind", _i),
    ]


class GruBwdArgs(C.Structure):
    """Mirror of ``GruBwdArgs`` in csrc/gru_cell.hip."""
    _fields_ = [
        ("B", _i), ("H", _i),
        ("dh_out", _p),
        ("dh_elem", _p),
        ("dhg", _p), ("ld_dhg", _i64), ("dhg_nslab", _i), ("dhg_slab", _i64),
        ("ru", _p), ("cand", _p), ("h_prev", _p),
        ("reset", _p),
        ("dinit_h", _p),
        ("dh_tot", _p),
        ("dpc", _p), ("dpc_lp", _p), ("dpc_kind", _i),
        ("drh", _p), ("ld_drh", _i64), ("drh_nslab", _i), ("drh_slab", _i64),
        ("dpg", _p), ("dpg_lp", _p), ("dpg_kind", _i),
        ("dh_elem_out", _p),
    ]


class FusedFwdArgs(C.Structure):
    """Mirror of ``FusedFwdArgs`` in csrc/lstm_fused.hip."""
    _fields_ = [
        ("B", _i), ("H", _i), ("nd", _i),
        ("A", _p), ("lda", _i64),
        ("WT", _p), ("w_gs", _i64),
        ("xp", _p), ("ld_xp", _i64),
        ("c_prev", _p),
        ("reset", _p),
        ("init_h", _p), ("init_c", _p),
        ("forget_bias", _f), ("keep", _f),
        ("seed", _p), ("stream", _u32), ("step", _u32),
        ("h_out", _p), ("c_out", _p), ("act", _p),
        ("h_carry", _p), ("c_carry", _p),
        ("h_next", _p), ("ld_next", _i64),
    ]


class FusedBwdArgs(C.Structure):
    """Mirror of ``FusedBwdArgs`` in csrc/lstm_fused.hip."""
    _fields_ = [
        ("B", _i), ("H", _i), ("nd", _i),
        ("dG_next", _p), ("ld_dgn", _i64),
        ("W", _p), ("w_gs", _i64),
        ("dh_extra", _p),
        ("dh_out", _p),
        ("dc_rec", _p),
        ("act", _p), ("c_new", _p), ("c_prev", _p),
        ("reset", _p),
        ("keep", _f), ("seed", _p), ("stream", _u32), ("step", _u32),
        ("dG", _p), ("dG_lp", _p),
        ("dinit_h", _p), ("dinit_c", _p),
    ]


class PFwdLayer(C.Structure):
    """Mirror of ``PFwdLayer`` in csrc/lstm_persist.hip."""
    _fields_ = [
        ("WT", _p), ("w_gs", _i64),
        ("kin", _i),
        ("xp", _p), ("xp_ts", _i64), ("xp_ld", _i64),
        ("c0", _p),
        ("init_h", _p), ("init_c", _p),
        ("hlp", _p), ("hup", _p), ("h_out", _p), ("c_out", _p), ("c_carry", _p), ("act", _p),
        ("hT", _p), ("cT", _p),
        ("keep", _f), ("stream", _u32),
        ("h_last", _p),
    ]


class PFwdArgs(C.Structure):
    _fields_ = [
        ("T", _i), ("B", _i), ("nd", _i), ("L", _i), ("H", _i), ("nrb", _i),
        ("ly", PFwdLayer * 2),
        ("reset", _p),
        ("forget_bias", _f),
        ("seed", _p),
        ("flags", _p),
        ("err", _p),
        ("tlen", _p),
    ]


class PBwdLayer(C.Structure):
    """Mirror of ``PBwdLayer`` in csrc/lstm_persist.hip."""
    _fields_ = [
        ("Wr", _p), ("wr_gs", _i64),
        ("Wu", _p),
        ("dh_out", _p),
        ("dhT", _p), ("dcT", _p),
        ("act", _p), ("c_out", _p), ("c_carry", _p), ("c0", _p),
        ("dg_lp", _p), ("dg", _p),
        ("dh0", _p), ("dc0", _p),
        ("dinit_h", _p), ("dinit_c", _p),
        ("keep", _f), ("stream", _u32),
        ("dh_last", _p),
    ]


class PBwdArgs(C.Structure):
    _fields_ = [
        ("T", _i), ("B", _i), ("nd", _i), ("L", _i), ("H", _i), ("nrb", _i),
        ("ly", PBwdLayer * 2),
        ("reset", _p),
        ("seed", _p),
        ("flags", _p),
        ("err", _p),
        ("tlen", _p),
    ]


class HeadFwd(C.Structure):
    """Mirror of ``HeadFwd`` in csrc/mdn_head.hip (fused MDN head forward)."""
    _fields_ = [
        ("X", _p), ("ldx", _i64), ("N", _i64), ("Hd", _i),
        ("Wt", _p), ("bias", _p), ("tgt", _p), ("ldt", _i64),
        ("M", _i), ("NOUT", _i), ("NOUTP", _i), ("mode", _i), ("mask_pen", _i),
        ("F", _f), ("log_floor", _f), ("inv_n", _f),
        ("keep", _f), ("seed", _p), ("stream", _u32),
        ("dz", _p), ("part", _p), ("x_bf16", _i), ("ldz", _i64),
    ]


class HeadDx(C.Structure):
    _fields_ = [
        ("dz", _p), ("N", _i64), ("NOUTP", _i),
        ("Wb", _p), ("Hd", _i),
        ("scale", _p), ("keep", _f), ("seed", _p), ("stream", _u32),
        ("dX", _p), ("lddx", _i64), ("ldz", _i64),
    ]


class HeadDw(C.Structure):
    _fields_ = [
        ("X", _p), ("ldx", _i64), ("N", _i64), ("Hd", _i),
        ("dz", _p), ("NOUTP", _i),
        ("scale", _p), ("keep", _f), ("seed", _p), ("stream", _u32),
        ("slab", _p), ("rows_per", _i64), ("ldz", _i64), ("x_bf16", _i),
    ]


class DecLayer(C.Structure):
    """Mirror of ``DecLayer`` in csrc/decode_ref.hip (fused whole-sketch decoder)."""
    _fields_ = [
        ("WT", _p), ("bias", _p), ("h0", _p), ("c0", _p),
        ("hbuf", _p), ("hup", _p), ("hT", _p), ("cT", _p),
    ]


class DecArgs(C.Structure):
    _fields_ = [
        ("N", _i), ("B", _i), ("L", _i), ("H", _i), ("mtw", _i), ("nrb", _i), ("M", _i), ("nout", _i),
        ("noutp", _i), ("mode", _i), ("greedy", _i), ("fix_pen", _i), ("forced", _i), ("row0", _i),
        ("temp", _f), ("forget_bias", _f),
        ("ly", DecLayer * 2),
        ("Wx0", _p), ("WoT", _p), ("bo", _p),
        ("xin", _p), ("out", _p), ("done", _p), ("zout", _p),
        ("seed", _p), ("flags", _p), ("err", _p),
    ]


class GemmProblem(C.Structure):
    """Mirror of ``GemmProblem`` in csrc/skinny_gemm.hip."""
    _fields_ = [
        ("A", _p), ("lda", _i64),
        ("Bt", _p), ("ldb", _i64),
        ("C", _p), ("ldc", _i64), ("c_slab", _i64),
        ("M", _i), ("N", _i), ("K", _i), ("splits", _i),
    ]


class SgProb(C.Structure):
    """Mirror of ``SgProb`` in csrc/small_gemm.hip (one product of skr_small_gemm_group)."""
    _fields_ = [
        ("A", _p), ("sam", _i64), ("sak", _i64), ("a_batch", _i64),
        ("B", _p), ("sbk", _i64), ("sbn", _i64), ("b_batch", _i64),
        ("C", _p), ("ldc", _i64), ("c_batch", _i64),
        ("bias", _p),
        ("M", _i), ("N", _i), ("K", _i), ("acc", _i), ("nbatch", _i),
        ("work", _p), ("work_elems", _i64),
    ]


class CsJob(C.Structure):
    """Mirror of ``CsJob`` in csrc/reduce.hip (one column reduction of skr_colsum_multi)."""
    _fields_ = [
        ("X", _p), ("Y", _p),
        ("R1", _i64), ("s1", _i64), ("R2", _i64), ("s2", _i64),
        ("C", _i), ("RS", _i), ("xbf", _i), ("ybf", _i),
        ("part_xy", _p), ("part_x", _p), ("out_xy", _p), ("out_x", _p),
    ]


class ChainSync(C.Structure):
    """Mirror of ``ChainSync`` in csrc/chain_step.hip (rotating arrival
    counters of a chained launch kind)."""
    _fields_ = [("counters", _p), ("n", _i), ("k", _i), ("err", _p)]


class ModDecode(C.Structure):
    """Mirror of ``ModDecode`` in csrc/hyper_mod.hip (decode-mode inputs of the
    HyperLSTM modulation kernel: the x-projection from the stroke)."""
    _fields_ = [
        ("xh_bf16", _i), ("x5", _p), ("w5", _p), ("ldw5", _i64), ("zp", _p), ("ldzp", _i64), ("probe", _i),
    ]


class DecodeSample(C.Structure):
    """Mirror of ``DecodeSample`` in csrc/decode_step.hip (the previous stroke's
    sampler folded into the decode-step hyper cell)."""
    _fields_ = [
        ("active", _i),
        ("zs", _p), ("ldz", _i64), ("nslab", _i), ("slab", _i64),
        ("bias", _p), ("nout", _i),
        ("M", _i), ("mode", _i), ("temp", _f), ("greedy", _i), ("fix_pen", _i),
        ("seed", _p), ("step", _u32), ("row0", _i),
        ("out_row", _p), ("ld_out", _i64),
        ("done", _p),
    ]


class HipLib:
    def __init__(self, lib: C.CDLL):
        self.lib = lib
        lib.skr_lstm_fwd_step.argtypes = [C.POINTER(LstmFwdArgs), _i, _i, _p]
        lib.skr_lstm_fwd_step.restype = _i
        lib.skr_lstm_bwd_step.argtypes = [C.POINTER(LstmBwdArgs), _i, _i, _p]
        lib.skr_lstm_bwd_step.restype = _i
        lib.skr_row_fwd_step.argtypes = [C.POINTER(LstmFwdArgs), _i, _p]
        lib.skr_row_fwd_step.restype = _i
        lib.skr_row_bwd_step.argtypes = [C.POINTER(LstmBwdArgs), _i, _p]
        lib.skr_row_bwd_step.restype = _i
        lib.skr_row_supported.argtypes = [_i]
        lib.skr_row_supported.restype = _i
        lib.skr_colsum2.argtypes = [_p, _i, _p, _i, _i64, _i64, _i64, _i64, _i, _i, _p, _p, _p, _p, _p]
        lib.skr_colsum2.restype = _i
        lib.skr_slab_sum2.argtypes = [_p, _i, _i64, _i64, _p, _i, _i64, _i64, _i, _i, _p, _p]
        lib.skr_slab_sum2.restype = _i
        lib.skr_small_gemm_batched.argtypes = [_p, _i64, _i64, _i64, _p, _i64, _i64, _i64, _p, _i64, _i64, _p, _i, _i,
                                               _i, _i, _i, _p, _i64, _p]
        lib.skr_small_gemm_batched.restype = _i
        lib.skr_small_gemm_splits.argtypes = [_i, _i, _i]
        lib.skr_small_gemm_splits.restype = _i
        lib.skr_small_gemm.argtypes = [_p, _i64, _i64, _p, _i64, _i64, _p, _i64, _p, _i, _i, _i, _i, _p, _i64, _p]
        lib.skr_small_gemm.restype = _i
        lib.skr_mdn_loss.argtypes = [_p, _i64, _p, _i64, _i64, _i, _i, _f, _i, _f, _p, _p, _p, _p]
        lib.skr_mdn_loss.restype = _i
        lib.skr_adam_step.argtypes = [_p, _p, _p, _p, _p, _p, _i64, _f, _f, _f, _i, _f, _i, _p]
        lib.skr_adam_step.restype = _i
        lib.skr_global_norm.argtypes = [_p, _i64, _p, _p, _p]
        lib.skr_global_norm.restype = _i
        for fn in (lib.skr_skinny_gemm_v2,):
            fn.argtypes = [_p, _i64, _i64, _p, _i64, _i64, _p, _i64, _i64, _i64, _i, _i, _i, _i, _i, _i, _p]
            fn.restype = _i
        lib.skr_skinny_gemm_f32.argtypes = [_p, _i64, _i64, _p, _i64, _i64, _p, _i64, _i64, _i64, _i, _i, _i, _i, _i,
                                             _p]
        lib.skr_skinny_gemm_f32.restype = _i
        lib.skr_mdn_sample.restype = _i
        lib.skr_mdn_sample_slabs.argtypes = [_p, _i64, _i, _i64, _p, _i, _i, _i, _f, _i, _i, _p, _u32, _i, _p, _i64,
                                             _p, _i64, _p, _p]
        lib.skr_mdn_sample_slabs.restype = _i
        lib.skr_inproj_fwd.argtypes = [_p, _p, _p, _p, _p, _i, _i, _i, _i, _p]
        lib.skr_inproj_fwd.restype = _i
        lib.skr_inproj_bwd.argtypes = [_p, _p, _p, _i, _p, _i, _i, _i, _i, _i, _p]
        lib.skr_inproj_bwd.restype = _i
        lib.skr_bproj_fwd.argtypes = [_p, _p, _p, _p, _i, _i, _i, _i, _i, _p]
        lib.skr_bproj_fwd.restype = _i
        lib.skr_bproj_bwd.argtypes = [_p, _p, _i, _i64, _p, _p, _i, _i, _i, _i, _p]
        lib.skr_bproj_bwd.restype = _i
        lib.skr_skew_ln_fwd.argtypes = [C.POINTER(LstmFwdArgs), _p, _p, C.POINTER(ChainSync), _p]
        lib.skr_skew_ln_fwd.restype = _i
        lib.skr_chain_ln_set_probe.argtypes = [_i]
        lib.skr_chain_ln_set_probe.restype = _i
        lib.skr_hyper_mod_set_probe.argtypes = [_i]
        lib.skr_hyper_mod_set_probe.restype = _i
        lib.skr_bproj_set_wide.argtypes = [_i]
        lib.skr_bproj_set_wide.restype = _i
        lib.skr_colsum.argtypes = [_p, _i, _p, _i, _i64, _i64, _i64, _i64, _i, _i, _p, _p, _p]
        lib.skr_colsum.restype = _i
        lib.skr_wgrad.argtypes = [_p, _i64, _i64, _p, _i64, _i64, _i64, _i, _i, _i, _i, _p, _p, _p, _p, _p]
        lib.skr_wgrad.restype = _i
        lib.skr_wgrad2.argtypes = [_p, _i64, _i64, _p, _i64, _i64, _i64, _i, _i, _i, _i, _p, _p, _p, _p, _i, _i, _p]
        lib.skr_wgrad2.restype = _i
        lib.skr_wgrad_set_variant.argtypes = [_i]
        lib.skr_wgrad_set_variant.restype = _i
        lib.skr_latent_mid.argtypes = [_p, _p, _p, _p, _u32, _i, _f, _p, _p, _p, _p, _p]
        lib.skr_latent_mid.restype = _i
        lib.skr_latent_mid_bwd.argtypes = [_p, _p, _p, _p, _f, _p, _p, _p, _p, _p, _i, _p, _p, _p]
        lib.skr_latent_mid_bwd.restype = _i
        lib.skr_tanh_split.argtypes = [_p, _i, _i, _i, C.POINTER(_i), C.POINTER(_p), _p]
        lib.skr_tanh_split.restype = _i
        lib.skr_tanh_split_bwd.argtypes = [_i, _i, _i, C.POINTER(_i), C.POINTER(_p), C.POINTER(_p), _p, _p]
        lib.skr_tanh_split_bwd.restype = _i
        lib.skr_hyper_fold.argtypes = [_p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p]
        lib.skr_hyper_fold.restype = _i
        lib.skr_occupancy_hog.argtypes = [_i, _i, _i, _i, _p, _p]
        lib.skr_occupancy_hog.restype = _i
        lib.skr_stream_create_cu_limited.argtypes = [_i, C.POINTER(C.c_void_p)]
        lib.skr_stream_create_cu_limited.restype = _i
        lib.skr_stream_destroy.argtypes = [_p]
        lib.skr_stream_destroy.restype = _i
        lib.skr_gru_fwd.argtypes = [C.POINTER(GruFwdArgs), _i, _p]
        lib.skr_gru_fwd.restype = _i
        lib.skr_gru_bwd.argtypes = [C.POINTER(GruBwdArgs), _i, _p]
        lib.skr_gru_bwd.restype = _i
        lib.skr_skinny_gemm_v2_bf16out.argtypes = [_p, _i64, _i64, _p, _i64, _i64, _p, _i64, _i64, _i, _i, _i, _i,
                                                    _p]
        lib.skr_skinny_gemm_v2_bf16out.restype = _i
        lib.skr_gemm_set_nstage.argtypes = [_i]
        lib.skr_gemm_set_nstage.restype = _i
        lib.skr_skinny_gemm_group.argtypes = [C.POINTER(GemmProblem), _i, _i, _p]
        lib.skr_skinny_gemm_group.restype = _i
        lib.skr_skinny_gemm_group_cellbwd.argtypes = [C.POINTER(GemmProblem), _i, C.POINTER(LstmBwdArgs), _p]
        lib.skr_skinny_gemm_group_cellbwd.restype = _i
        lib.skr_chain_bwd_main.argtypes = [C.POINTER(GemmProblem), _i, C.POINTER(LstmBwdArgs), C.POINTER(ChainSync), _p]
        lib.skr_cell_set_oversub.argtypes = [_i]
        lib.skr_cell_set_oversub.restype = _i
        lib.skr_hyper_mod_set_zgrid.argtypes = [_i]
        lib.skr_hyper_mod_set_zgrid.restype = _i
        lib.skr_gemm_set_ra.argtypes = [_i]
        lib.skr_gemm_set_ra.restype = _i
        lib.skr_chain_ln_fwd.argtypes = [C.POINTER(GemmProblem), _i, C.POINTER(LstmFwdArgs), C.POINTER(ChainSync), _p]
        lib.skr_chain_ln_fwd.restype = _i
        lib.skr_chain_ln_bwd.argtypes = [C.POINTER(GemmProblem), _i, C.POINTER(LstmBwdArgs), C.POINTER(ChainSync), _p]
        lib.skr_chain_ln_bwd.restype = _i
        lib.skr_chain_bwd_main.restype = _i
        lib.skr_chain_bwd_main3.argtypes = [C.POINTER(GemmProblem), _i, C.POINTER(GemmProblem), C.POINTER(LstmBwdArgs),
                                            C.POINTER(ChainSync), C.POINTER(ChainSync), _p]
        lib.skr_chain_bwd_main3.restype = _i
        lib.skr_mx8_quant_t.argtypes = [_p, _i64, _i, _i, _p, _p, _p]
        lib.skr_mx8_quant_t.restype = _i
        lib.skr_mx8_quant_rows.argtypes = [_p, _i64, _i, _i, _i, _p, _i64, _p, _p]
        lib.skr_mx8_quant_rows.restype = _i
        lib.skr_mx8_gemm.argtypes = [_p, _i64, _p, _p, _i64, _p, _p, _i64, _i, _i, _i, _p]
        lib.skr_mx8_gemm.restype = _i
        lib.skr_mx8_set_layout.argtypes = [_i]
        lib.skr_mx8_set_layout.restype = _i
        lib.skr_chain_set_poll.argtypes = [_i]
        lib.skr_chain_set_poll.restype = _i
        lib.skr_chain3_set_probe.argtypes = [_i]
        lib.skr_chain3_set_probe.restype = _i
        lib.skr_lstm_fused_fwd.argtypes = [C.POINTER(FusedFwdArgs), _p]
        lib.skr_lstm_fused_fwd.restype = _i
        lib.skr_lstm_fused_bwd.argtypes = [C.POINTER(FusedBwdArgs), _p]
        lib.skr_lstm_fused_bwd.restype = _i
        lib.skr_lstm_persist_fwd.argtypes = [C.POINTER(PFwdArgs), _p]
        lib.skr_lstm_persist_fwd.restype = _i
        lib.skr_lstm_persist_bwd.argtypes = [C.POINTER(PBwdArgs), _p]
        lib.skr_lstm_persist_bwd.restype = _i
        lib.skr_small_gemm_group.argtypes = [C.POINTER(SgProb), _i, _p]
        lib.skr_small_gemm_group.restype = _i
        lib.skr_colsum_multi.argtypes = [C.POINTER(CsJob), _i, _i, _p]
        lib.skr_colsum_multi.restype = _i
        lib.skr_persist_set_spin_limit.argtypes = [C.c_uint]
        lib.skr_persist_set_spin_limit.restype = _i
        lib.skr_mdn_head_fwd.argtypes = [C.POINTER(HeadFwd), _p, _p]
        lib.skr_mdn_head_fwd.restype = _i
        lib.skr_mdn_head_nblocks.argtypes = [_i64]
        lib.skr_mdn_head_nblocks.restype = _i
        lib.skr_mdn_head_dx.argtypes = [C.POINTER(HeadDx), _p]
        lib.skr_mdn_head_dx.restype = _i
        lib.skr_mdn_head_dw.argtypes = [C.POINTER(HeadDw), _i, _i, _p, _p, _p]
        lib.skr_mdn_head_dw.restype = _i
        lib.skr_hyper_mod_fwd.argtypes = [_p, _i64, _p, _p, _p, _p, _i64, _i, _p, _p, _p, _p, _i, _i, _i,
                                          C.POINTER(ModDecode), _p]
        lib.skr_hyper_mod_fwd.restype = _i
        lib.skr_hyper_mod_chain.argtypes = [_p, _i64, _p, _p, _p, _i, _p, _i64, _i, _p, _p, C.POINTER(LstmFwdArgs),
                                            C.POINTER(ChainSync), _p]
        lib.skr_hyper_mod_chain.restype = _i
        lib.skr_hyper_cell_mod.argtypes = [C.POINTER(LstmFwdArgs), _p, _p, _p, _i, _p, _i64, _i, _p, _p, _p, _p, _i,
                                           C.POINTER(ChainSync), _p]
        lib.skr_hyper_cell_mod.restype = _i
        lib.skr_cast_transpose_bf16.argtypes = [_p, _i64, _i64, _i, _i, _i, _p, _i64, _i64, _p, _i64, _i64, _p]
        lib.skr_cast_transpose_bf16.restype = _i
        lib.skr_hash_normal.argtypes = [_p, _u32, _u32, _p, _i64, _p]
        lib.skr_hash_normal.restype = _i
        lib.skr_decode_hyper_cell.argtypes = [C.POINTER(LstmFwdArgs), C.POINTER(DecodeSample), _p, _p, _i64, _p]
        lib.skr_decode_hyper_cell.restype = _i
        lib.skr_decode_ref.argtypes = [C.POINTER(DecArgs), _p]
        lib.skr_decode_ref.restype = _i
        for name, cls in (("skr_lstm_fwd_args_size", LstmFwdArgs), ("skr_lstm_bwd_args_size", LstmBwdArgs),
                          ("skr_gru_fwd_args_size", GruFwdArgs), ("skr_gru_bwd_args_size", GruBwdArgs),
                          ("skr_lstm_fused_fwd_args_size", FusedFwdArgs),
                          ("skr_lstm_fused_bwd_args_size", FusedBwdArgs),
                          ("skr_lstm_persist_fwd_args_size", PFwdArgs),
                          ("skr_lstm_persist_bwd_args_size", PBwdArgs),
                          ("skr_mdn_head_fwd_args_size", HeadFwd),
                          ("skr_mdn_head_dx_args_size", HeadDx),
                          ("skr_mdn_head_dw_args_size", HeadDw),
                          ("skr_decode_ref_args_size", DecArgs),
                          ("skr_gemm_problem_size", GemmProblem),
                          ("skr_decode_sample_size", DecodeSample),
                          ("skr_chain_sync_size", ChainSync),
                          ("skr_colsum_job_size", CsJob),
                          ("skr_small_gemm_prob_size", SgProb)):
            fn = getattr(lib, name)
            fn.restype = _i
            if fn() != C.sizeof(cls):
                raise RuntimeError("libskrnn_hip.so arg-struct layout mismatch: %s %d vs %d"
                                   % (cls.__name__, fn(), C.sizeof(cls)))


def bind(lib: C.CDLL) -> HipLib:
    return HipLib(lib)
