"""ctypes signatures of the C ABI exported by ``libbiscotti_hip.so``."""
from __future__ import annotations

import ctypes as C

P = C.c_void_p
I = C.c_int
L = C.c_longlong
D = C.c_double
F = C.c_float
U64 = C.c_uint64

SIGNATURES = {
    # msm.hip
    "bsc_fp_op": [P, P, P, I, I, P],
    "bsc_point_op": [P, P, P, P, I, I, P],
    "bsc_witness_bases": [P, I, I, I, P, P],
    "bsc_fb_table": [P, I, I, I, I, I, I, L, L, L, P, P, P],
    "bsc_shares_msm": [P, I, P, I, P, P, I, I, I, I, I, P, P, I, P, P, P],
    "bsc_alive_compact": [P, I, P, P],
    "bsc_set_alive": [P, P, I, P, P],
    "bsc_sum_rows": [P, I, P, I, P, I, P, P],
    "bsc_segment_sum": [P, I, I, I, I, P, P],
    "bsc_sum_rows2": [P, I, P, I, P, I, P, P, P],
    "bsc_sum_rows2_pos": [P, I, P, I, P, I, P, P, P],
    "bsc_round_csum_early": [P, P, P, P, I, P, P, P],
    "bsc_round_spec_msm2": [P, I, P, P, P, I, P, I, I, P, P, P, P, P, P],
    "bsc_round_spec_topup": [P, I, P, I, P, I, P, P, I, I, P, P, P, P, P],
    "bsc_round_set_spec_ring": [P, P, I, I],
    "bsc_round_set_witness_stream": [P, P],
    "bsc_wave_prio": [I],
    "bsc_round_prestep": [P, P, P, P, P, P, P, P, I, I, I, I, U64, I, F, D, I, P, P, P, P, P, P, P, P,
                          I, P, I, L, I, P, P, P, P, P, P, P, I, P],
    "bsc_commit_rows": [P, I, P, I, P, I, I, P, P, P],
    "bsc_stream_create_cumask": [I, P],
    "bsc_stream_destroy": [P],
    "bsc_h2d_async": [P, P, L, P],
    "bsc_d2h_async": [P, P, L, P],
    "bsc_marshal": [P, I, P, P],
    "bsc_to_affine": [P, I, P, P],
    "bsc_chunk_check": [P, I, I, P, I, I, P, I, I, P, P],
    # vrf.hip
    "bsc_vrf_prove": [P, P, P, P, I, I, P, P, P, P, P],
    "bsc_vrf_prove_p": [P, P, P, P, I, I, P, P, P, P, I, P],
    # kzg.hip
    "bsc_kzg_blocks": [I, I],
    "bsc_kzg_rlc": [P, P, P, P, I, I, I, P, I, I, U64, P, P, P],
    # ml.hip
    "bsc_softmax_step": [P, P, P, P, P, P, I, I, I, I, U64, I, F, D, P, P, P, I, P],
    "bsc_logreg_step": [P, P, P, P, P, P, I, I, I, U64, P, D, D, P, D, P, P, P],
    "bsc_dp_noise": [P, I, I, P, I, P, U64, I, P, P],
    "bsc_krum": [P, I, I, I, P, P, P, P, I, I, P],
    "bsc_krum_committee": [P, I, I, I, P, I, I, I, I, I, P, I, P, P, P, P, P, P, P, P],
    "bsc_gram_stacked": [P, I, P, I, L, I, I, P, P, P, P, P],
    "bsc_gram_stacked_range": [P, I, P, I, L, I, I, I, I, P, P, P, P, P],
    "bsc_krum_committee_noise": [P, I, I, P, P, I, P, I, I, I, I, I, P, I, P, P, P, P, P],
    "bsc_krum_committee_noise2": [P, I, I, P, P, I, P, I, I, I, I, I, P, I, P, P, P, P, P, P, I, P, P],
    "bsc_krum_committee_noise_ka": [P, I, I, P, P, I, P, I, I, I, I, I, P, I, P, P, P, P, P, P, I, P, P],
    "bsc_eval_error": [P, P, I, I, I, P, I, I, P, P],
    "bsc_eval_error_rb": [P, P, I, I, I, P, I, I, P, P, P],
    "bsc_eval_error_t_rb": [P, P, I, I, I, I, P, I, P, P, P],
    "bsc_noise_table": [I, I, U64, P, P],
    "bsc_dp_noise_tbl": [P, I, I, P, I, P, P, I, P, P, P],
    "bsc_recover": [P, I, I, P, I, I, P, D, P, P, P, P],
    "bsc_add_rows": [P, I, P, I, P, P, P],
    "bsc_sum_rows_i64": [P, I, L, P, I, P, P, P],
    "bsc_lsh_codes": [P, P, I, I, P, I, I, P, P],
    "bsc_lsh_count": [P, I, P, I, P, I, D, P, P],
    "bsc_weighted_rows": [P, I, I, P, P, P],
    "bsc_recover_w": [P, I, I, I, P, P, P, I, P, P, I, I, U64, U64, I, P, D, P, P, P, P, P],
    "bsc_recover_w_strided": [P, I, L, I, I, P, P, P, I, P, P, I, I, U64, U64, I, P, D, P, P, P, P, P],
    # round.hip
    "bsc_round_create": [P, P, P, P, I, I, I, I, I, D],
    "bsc_round_destroy": [P],
    "bsc_round_secagg": [P, P, I, P, P, P, P, I, P, P, I, P, P, I, U64, U64, P, P, P, P, P, P, P, P, P, I],
    "bsc_round_audit": [P, P, P, P, P],
    "bsc_round_wait": [P, I],
    "bsc_round_audit_slot": [P],
    "bsc_set_host_spin_ns": [L],
    "bsc_round_row_bytes": [I, I],
    "bsc_round_partials": [P, P, I, P, P, P, P, I, P, P, L, I],
    "bsc_round_combine": [P, P, I, L, P, P, I, P, P, I, U64, U64, P, P, P, P, P, P, P, P, P, I],
    "bsc_round_bind_outputs": [P, P, I, P, P, P, P, P, P, P],
    "bsc_round_add_layout": [P, P, P, I, P, P, I, P, P, I, U64, U64, P, P],
    "bsc_round_bind_task": [P, P, P, P, P, P, P, I, I, I, I, U64, F, D, I, P, P, P, I, I, P],
    "bsc_round_add_pre_slot": [P, P, P, P, P, P, P, P, P, P, P, P, P],
    "bsc_round_pick_W": [P, P],
    "bsc_round_prestep_slot": [P, P, I, I],
    "bsc_round_set_nn_table": [P, P],
    "bsc_round_after_select": [P, P, P, P, I, P, P, P, P, I, P, I, P, I, I, I, I, P],
    "bsc_round_select_partials": [P, P, P, P, I, P, P, P, P, I, P, I, P, L, I],
    "bsc_round_after_gather": [P, P, I, L, I, P, P, I, I, I, P],
    "bsc_ring_pick": [P, I, P, P, P],
    "bsc_rccl_load": [C.c_char_p],
    "bsc_set_side_prio": [I],
    "bsc_sum_cols_serial": [P, I, I, P, I, P, P, P],
    "bsc_set_witness_tree": [I],
    "bsc_rccl_unique_id": [P],
    "bsc_round_comm_init": [P, P, I, I, P, I, D],
    "bsc_round_bind_multi": [P, P, P, L, P, I, P, P, P, I, I, I, P, P, L],
    "bsc_round_agg_multi": [P, P, P, P, I, P, P, P, P, I, P, I, L, P, I, I, I, I, P],
    "bsc_round_vg_exchange": [P, I, L, L, L, P, I, I, P, P, P, I, I, I, I, P, I, P, P, P, P, P],
    # gather.hip
    "bsc_vg_limits": [P],
    "bsc_vg_pack": [P, L, L, L, P, I, I, P, P, P, I, P],
    "bsc_vg_unpack": [P, L, I, I, L, L, L, I, I, I, I, P, I, P, P, P, P, P],
}


RESTYPES = {"bsc_stream_create_cumask": C.c_void_p, "bsc_round_create": C.c_void_p, "bsc_round_destroy": None,
            "bsc_set_host_spin_ns": None}


def declare(lib) -> None:
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = RESTYPES.get(name, C.c_int)
