"""ctypes binding of the C ABI in include/lf.h (liblatticeum_amd.so, built in-tree).

This module only loads the shared library and declares signatures; there is no
Python compute fallback. Loading fails loudly if the library is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = PKG / "liblatticeum_amd.so"

SZ, I, U64, VP = C.c_size_t, C.c_int, C.c_uint64, C.c_void_p
U64P = C.POINTER(C.c_uint64)
U8P = C.POINTER(C.c_uint8)


class LfParams(C.Structure):
    _fields_ = [("d", I), ("B", U64), ("L", I), ("b_small", U64), ("K", I)]


class LfFoldStepBufs(C.Structure):
    _fields_ = [
        ("w_ccs", VP), ("acc_cm", VP), ("acc_f_coeff", VP), ("rho", VP),
        ("f_coeff", VP), ("f", VP), ("cm", VP),
        ("fk_coeff", VP * 2), ("fk", VP * 2), ("wk", VP * 2), ("y", VP * 2),
        ("f0", VP), ("f0_coeff", VP), ("w_ccs0", VP), ("cm0", VP), ("planes", VP * 2),
    ]


class LfRingSlice(C.Structure):
    _fields_ = [("elems", VP), ("n", SZ)]


class LfLcccs(C.Structure):
    _fields_ = [("d", I), ("r", LfRingSlice), ("v", LfRingSlice), ("cm", LfRingSlice), ("u", LfRingSlice),
                ("x_w", LfRingSlice), ("h", VP)]


class LfDecompositionProof(C.Structure):
    _fields_ = [("u_s", VP), ("v_s", VP), ("x_s", VP), ("y_s", VP), ("n_u", SZ), ("n_v", SZ), ("n_x", SZ),
                ("n_y", SZ)]


class LfLfproof(C.Structure):
    _fields_ = [("d", I), ("lin_sumcheck", VP), ("lin_rounds", SZ), ("lin_evals", SZ), ("lin_v", LfRingSlice),
                ("lin_u", LfRingSlice), ("dec", LfDecompositionProof * 2), ("fold_sumcheck", VP),
                ("fold_rounds", SZ), ("fold_evals", SZ), ("theta_s", VP), ("eta_s", VP), ("n_theta", SZ),
                ("n_eta", SZ)]


class LfWitness(C.Structure):
    _fields_ = [("w_ccs", VP), ("f", VP), ("f_coeff", VP)]


class LfLcccsMut(C.Structure):
    _fields_ = [("r", VP), ("v", VP), ("cm", VP), ("u", VP), ("x_w", VP), ("h", VP)]


class LfLfproofMut(C.Structure):
    _fields_ = [("lin_sumcheck", VP), ("lin_v", VP), ("lin_u", VP), ("u_s", VP * 2), ("v_s", VP * 2),
                ("x_s", VP * 2), ("y_s", VP * 2), ("fold_sumcheck", VP), ("theta_s", VP), ("eta_s", VP)]


REPLAY_FIELDS = ("lin_beta", "lin_claimed_sums", "lin_subterms", "lin_point", "lin_expected", "lin_inner",
                 "lin_products", "lin_eq_xy", "lin_eq_factors", "lin_eq_sub", "alpha", "beta", "zeta", "mu",
                 "claim_g1_h1", "claim_g1_h2", "claim_g1_terms", "claim_g1", "claim_g3_h", "claim_g3_terms",
                 "claim_g3", "fold_claimed_sums", "fold_subterms", "fold_point", "fold_expected", "should_equal_s",
                 "rho", "final_cm", "final_u", "final_x")


class LfReplayVars(C.Structure):
    _fields_ = [(k, VP) for k in REPLAY_FIELDS]


class LfCcsDesc(C.Structure):
    _fields_ = [("t", I), ("m", SZ), ("l", SZ), ("degree", I), ("q", I), ("c", VP), ("S_off", VP), ("S_idx", VP)]


class LfComb(C.Structure):
    _fields_ = [("kind", I), ("nk", I), ("tau", I), ("bsmall", I), ("mu", VP), ("q", I), ("c", VP),
                ("S_off", VP), ("S_idx", VP)]


# every function exported by include/lf.h: name -> (restype, argtypes)
SIGNATURES = {
    "lf_goldilocks_dp": (LfParams, [I]),
    "lf_ctx_create": (I, [I, C.POINTER(VP)]),
    "lf_ctx_destroy": (None, [VP]),
    "lf_status_string": (C.c_char_p, [I]),
    "lf_ctx_last_error": (C.c_char_p, [VP]),
    "lf_ctx_set_error": (None, [VP, C.c_char_p]),
    "lf_ctx_set_stream": (I, [VP, VP]),
    "lf_ctx_get_stream": (VP, [VP]),
    "lf_stream_create_cu_mask": (I, [I, VP, I, VP]),
    "lf_stream_destroy": (I, [VP]),
    "lf_ctx_set_cu_count": (I, [VP, I]),
    "lf_ctx_set_contract_stream": (I, [VP, VP]),
    "lf_ctx_sync": (I, [VP]),
    "lf_ctx_reserve": (I, [VP, SZ, SZ, I, I]),
    "lf_ctx_kernel_timing": (I, [VP, I]),
    "lf_ctx_kernel_stats": (I, [VP, I, C.POINTER(C.c_double), C.POINTER(C.c_long)]),
    "lf_ctx_phase_stats": (I, [VP, I, C.POINTER(C.c_double), C.POINTER(C.c_long)]),
    "lf_crt": (I, [VP, VP, SZ, I, I]),
    "lf_icrt": (I, [VP, VP, SZ, I, I]),
    "lf_ring_mul": (I, [VP, VP, VP, VP, SZ, I, I]),
    "lf_ajtai_create": (I, [VP, VP, SZ, SZ, I, I, C.POINTER(VP)]),
    "lf_ajtai_create_device": (I, [VP, VP, SZ, SZ, I, C.POINTER(VP)]),
    "lf_ajtai_destroy": (None, [VP]),
    "lf_ajtai_kappa": (SZ, [VP]),
    "lf_ajtai_width": (SZ, [VP]),
    "lf_ajtai_d": (I, [VP]),
    "lf_ajtai_layout": (I, [VP]),
    "lf_ajtai_commit": (I, [VP, VP, VP, SZ, VP, I]),
    "lf_witness_from_w_ccs": (I, [VP, C.POINTER(LfParams), VP, SZ, VP, VP, I]),
    "lf_witness_from_f": (I, [VP, C.POINTER(LfParams), VP, SZ, VP, VP, I]),
    "lf_decompose_witness": (I, [VP, C.POINTER(LfParams), VP, SZ, VP, VP, VP, I]),
    "lf_commit": (I, [VP, VP, C.POINTER(LfParams), VP, SZ, SZ, VP, VP, VP, I]),
    "lf_fold_hot": (I, [VP, VP, C.POINTER(LfParams), VP, VP, VP, VP, SZ, VP, VP, VP, VP, VP, VP, I]),
    "lf_short_challenge": (I, [VP, SZ, I, VP]),
    "lf_poseidon2_permute": (I, [VP, VP, SZ]),
    "lf_dev_crt": (I, [VP, VP, SZ, I]),
    "lf_dev_icrt": (I, [VP, VP, SZ, I]),
    "lf_dev_ring_mul": (I, [VP, VP, VP, VP, SZ, I]),
    "lf_dev_to_montgomery": (I, [VP, VP, SZ]),
    "lf_dev_from_montgomery": (I, [VP, VP, SZ]),
    "lf_dev_witness_from_w_ccs": (I, [VP, C.POINTER(LfParams), VP, SZ, VP, VP]),
    "lf_dev_witness_from_f": (I, [VP, C.POINTER(LfParams), VP, SZ, VP, VP]),
    "lf_dev_decompose_witness": (I, [VP, C.POINTER(LfParams), VP, SZ, VP, VP, VP]),
    "lf_dev_ajtai_commit": (I, [VP, VP, C.POINTER(VP), I, VP]),
    "lf_dev_commit_y0": (I, [VP, C.POINTER(LfParams), VP, VP, SZ]),
    "lf_dev_fold": (I, [VP, I, VP, C.POINTER(VP), I, SZ, VP]),
    "lf_dev_fold_step": (I, [VP, VP, C.POINTER(LfParams), SZ, C.POINTER(LfFoldStepBufs)]),
    "lf_dev_fold_step_batch": (I, [VP, I, VP, C.POINTER(LfParams), SZ, VP]),
    "lf_dev_poseidon2_permute": (I, [VP, VP, SZ]),
    "lf_dev_poseidon2_permute_rounds": (I, [VP, VP, SZ, I]),
    "lf_dev_fill_uniform": (I, [VP, VP, SZ, U64]),
    "lf_dev_modp_sum": (I, [VP, VP, I, SZ, VP]),
    "lf_dev_limb_split": (I, [VP, VP, SZ, VP, VP]),
    "lf_dev_limb_join": (I, [VP, VP, VP, SZ, VP]),
    "lf_transcript_new": (VP, []),
    "lf_transcript_free": (None, [VP]),
    "lf_transcript_observe": (None, [VP, U64]),
    "lf_transcript_sample": (U64, [VP]),
    "lf_transcript_absorb_ring": (None, [VP, VP, SZ, I, I]),
    "lf_transcript_get_challenge": (None, [VP, VP]),
    "lf_transcript_squeeze_bytes": (None, [VP, VP, SZ]),
    "lf_transcript_get_short_challenges": (I, [VP, I, SZ, VP]),
    "lf_hash_iter": (None, [VP, SZ, VP]),
    "lf_hash_iter_nperm": (SZ, [SZ]),
    "lf_hash_iter_states": (I, [VP, SZ, VP, VP, SZ]),
    "lf_acc_comm": (I, [C.POINTER(LfLcccs), I, VP]),
    "lf_ivc_step_comm": (I, [U64, VP, VP, VP, VP, VP]),
    "lf_state_i_comm": (I, [VP, U64, VP, VP, VP, VP]),
    "lf_vm_regs_comm": (I, [VP, SZ, VP]),
    "lf_vm_mem_ops_vec_comm": (I, [VP, U64, C.c_uint32, C.c_uint32, VP]),
    "lf_witness_split_w": (SZ, []),
    "lf_dev_poseidon2_w8_permute": (I, [VP, VP, SZ]),
    "lf_dev_merkle_tree": (I, [VP, VP, SZ, SZ, VP]),
    "lf_merkle_open": (I, [VP, VP, SZ, SZ, VP]),
    "lf_merkle_nodes_len": (SZ, [SZ]),
    "lf_dev_hash_w8_rows": (I, [VP, VP, SZ, SZ, VP]),
    "lf_vm_code_comm": (I, [VP, VP, SZ, VP]),
    "lf_hash_w8": (None, [VP, SZ, VP]),
    "lf_vm_mem_comm": (I, [VP, SZ, VP]),
    "lf_lcccs_serialize": (I, [C.POINTER(LfLcccs), I, VP, SZ, C.POINTER(SZ)]),
    "lf_lcccs_deserialize": (I, [VP, SZ, I, I, VP, SZ, C.POINTER(LfLcccs)]),
    "lf_lfproof_serialize": (I, [C.POINTER(LfLfproof), I, VP, SZ, C.POINTER(SZ)]),
    "lf_dev_eq_table": (I, [VP, I, VP, I, VP]),
    "lf_dev_get_fhat": (I, [VP, I, VP, SZ, I, VP]),
    "lf_dev_expand_planes": (I, [VP, C.POINTER(LfParams), VP, SZ, VP, VP]),
    "lf_ccs_create": (I, [VP, I, I, SZ, SZ, VP, VP, VP, I, C.POINTER(VP)]),
    "lf_ccs_destroy": (None, [VP]),
    "lf_ccs_set_structure": (I, [VP, VP, SZ, I, I, VP, VP, VP, I]),
    "lf_ccs_shape": (I, [VP, C.POINTER(I), C.POINTER(SZ), C.POINTER(SZ), C.POINTER(SZ), C.POINTER(I), C.POINTER(I)]),
    "lf_ccs_get_structure": (I, [VP, VP, VP, VP]),
    "lf_ccs_c_device": (VP, [VP]),
    "lf_ccs_row_live": (I, [VP, I, VP]),
    "lf_ccs_is_scalar": (I, [VP]),
    "lf_prover_create": (I, [VP, VP, C.POINTER(LfParams), VP, C.POINTER(VP)]),
    "lf_prover_destroy": (None, [VP]),
    "lf_prover_last_error": (C.c_char_p, [VP]),
    "lf_prover_timing": (I, [VP, I, VP]),
    "lf_fold_prove": (I, [VP, C.POINTER(LfLcccs), C.POINTER(LfWitness), VP, VP, C.POINTER(LfWitness),
                          C.POINTER(LfLcccsMut), C.POINTER(LfWitness), C.POINTER(LfLfproofMut), I]),
    "lf_linearize": (I, [VP, VP, VP, C.POINTER(LfWitness), C.POINTER(LfLcccsMut), VP, I]),
    "lf_dev_decompose_commit": (I, [VP, VP, C.POINTER(LfParams), SZ, C.POINTER(LfFoldStepBufs)]),
    "lf_dev_fold_combine": (I, [VP, VP, C.POINTER(LfParams), SZ, C.POINTER(LfFoldStepBufs)]),
    "lf_dev_fhat_evaluate": (I, [VP, I, VP, SZ, SZ, I, I, VP, VP]),
    "lf_dev_mle_lincomb": (I, [VP, I, VP, SZ, I, I, VP, VP]),
    "lf_ctx_device": (I, [VP]),
    "lf_fold_replay": (I, [C.POINTER(LfCcsDesc), C.POINTER(LfParams), C.POINTER(LfLcccs), VP, VP,
                           C.POINTER(LfLfproofMut), C.POINTER(LfReplayVars), I]),
    "lf_fold_verify": (I, [C.POINTER(LfCcsDesc), C.POINTER(LfParams), C.POINTER(LfLcccs), VP, VP,
                           C.POINTER(LfLfproofMut), C.POINTER(LfLcccsMut), C.POINTER(I), I]),
    "lf_fold_replay_samples": (I, [C.POINTER(LfCcsDesc), C.POINTER(LfParams), C.POINTER(LfLcccs), VP, VP,
                                   C.POINTER(LfLfproofMut), VP, SZ, C.POINTER(LfReplayVars), I]),
    "lf_prover_samples": (SZ, [VP, VP, SZ]),
    "lf_fold_prove_vars": (I, [VP, C.POINTER(LfLcccs), C.POINTER(LfWitness), VP, VP, C.POINTER(LfWitness),
                               C.POINTER(LfLcccsMut), C.POINTER(LfWitness), C.POINTER(LfLfproofMut),
                               C.POINTER(LfReplayVars), I]),
    "lf_transcript_record": (None, [VP]),
    "lf_transcript_samples": (SZ, [VP, VP, SZ]),
    "lf_transcript_new_playback": (VP, [VP, SZ]),
    "lf_transcript_playback_status": (I, [VP]),
    "lf_dev_mz_mles": (I, [VP, VP, VP, I, I, VP]),
    "lf_dev_mz_mles_sel": (I, [VP, VP, VP, VP, I, I, VP]),
    "lf_dev_mz_challenged": (I, [VP, VP, VP, VP, I, I, VP]),
    "lf_dev_mz_challenged_pair": (I, [VP, VP, VP, VP, VP, VP, I, I, VP, VP]),
    "lf_dev_mz_evaluate": (I, [VP, VP, VP, I, I, VP, VP]),
    "lf_ccs_weights_len": (SZ, [VP]),
    "lf_dev_mz_weights": (I, [VP, VP, I, VP, VP]),
    "lf_dev_mz_dots": (I, [VP, VP, VP, VP, I, VP]),
    "lf_dev_fhat_evaluate_eq": (I, [VP, I, VP, SZ, SZ, I, I, VP, VP]),
    "lf_dev_mle_fix_first": (I, [VP, I, VP, SZ, I, I, VP, VP, SZ]),
    "lf_dev_mle_evaluate": (I, [VP, I, VP, I, I, VP, VP]),
    "lf_dev_mle_evaluate_eq": (I, [VP, I, VP, I, I, VP, VP]),
    "lf_dev_sumcheck_round": (I, [VP, C.POINTER(LfComb), VP, SZ, I, I, I, I, VP]),
    "lf_sumcheck_prove": (I, [VP, VP, C.POINTER(LfComb), VP, I, I, I, I, VP, VP]),
    "lf_sumcheck_prove_ptrs": (I, [VP, VP, C.POINTER(LfComb), VP, I, I, I, I, VP, VP, VP]),
    "lf_sumcheck_prove_lin": (I, [VP, VP, C.POINTER(LfComb), VP, I, I, I, I, VP, VP, VP, VP, VP]),
    "lf_sumcheck_prove_lin_sparse": (I, [VP, VP, C.POINTER(LfComb), VP, I, I, I, I, VP, VP, VP, VP, VP, VP, VP]),
    "lf_sumcheck_prove_fold_digits": (I, [VP, VP, C.POINTER(LfComb), VP, VP, VP, I, SZ, SZ, I, I, VP, VP, VP]),
    "lf_fold_lcccs": (I, [VP, I, I, VP, VP, VP, SZ, VP, SZ, VP, VP, VP, VP, I]),
    "lf_dev_fold_lcccs": (I, [VP, I, I, VP, VP, VP, SZ, VP, SZ, VP, VP, VP, VP]),
    "lf_compute_x_s": (I, [VP, C.POINTER(LfParams), VP, SZ, VP, I]),
    "lf_dev_compute_x_s": (I, [VP, C.POINTER(LfParams), VP, SZ, VP]),
    "lf_fold_step_partial_len": (SZ, [VP, C.POINTER(LfParams)]),
    "lf_dev_fold_step_partial": (I, [VP, VP, C.POINTER(LfParams), SZ, C.POINTER(LfFoldStepBufs), VP]),
    "lf_dev_fold_step_finish": (I, [VP, VP, C.POINTER(LfParams), SZ, C.POINTER(LfFoldStepBufs), VP]),
    "lf_dev_fold_step_sharded": (I, [VP, VP, C.POINTER(LfParams), SZ, C.POINTER(LfFoldStepBufs), VP]),
    "lf_comm_unique_id": (I, [VP, SZ]),
    "lf_comm_init": (I, [VP, I, I, VP, SZ, C.POINTER(VP)]),
    "lf_comm_wrap": (I, [VP, VP, C.POINTER(VP)]),
    "lf_comm_destroy": (None, [VP]),
    "lf_comm_size": (I, [VP]),
    "lf_comm_rank": (I, [VP]),
    "lf_comm_allreduce_modp": (I, [VP, VP, VP, SZ]),
    "lf_fold_reduce_allranks": (I, [VP, VP, VP, SZ, VP, SZ]),
}

_lib = None


def load() -> C.CDLL:
    """Load liblatticeum_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch bundles libamdhip64.so.7 /
    # libhsa-runtime64.so.1 (same SONAMEs as /opt/rocm). Importing torch first
    # makes the dynamic linker bind this library to torch's already-loaded
    # runtime, so device pointers, streams and events are shared with torch
    # (which provides allocation and RCCL plumbing) instead of two HSA runtimes.
    try:
        import torch  # noqa: F401
    except ImportError:  # plain C-ABI use without torch binds /opt/rocm's runtime
        pass
    path = Path(os.environ.get("LATTICEUM_AMD_LIB", LIB_PATH))
    if not path.exists():
        raise ImportError(
            f"latticeum_amd: native library {path} not found -- build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = C.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
