"""halo2_svd041_amd — MI355X-native witness engine for the SVD-verify path of
neilcouture/halo2-svd041 (ZkMatrix / ZkVector / check_svd_phase0/1).

The compute path is the HIP library libsvdw.so (gfx950 kernels behind the C
ABI of include/svdw.h); this package is the host-side mirror of the
reference API over that ABI. There is no CPU fallback.
"""
from .zk import (  # noqa: F401
    P_MOD, Context, SvdConfigPy, SvdPayload, SvdwError, ZkMatrix, ZkVector, check_mat_diff,
    check_mat_entries_bounded, check_mat_id, check_svd_phase0, check_svd_phase1, err_calc,
    field_mat_vec_mul, honest_prover_mat_mul, int_to_words, mat_times_diag_mat, plan_svd,
    parse_svd_input, parse_svd_input_device, svd_witness, verify_mul_witness, words_to_int)

__version__ = "0.1.0"
