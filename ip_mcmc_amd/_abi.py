"""ctypes mirror of include/ipmc.h (the C-ABI of libipmc.so).

Only layout and constants live here; compute goes through ``_lib``.
"""
import ctypes as C

ABI_VERSION = 13

OK, ERR_INVALID, ERR_UNSUPPORTED, ERR_DEVICE = 0, 1, 2, 3
F32, F64 = 0, 1
MODEL_LINEAR, MODEL_LORENZ63, MODEL_LORENZ96, MODEL_BURGERS, MODEL_LORENZ96_2S = 0, 1, 2, 3, 4
ARITH_FMA, ARITH_REFERENCE = 0, 1
DT_FIXED, DT_CFL = 0, 1
PROPOSAL_PCN, PROPOSAL_RW = 0, 1

STATUS_NAMES = {
    OK: "IPMC_OK",
    ERR_INVALID: "IPMC_ERR_INVALID",
    ERR_UNSUPPORTED: "IPMC_ERR_UNSUPPORTED",
    ERR_DEVICE: "IPMC_ERR_DEVICE",
}


class IpmcModel(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("arith", C.c_int32),
        ("k", C.c_int32),
        ("q", C.c_int32),
        ("dim", C.c_int32),
        ("n_steps", C.c_int32),
        ("dt", C.c_double),
        ("x0", C.c_void_p),
        ("theta0", C.c_void_p),
        ("A", C.c_void_p),
        ("dt_mode", C.c_int32),
        ("n_windows", C.c_int32),
        ("win_lo", C.c_void_p),
        ("win_hi", C.c_void_p),
        ("dx", C.c_double),
        ("t_end", C.c_double),
        ("cfl", C.c_double),
        ("nu", C.c_double),
        ("meas_scale", C.c_double),
        ("meas_dx", C.c_double),
        ("max_iter", C.c_int32),
        ("reserved", C.c_int32),
        ("fast_per_slow", C.c_int32),
        ("moment_mode", C.c_int32),
        ("coupling_c", C.c_double),
    ]


class IpmcSweep(C.Structure):
    _fields_ = [
        ("dtype", C.c_int32),
        ("lanes_per_chain", C.c_int32),
        ("chains_per_lane", C.c_int32),
        ("spec_width", C.c_int32),
        ("n_chains", C.c_int64),
        ("chain_offset", C.c_int64),
        ("u", C.c_void_p),
        ("phi", C.c_void_p),
        ("accepts", C.c_void_p),
        ("calls", C.c_void_p),
        ("y", C.c_void_p),
        ("gamma_inv", C.c_void_p),
        ("prior_sqrt", C.c_void_p),
        ("box_lo", C.c_void_p),
        ("box_hi", C.c_void_p),
        ("box_off", C.c_void_p),
        ("beta", C.c_double),
        ("contraction", C.c_double),
        ("beta_schedule", C.c_void_p),
        ("proposal", C.c_int32),
        ("reserved1", C.c_int32),
        ("reg_scale", C.c_void_p),
        ("seed", C.c_uint64),
        ("step0", C.c_uint64),
        ("n_steps", C.c_int64),
        ("sample_out", C.c_void_p),
        ("sample_stride", C.c_int64),
        ("sum_u", C.c_void_p),
        ("sum_u2", C.c_void_p),
        ("prior_chol", C.c_void_p),
        ("sample_every", C.c_int64),
        ("sample_step_stride", C.c_int64),
        ("accepts_step0", C.c_uint64),
    ]


class IpmcPlan(C.Structure):
    _fields_ = [
        ("lanes_per_chain", C.c_int32),
        ("chains_per_lane", C.c_int32),
        ("spec_width", C.c_int32),
        ("reserved", C.c_int32),
    ]


# Exported symbols of libipmc.so and their ctypes signatures (include/ipmc.h).
SIGNATURES = {
    "ipmc_pcn_sweep": (C.c_int, [C.POINTER(IpmcModel), C.POINTER(IpmcSweep), C.c_void_p]),
    "ipmc_pcn_run": (C.c_int, [C.POINTER(IpmcModel), C.POINTER(IpmcSweep), C.c_int64, C.c_int64, C.c_int64,
                               C.c_void_p]),
    "ipmc_init_phi": (C.c_int, [C.POINTER(IpmcModel), C.POINTER(IpmcSweep), C.c_void_p]),
    "ipmc_potential": (
        C.c_int,
        [C.POINTER(IpmcModel), C.c_int32, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    ),
    "ipmc_forward": (C.c_int, [C.POINTER(IpmcModel), C.c_int32, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]),
    "ipmc_normal": (
        C.c_int,
        [C.c_uint64, C.c_int64, C.c_int64, C.c_uint64, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p],
    ),
    "ipmc_uniform": (C.c_int, [C.c_uint64, C.c_int64, C.c_int64, C.c_uint64, C.c_void_p, C.c_void_p]),
    "ipmc_pcn_draws": (
        C.c_int,
        [C.c_uint64, C.c_int64, C.c_int64, C.c_uint64, C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
         C.c_void_p, C.c_void_p, C.c_void_p],
    ),
    "ipmc_copy_rows_d2h": (
        C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p]),
    "ipmc_autocorr": (
        C.c_int,
        [C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p],
    ),
    "ipmc_burn_in": (
        C.c_int,
        [C.c_void_p, C.c_int32, C.c_int64, C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int32,
         C.c_double, C.c_void_p, C.c_void_p, C.c_void_p],
    ),
    "ipmc_ordered_sum": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_void_p,
                                   C.c_void_p]),
    "ipmc_block_sums": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_void_p,
                                  C.c_void_p]),
    "ipmc_auto_lanes": (C.c_int, [C.POINTER(IpmcModel), C.c_int32, C.c_int64]),
    "ipmc_auto_layout": (C.c_int, [C.POINTER(IpmcModel), C.c_int32, C.c_int64]),
    "ipmc_plan_sweep": (C.c_int, [C.POINTER(IpmcModel), C.POINTER(IpmcSweep), C.POINTER(IpmcPlan)]),
    "ipmc_last_error": (C.c_char_p, []),
    "ipmc_abi_version": (C.c_int, []),
}
