"""ctypes binding of libfiode.so (include/fiode.h).

The product path has no fallback: if the HIP library is missing or fails to load, importing
anything that needs it raises ``FiodeLibraryError`` immediately.
"""
from __future__ import annotations

import ctypes as ct
import os
import pathlib

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = pathlib.Path(os.environ.get("FIODE_LIB", _HERE / "libfiode.so"))

FIODE_SAMPLER_GIVEN, FIODE_SAMPLER_COMPOSITE, FIODE_SAMPLER_DECISION_BOUNDARY, FIODE_SAMPLER_TRAJECTORY = 0, 1, 2, 3
FIODE_DROPOUT_OFF, FIODE_DROPOUT_GIVEN, FIODE_DROPOUT_PHILOX = 0, 1, 2

class FiodeLibraryError(RuntimeError):
    pass


class FiodeError(RuntimeError):
    pass


_fp = ct.POINTER(ct.c_float)
_vp = ct.c_void_p


class DynWeights(ct.Structure):
    _fields_ = [(n, ct.c_void_p) for n in ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")]


class DynConfig(ct.Structure):
    _fields_ = [("n_hidden", ct.c_int32), ("mlp_size", ct.c_int32), ("x_dim", ct.c_int32),
                ("alpha_1", ct.c_float), ("alpha_2", ct.c_float), ("sigma_1", ct.c_float),
                ("scale_nominal", ct.c_int32), ("dropout", ct.c_float), ("qp_max_iter", ct.c_int32),
                ("qp_tol", ct.c_float)]


class LyapConfig(ct.Structure):
    _fields_ = [("batch", ct.c_int32), ("sample_size", ct.c_int32), ("n_uniform", ct.c_int32),
                ("sampler", ct.c_int32), ("dropout_mode", ct.c_int32), ("kappa", ct.c_float),
                ("seed", ct.c_uint64), ("offset", ct.c_uint64)]


class LyapIO(ct.Structure):
    _fields_ = [(n, ct.c_void_p) for n in ("x_feat", "y", "h", "masks", "scalars", "h_out", "V", "Vdot",
                                           "f", "f_log", "qp_lower", "qp_nominal", "g_ftilde", "events")] + \
        [("n_events", ct.c_int32), ("offset_dev", ct.c_void_p), ("exp_draws", ct.c_void_p),
         ("exp_draws_out", ct.c_void_p), ("keep_words_out", ct.c_void_p), ("kappa_dev", ct.c_void_p)]


LYAP_KERNELS = ("k_static_proj", "k_lyap_prep", "k_lyap_fwd", "k_lyap_bwd", "k_lyap_reduce", "k_lyap_static_grads")


class LyapGrads(ct.Structure):
    _fields_ = [(n, ct.c_void_p) for n in ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3", "x_feat")]


FIODE_ODE_RK4, FIODE_ODE_DOPRI5 = 0, 1
FIODE_DTYPE_F32, FIODE_DTYPE_C64 = 0, 1
FIODE_INV_MAX_N = 128
FIODE_ODE_MAX_BATCH = 4096          # fiode_odetrain_*
FIODE_ODETRAIN_MAX_ATTEMPTS = 1024  # fiode_odetrain_config.max_attempts
FIODE_ODEINT_MAX_BATCH = 65536      # fiode_odeint (tile-parallel eval-mode solve)
FIODE_SMALL_CAYLEY_MAX_K, FIODE_SMALL_CAYLEY_MAX_RK = 16, 8192


class OdeConfig(ct.Structure):
    _fields_ = [("method", ct.c_int32), ("batch", ct.c_int32), ("n_times", ct.c_int32), ("max_steps", ct.c_int32),
                ("rtol", ct.c_double), ("atol", ct.c_double), ("step_size", ct.c_double)]


class OdeTrainConfig(ct.Structure):
    _fields_ = [("batch", ct.c_int32), ("dropout_mode", ct.c_int32), ("seed", ct.c_uint64), ("offset", ct.c_uint64),
                ("t0", ct.c_double), ("t1", ct.c_double), ("step_size", ct.c_double), ("method", ct.c_int32),
                ("max_attempts", ct.c_int32), ("rtol", ct.c_double), ("atol", ct.c_double)]


class SpectralConfig(ct.Structure):
    _fields_ = [("cout", ct.c_int32), ("cin", ct.c_int32), ("ks", ct.c_int32), ("n", ct.c_int32)]


ABI_VERSION = 5            # FIODE_ABI_VERSION (include/fiode.h)
FIODE_ODETRAIN_NSAVED = 14  # entries fiode_odetrain_saved_offsets writes
FIODE_GUARD_MAX_STATUS = 4


class StepGuard(ct.Structure):
    """fiode_step_guard: device pointers (nullable) whose values decide whether a step is applied."""
    _fields_ = [("flag", ct.c_void_p), ("loss", ct.c_void_p), ("status", ct.c_void_p * FIODE_GUARD_MAX_STATUS),
                ("skipped", ct.c_void_p)]


class AdamConfig(ct.Structure):
    _fields_ = [("n_tensors", ct.c_int32), ("decoupled", ct.c_int32), ("maximize", ct.c_int32),
                ("increment_steps", ct.c_int32),
                ("lr", ct.c_double), ("beta1", ct.c_double), ("beta2", ct.c_double), ("eps", ct.c_double),
                ("weight_decay", ct.c_double), ("step", ct.c_double), ("lr_dev", ct.c_void_p),
                ("lr_dev_is_double", ct.c_int32), ("pad2_", ct.c_int32)]


class SconvConfig(ct.Structure):
    _fields_ = [("n", ct.c_int32), ("C", ct.c_int32), ("B", ct.c_int32), ("downsample", ct.c_int32),
                ("nchw", ct.c_int32)]


class DenseConfig(ct.Structure):
    _fields_ = [("batch", ct.c_int32), ("cout", ct.c_int32), ("cin", ct.c_int32)]


class GemmDesc(ct.Structure):
    """fiode_gemm_desc (include/fiode.h)."""
    _fields_ = [("batch", ct.c_int32), ("M", ct.c_int32), ("N", ct.c_int32), ("K", ct.c_int32),
                ("trans_a", ct.c_int32), ("trans_b", ct.c_int32), ("lda", ct.c_int64), ("ldb", ct.c_int64),
                ("ldc", ct.c_int64), ("stride_a", ct.c_int64), ("stride_b", ct.c_int64), ("stride_c", ct.c_int64),
                ("alpha", ct.c_float), ("beta", ct.c_float), ("split_k", ct.c_int32), ("max_workgroups", ct.c_int32)]


class CertifyConfig(ct.Structure):
    _fields_ = [("n_classes", ct.c_int32), ("T", ct.c_int32), ("batches", ct.c_int32), ("label", ct.c_int32),
                ("eps", ct.c_float), ("min_std", ct.c_float)]


def _load():
    if not LIB_PATH.exists():
        raise FiodeLibraryError(
            f"libfiode.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:
        lib = ct.CDLL(str(LIB_PATH))
    except OSError as e:  # pragma: no cover - depends on the box
        raise FiodeLibraryError(f"failed to load {LIB_PATH}: {e}") from e
    sig = {
        "fiode_lyap_workspace_bytes": (ct.c_size_t, [ct.POINTER(LyapConfig), ct.POINTER(DynConfig)]),
        "fiode_lyap_step": (ct.c_int, [_vp, ct.POINTER(LyapConfig), ct.POINTER(DynConfig), ct.POINTER(DynWeights),
                                       ct.POINTER(LyapIO), ct.POINTER(LyapGrads), _vp, ct.c_size_t]),
        "fiode_qp_forward": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, _vp, _vp, ct.c_int32, ct.c_float, _vp, _vp,
                                        _vp, _vp, ct.c_size_t]),
        "fiode_qp_backward": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
        "fiode_dyn_eval_workspace_bytes": (ct.c_size_t, [ct.c_int32]),
        "fiode_dyn_eval": (ct.c_int, [_vp, ct.POINTER(DynConfig), ct.POINTER(DynWeights), ct.c_int32, ct.c_int32,
                                      _vp, _vp, _vp, _vp, _vp, ct.c_size_t]),
        "fiode_odeint_workspace_bytes": (ct.c_size_t, [ct.c_int32]),
        "fiode_odeint": (ct.c_int, [_vp, ct.POINTER(OdeConfig), ct.POINTER(DynConfig), ct.POINTER(DynWeights),
                                    _vp, _vp, _vp, _vp, _vp, _vp, _vp, ct.c_size_t]),
        "fiode_certify_grid_rows": (ct.c_int64, [ct.c_int32, ct.c_int32]),
        "fiode_certify_grid": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, _vp]),
        "fiode_certify_workspace_bytes": (ct.c_size_t, [ct.c_int64, ct.c_int32]),
        "fiode_certify": (ct.c_int, [_vp, ct.POINTER(CertifyConfig), ct.POINTER(DynConfig), ct.POINTER(DynWeights),
                                     _vp, _vp, ct.c_int64, _vp, _vp, _vp, ct.c_size_t]),
        "fiode_odetrain_evals": (ct.c_int32, [ct.POINTER(OdeTrainConfig)]),
        "fiode_odetrain_saved_offsets": (ct.c_int, [ct.POINTER(OdeTrainConfig), _vp]),
        "fiode_odetrain_workspace_bytes": (ct.c_size_t, [ct.POINTER(OdeTrainConfig)]),
        "fiode_odetrain_forward": (ct.c_int, [_vp, ct.POINTER(OdeTrainConfig), ct.POINTER(DynConfig),
                                              ct.POINTER(DynWeights), _vp, _vp, _vp, _vp, _vp, _vp, _vp, ct.c_size_t]),
        "fiode_odetrain_backward": (ct.c_int, [_vp, ct.POINTER(OdeTrainConfig), ct.POINTER(DynConfig),
                                               ct.POINTER(DynWeights), _vp, _vp, ct.POINTER(LyapGrads), _vp, _vp,
                                               ct.c_size_t]),
        "fiode_odetrain_backward_x": (ct.c_int, [_vp, ct.POINTER(OdeTrainConfig), ct.POINTER(DynConfig),
                                                 ct.POINTER(DynWeights), _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                 ct.c_size_t]),
        "fiode_odetrain_backward_weights": (ct.c_int, [_vp, ct.POINTER(OdeTrainConfig), ct.POINTER(DynConfig),
                                                       ct.POINTER(DynWeights), _vp, ct.POINTER(LyapGrads), _vp,
                                                       ct.c_size_t]),
        "fiode_groupsort_forward": (ct.c_int, [_vp, ct.c_int64, ct.c_int64, ct.c_int64, _vp, _vp]),
        "fiode_groupsort_backward": (ct.c_int, [_vp, ct.c_int64, ct.c_int64, ct.c_int64, _vp, _vp, _vp]),
        "fiode_head_out": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, ct.c_int32, _vp, _vp, _vp, _vp]),
        "fiode_head_out_backward_gs": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, ct.c_int32, _vp, _vp, _vp, _vp]),
        "fiode_batched_inverse": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, ct.c_int32, _vp, ct.c_int64, _vp,
                                             ct.c_int64]),
        "fiode_block_inverse_workspace_bytes": (ct.c_size_t, [ct.c_int32]),
        "fiode_block_inverse": (ct.c_int, [_vp, ct.c_int32, _vp, _vp, _vp, ct.c_size_t]),
        "fiode_block_inverse_batched": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, _vp, _vp, _vp, ct.c_size_t]),
        "fiode_block_inverse_cond": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, _vp, _vp, _vp, ct.c_size_t, _vp]),
        "fiode_normalize_hwcb": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, ct.c_int32, ct.c_int32, _vp, _vp, _vp, _vp]),
        "fiode_ode_nll": (ct.c_int, [_vp, ct.c_int32, _vp, _vp, _vp, _vp]),
        "fiode_ode_loss_mix": (ct.c_int, [_vp, ct.c_int32, _vp, _vp, _vp, ct.c_float, _vp, _vp, _vp]),
        "fiode_small_cayley_forward": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, ct.c_int32, _vp, _vp, _vp, _vp, _vp]),
        "fiode_small_cayley_backward": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, ct.c_int32, _vp, _vp, _vp, _vp, _vp,
                                                   _vp, _vp]),
        "fiode_dense_cayley_prep": (ct.c_int, [_vp, ct.POINTER(DenseConfig), _vp, _vp, _vp, _vp, _vp]),
        "fiode_dense_norm_workspace_bytes": (ct.c_size_t, [ct.POINTER(DenseConfig)]),
        "fiode_dense_norm_partials": (ct.c_int, [_vp, ct.POINTER(DenseConfig), _vp, _vp, ct.c_size_t]),
        "fiode_dense_cayley_prep_normed": (ct.c_int, [_vp, ct.POINTER(DenseConfig), _vp, _vp, _vp, _vp, _vp, _vp]),
        "fiode_dense_norm_partials_clear": (ct.c_int, [_vp, ct.POINTER(DenseConfig), _vp, _vp, ct.c_size_t, _vp,
                                                       ct.c_size_t, ct.c_size_t]),
        "fiode_dense_inverse_flag_bytes": (ct.c_size_t, [ct.c_int32]),
        "fiode_dense_cayley_inverse": (ct.c_int, [_vp, ct.POINTER(DenseConfig), _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                  _vp, ct.c_size_t]),
        "fiode_dense_cayley_finish": (ct.c_int, [_vp, ct.POINTER(DenseConfig), _vp, _vp, _vp, _vp, _vp]),
        "fiode_dense_cayley_ginv": (ct.c_int, [_vp, ct.POINTER(DenseConfig), _vp, _vp, _vp, _vp, _vp]),
        "fiode_dense_cayley_h": (ct.c_int, [_vp, ct.POINTER(DenseConfig), _vp, _vp, _vp]),
        "fiode_dense_cayley_workspace_bytes": (ct.c_size_t, [ct.POINTER(DenseConfig)]),
        "fiode_dense_cayley_grad": (ct.c_int, [_vp, ct.POINTER(DenseConfig), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                               _vp, ct.c_size_t]),
        "fiode_dense_gemm": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, ct.c_int32, ct.c_int32, _vp, _vp, _vp]),
        "fiode_gemm_splits": (ct.c_int32, [ct.POINTER(GemmDesc)]),
        "fiode_gemm_counter_bytes": (ct.c_size_t, [ct.POINTER(GemmDesc)]),
        "fiode_gemm_workspace_bytes": (ct.c_size_t, [ct.POINTER(GemmDesc)]),
        "fiode_gemm": (ct.c_int, [_vp, ct.POINTER(GemmDesc), _vp, _vp, _vp, _vp, _vp, ct.c_size_t]),
        "fiode_gemm_pair_workspace_bytes": (ct.c_size_t, [ct.POINTER(GemmDesc), ct.POINTER(GemmDesc)]),
        "fiode_gemm_pair": (ct.c_int, [_vp, ct.POINTER(GemmDesc), _vp, _vp, _vp, _vp, ct.POINTER(GemmDesc), _vp, _vp,
                                       _vp, _vp, _vp, ct.c_size_t]),
        "fiode_sconv_rfft2": (ct.c_int, [_vp, ct.POINTER(SconvConfig), _vp, _vp, _vp, _vp]),
        "fiode_sconv_irfft2": (ct.c_int, [_vp, ct.POINTER(SconvConfig), _vp, _vp, ct.c_int32, _vp, _vp]),
        "fiode_sconv_rfft2_nchw": (ct.c_int, [_vp, ct.POINTER(SconvConfig), _vp, _vp, _vp, _vp]),
        "fiode_sconv_irfft2_qx": (ct.c_int, [_vp, ct.POINTER(SconvConfig), _vp, _vp, ct.c_int32, _vp, ct.c_int32,
                                             _vp, _vp]),
        "fiode_cgemm": (ct.c_int, [_vp, ct.c_int32, ct.c_int32, ct.c_int32, ct.c_int32, ct.c_int32, ct.c_int32, _vp,
                                   _vp, _vp, _vp]),
        "fiode_spectral_workspace_bytes": (ct.c_size_t, [ct.POINTER(SpectralConfig)]),
        "fiode_spectral_cayley_forward": (ct.c_int, [_vp, ct.POINTER(SpectralConfig), _vp, _vp, _vp, _vp, _vp,
                                                     ct.c_size_t]),
        "fiode_spectral_cayley_backward": (ct.c_int, [_vp, ct.POINTER(SpectralConfig), _vp, _vp, _vp, _vp, _vp, _vp,
                                                      _vp, ct.c_size_t]),
        "fiode_adam_step": (ct.c_int, [_vp, ct.POINTER(AdamConfig), _vp, _vp, _vp, _vp, _vp, _vp,
                                       ct.POINTER(StepGuard)]),
        "fiode_step_guard_flag": (ct.c_int, [_vp, ct.POINTER(StepGuard), _vp]),
        "fiode_error_string": (ct.c_char_p, [ct.c_int]),
        "fiode_abi_version": (ct.c_int, []),
    }
    for name, (res, args) in sig.items():
        if not hasattr(lib, name) and "FIODE_LIB" in os.environ:
            continue        # an older build under an A/B (tools/gpu_lib_ab.sh): callers check hasattr
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        lb = _load()
        v = lb.fiode_abi_version()
        if v != ABI_VERSION:
            raise FiodeLibraryError(f"{LIB_PATH}: ABI version {v}, this package binds {ABI_VERSION} "
                                    "(stale build: run `make -C fi-ode_amd/csrc`)")
        _LIB = lb
    return _LIB


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().fiode_error_string(rc)
        raise FiodeError(f"{what} failed: {msg.decode() if msg else rc} (code {rc})")
