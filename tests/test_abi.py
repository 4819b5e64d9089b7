"""CPU checks of the C-ABI boundary: libfiode.so loads and exports every symbol include/fiode.h
declares, with host-only entry points callable (no GPU needed)."""
import ctypes as ct
import pathlib
import re

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def declared_symbols():
    text = (ROOT / "include" / "fiode.h").read_text()
    return re.findall(r"FIODE_API\s+[\w\s\*]+?\b(fiode_\w+)\s*\(", text)


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("fiode_lyap_step", "fiode_lyap_workspace_bytes", "fiode_qp_forward", "fiode_qp_backward",
              "fiode_dyn_eval", "fiode_error_string", "fiode_abi_version"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from fiode_amd import _lib
    lib = ct.CDLL(str(_lib.LIB_PATH))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_host_only_entry_points():
    from fiode_amd import _lib
    lib = _lib.lib()
    assert lib.fiode_abi_version() == _lib.ABI_VERSION == 5
    hdr = (pathlib.Path(__file__).resolve().parents[1] / "include" / "fiode.h").read_text()
    for name in ("FIODE_ABI_VERSION", "FIODE_ODETRAIN_NSAVED"):
        val = int(re.search(r"#define %s (\d+)" % name, hdr).group(1))
        assert val == getattr(_lib, name.replace("FIODE_ABI_", "ABI_")), name
    assert lib.fiode_error_string(2).decode().startswith("unsupported shape")
    cfg = _lib.LyapConfig(128, 256, 204, 1, 2, 2.0, 0, 0)
    dyn = _lib.DynConfig(10, 128, 10, 100.0, 20.0, 0.02, 1, 0.5, 30, 1e-4)
    N = 128 * 256
    slab = 19216 * 4
    # the fused backward keeps activations on chip: h, ft (2 passes), keep words, the per-tile g_u
    # partials and one fixed-order fp32 weight-gradient slab per backward workgroup (256 at this N)
    nb = lib.fiode_lyap_workspace_bytes(ct.byref(cfg), ct.byref(dyn))
    assert 256 * slab <= nb < 4 * N * 128 * 4


def test_bad_shapes_rejected_before_launch():
    """Shape/argument errors are refused on the host (no kernel is launched)."""
    from fiode_amd import _lib
    lib = _lib.lib()
    dyn_bad = _lib.DynConfig(12, 128, 10, 100.0, 20.0, 0.02, 1, 0.5, 30, 1e-4)
    cfg = _lib.LyapConfig(4, 8, 8, 0, 0, 2.0, 0, 0)
    rc = lib.fiode_lyap_step(None, ct.byref(cfg), ct.byref(dyn_bad), None, None, None, None, 0)
    assert rc == 2
    assert lib.fiode_qp_forward(None, 5, 11, None, None, 30, 1e-4, None, None, None, None, 0) == 2
    dyn = _lib.DynConfig(10, 128, 10, 100.0, 20.0, 0.02, 1, 0.5, 40, 1e-4)     # qp_max_iter > 32
    assert lib.fiode_lyap_step(None, ct.byref(cfg), ct.byref(dyn), None, None, None, None, 0) == 1


def test_batched_inverse_argument_checks():
    """fiode_batched_inverse validates before launching: n <= 128, known dtype, strides >= n*n;
    an empty batch is a no-op."""
    from fiode_amd import _lib
    lib = _lib.lib()
    assert lib.fiode_batched_inverse(None, 0, 0, 4, None, 16, None, 16) == 0
    assert lib.fiode_batched_inverse(None, 0, 1, 129, None, 0, None, 0) == 1
    assert lib.fiode_batched_inverse(None, 7, 1, 4, None, 16, None, 16) == 1
    buf = ct.create_string_buffer(64)
    assert lib.fiode_batched_inverse(None, 0, 1, 4, buf, 15, buf, 16) == 2


def test_spectral_cayley_host_checks():
    """fiode_spectral_*: workspace sizing and argument checks run on the host (no launch)."""
    import ctypes as ct
    from fiode_amd import _lib
    lib = _lib.lib()
    ok = _lib.SpectralConfig(64, 256, 3, 8)          # KWLarge conv 4 (wide, K = 64)
    nf = 8 * 5
    nb = lib.fiode_spectral_workspace_bytes(ct.byref(ok))
    assert nb >= nf * 64 * 256 * 8 + nf * 4           # gX scratch + D partials
    assert lib.fiode_spectral_workspace_bytes(ct.byref(_lib.SpectralConfig(8, 8, 5, 16))) == 0   # 5x5 taps
    assert lib.fiode_spectral_workspace_bytes(ct.byref(_lib.SpectralConfig(128, 128, 3, 16))) == 0  # K > 64
    assert lib.fiode_spectral_workspace_bytes(ct.byref(_lib.SpectralConfig(8, 8, 3, 7))) == 0     # odd n
    assert lib.fiode_spectral_cayley_forward(None, ct.byref(ok), None, None, None, None, None, 0) == 1
    dummy = ct.c_void_p(1)
    assert lib.fiode_spectral_cayley_forward(None, ct.byref(ok), dummy, dummy, dummy, dummy, dummy, nb - 1) == 3
    assert lib.fiode_spectral_cayley_backward(None, ct.byref(_lib.SpectralConfig(8, 8, 5, 16)), dummy, dummy, dummy,
                                              dummy, dummy, dummy, dummy, nb) == 2


def test_block_inverse_host_checks():
    from fiode_amd import _lib
    lib = _lib.lib()
    # n = 128 .. 512 in 64-steps: the one-launch inverse (flags, 8 versions of the 64 tiles, 8 pivot
    # inverses, an input copy for in == out)
    assert lib.fiode_block_inverse_workspace_bytes(512) == (576 + 8 * 64 * 4096 + 8 * 4096 + 64 * 4096) * 4
    assert lib.fiode_block_inverse_workspace_bytes(65) == (2 * 128 * 128 + 2 * 64 * 64) * 4
    assert lib.fiode_block_inverse(None, 0, None, None, None, 0) == 1
    dummy = ct.c_void_p(1)
    assert lib.fiode_block_inverse(None, 512, dummy, dummy, dummy, 100) == 3


def test_small_cayley_host_checks():
    """fiode_small_cayley_*: k = min(cout, cin) <= 16 and max(cout, cin) * k <= 8192, else EINVAL
    (checked before any launch); an empty batch is a no-op."""
    from fiode_amd import _lib as L
    lib = L.lib()
    assert lib.fiode_small_cayley_forward(None, 1, 17, 40, None, None, None, None, None) == 1
    assert lib.fiode_small_cayley_forward(None, 1, 10, 820, None, None, None, None, None) == 1
    assert lib.fiode_small_cayley_forward(None, 1, 10, 20, None, None, None, None, None) == 1   # NULL pointers
    assert lib.fiode_small_cayley_forward(None, 0, 10, 20, None, None, None, None, None) == 0
    assert lib.fiode_small_cayley_backward(None, 1, 16, 513, None, None, None, None, None, None, None) == 1


def test_adam_step_host_checks():
    """fiode_adam_step validates the tensor table before launching: n_tensors <= 64, numel >= 0,
    no NULL pointer for a non-empty tensor; zero tensors is a no-op."""
    from fiode_amd import _lib as L
    lib = L.lib()
    cfg = L.AdamConfig(2, 0, 0, 0, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0)
    arr = ct.c_void_p * 2
    one = arr(1, 2)
    assert lib.fiode_adam_step(None, ct.byref(cfg), one, one, one, one, (ct.c_int64 * 2)(5, -1), None, None) == 1
    assert lib.fiode_adam_step(None, ct.byref(cfg), arr(1, None), one, one, one, (ct.c_int64 * 2)(5, 3), None, None) == 1
    cfg.n_tensors = 65
    assert lib.fiode_adam_step(None, ct.byref(cfg), None, None, None, None, None, None, None) == 1
    cfg.n_tensors = 0
    assert lib.fiode_adam_step(None, ct.byref(cfg), None, None, None, None, None, None, None) == 0
    # the library increments the step counts only through a step-pointer table
    cfg.n_tensors, cfg.increment_steps = 2, 1
    assert lib.fiode_adam_step(None, ct.byref(cfg), one, one, one, one, (ct.c_int64 * 2)(5, 3), None, None) == 1
    g = L.StepGuard()
    assert lib.fiode_step_guard_flag(None, None, None) == 1
    assert lib.fiode_step_guard_flag(None, ct.byref(g), None) == 1


def test_fiode_adam_cpu_params_use_torch_step():
    """FiodeAdam on CPU parameters is torch.optim.Adam exactly (the kernel covers ROCm tensors)."""
    import torch
    from fiode_amd.optim import FiodeAdam
    g = torch.Generator().manual_seed(0)
    p = torch.nn.Parameter(torch.randn(7, generator=g))
    q = torch.nn.Parameter(p.detach().clone())
    o1 = FiodeAdam([p], lr=1e-2, weight_decay=1e-3)
    o2 = torch.optim.Adam([q], lr=1e-2, weight_decay=1e-3)
    for _ in range(3):
        gr = torch.randn(7, generator=g)
        p.grad, q.grad = gr.clone(), gr.clone()
        o1.step()
        o2.step()
    assert torch.equal(p, q)
    assert isinstance(o1, torch.optim.Adam)
    assert o1.state_dict()["state"][0]["step"].item() == 3


def test_odetrain_backward_parts_host_checks():
    """fiode_odetrain_backward_x / _weights refuse missing arguments before any launch (gx_add
    without its scale; a NULL gradient output)."""
    from fiode_amd import _lib as L
    lib = L.lib()
    assert lib.fiode_odetrain_backward_x(None, None, None, None, None, None, None, None, None, None, None, 0) == 1
    assert lib.fiode_odetrain_backward_weights(None, None, None, None, None, None, None, 0) == 1
    cfg = L.OdeTrainConfig(8, 0, 0, 0, 0.0, 1.0, 0.25)
    dyn = L.DynConfig(10, 128, 10, 100.0, 20.0, 0.02, 1, 0.5, 30, 1e-4)
    d = ct.c_void_p(1)
    w = L.DynWeights(*([d] * 8))
    big = 1 << 40
    # gx_add given, scale missing
    assert lib.fiode_odetrain_backward_x(None, ct.byref(cfg), ct.byref(dyn), ct.byref(w), d, d, d, d, None, None, d,
                                         big) == 1
    g = L.LyapGrads(*([d] * 8 + [None]))
    g.Q2 = None
    assert lib.fiode_odetrain_backward_weights(None, ct.byref(cfg), ct.byref(dyn), ct.byref(w), d, ct.byref(g), d,
                                               big) == 1


def test_odetrain_dopri5_shape_on_host():
    """The dopri5 train_ode solve's host-side shape (no kernel): eval capacity 2 + 6 max_attempts,
    the dopri5 extras in the saved offsets, invalid tolerances / capacities refused; the module's
    plan for the YAML's train_ode_solver dopri5 (cifar_train.yaml:30,32) is a dopri5 config with
    rtol = atol = train_ode_tol."""
    import ctypes as ct
    from fiode_amd import _lib, ops
    lib = _lib.lib()
    cfg = ops.odetrain_config(128, 0.0, 1.0, 0.0, _lib.FIODE_DROPOUT_PHILOX, method="dopri5", rtol=1e-3, atol=1e-3,
                              max_attempts=64)
    assert lib.fiode_odetrain_evals(ct.byref(cfg)) == 2 + 6 * 64
    rk = ops.odetrain_config(128, 0.0, 1.0, 0.1, _lib.FIODE_DROPOUT_PHILOX)
    assert lib.fiode_odetrain_evals(ct.byref(rk)) == 40
    assert lib.fiode_odetrain_workspace_bytes(ct.byref(cfg)) > lib.fiode_odetrain_workspace_bytes(ct.byref(rk))
    off = (ct.c_int64 * _lib.FIODE_ODETRAIN_NSAVED)()
    assert lib.fiode_odetrain_saved_offsets(ct.byref(cfg), ct.cast(off, ct.c_void_p)) == 0
    assert all(off[i] > 0 for i in (9, 10, 11))
    assert lib.fiode_odetrain_saved_offsets(ct.byref(rk), ct.cast(off, ct.c_void_p)) == 0
    assert all(off[i] == 0 for i in (9, 10, 11))
    for bad in (dict(rtol=0.0), dict(max_attempts=0), dict(max_attempts=5000)):
        kw = dict(rtol=1e-3, atol=1e-3, max_attempts=64)
        kw.update(bad)
        c = ops.odetrain_config(128, 0.0, 1.0, 0.0, _lib.FIODE_DROPOUT_PHILOX, method="dopri5", **kw)
        assert lib.fiode_odetrain_evals(ct.byref(c)) == -1
        assert lib.fiode_odetrain_workspace_bytes(ct.byref(c)) == 0
    import bench
    import torch
    mod = bench.build_module(torch.device("cpu"), train_ode=True, solver="dopri5")
    plan = mod.ode_plan(128)
    assert plan["cfg"].method == _lib.FIODE_ODE_DOPRI5 and plan["cfg"].rtol == plan["cfg"].atol == 1e-3
