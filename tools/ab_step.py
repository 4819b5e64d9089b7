"""Interleaved A/B of step variants (not a test): every variant's hipGraph step is captured first,
then replayed round-robin (R rounds x K steps each), so box-level drift hits all variants alike.

python tools/ab_step.py [rounds] [variant,variant,...]  ->  one JSON line: median ms per step per variant

The round-2 scheduling knobs (linear maps ahead, late refresh, split weight-gradient node, prefetch
orders / stream layouts, warm-started inverses) were measured here and removed from the product
(DESIGN.md section 4 keeps their numbers); the variants left are the ones the product still has.
"""
import json
import os
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd.graph_step import GraphTrainStep  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)


def make(setup):
    # FIODE_AB_SOLVER=dopri5: the configs[2] step (train_ode dopri5, tol 1e-3) instead of rk4
    mod = bench.build_module(dev, train_ode=True, solver=os.environ.get("FIODE_AB_SOLVER", "rk4"))
    setup(mod)
    opt = mod.configure_optimizers(capturable=True)[0][0]
    if getattr(mod, "_torch_adam", False):
        g0 = opt.param_groups[0]
        opt = torch.optim.Adam(mod.parameters(), lr=g0["lr"], betas=g0["betas"], weight_decay=g0["weight_decay"],
                               fused=True, capturable=True)
    g = torch.Generator(device="cpu").manual_seed(1234)
    x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (128,), generator=g).to(dev)
    return GraphTrainStep(mod, opt, x, y, maps_ahead=not getattr(mod, "_no_ahead", False),
                          warm_capture=not getattr(mod, "_no_warm", False),
                          placement_trials=int(os.environ.get("FIODE_PLACEMENT_TRIALS", "1")))


def default(m):
    pass


def after_ode(m):
    m.lyap_after_ode = True


def no_ahead(m):
    m._no_ahead = True


def torch_adam(m):
    m._torch_adam = True


def unfused_loss(m):
    m.fused_ode_loss = False


def pf_conv0(m):
    m._prefetch_at = 0        # map prefetch captured after conv layer 0 instead of before it


def pf_conv1(m):
    m._prefetch_at = 1


RESTORE = []      # module-level switches a variant flips for its own capture only


def dense_bwd_side(m):
    from fiode_amd import cayley as CY
    CY.DENSE_BWD_ON_MAIN = False  # each dense map's backward on its forward's (prefetch) stream
    RESTORE.append(lambda: setattr(CY, "DENSE_BWD_ON_MAIN", True))


def lib_gmn(m):
    from fiode_amd import cayley as CY
    CY.DENSE_GEMM = False         # the dense maps' GMn products by the library GEMM
    RESTORE.append(lambda: setattr(CY, "DENSE_GEMM", True))




def ode_on_main(m):
    m.ode_side_stream = False


def seed1000(m):
    m.seed = 1000




def old_seed(m):
    """The round-3 fused-loss backward: loss.backward() (a ones fill), g_y = gunit * go,
    lyap * (go * (1 - p)) and a separate add -- for the A/B of the unit-seed backward."""
    from fiode_amd import graph_step as GS, lyapunov as LY, ops

    def old_backward(ctx, go):
        gunit, xo, w, oplan, ws = ctx.ode
        ctx.ode = None
        gr, _ = ops.odetrain_backward(gunit * go, xo, w, oplan["dyn"], oplan["cfg"], ws)
        keys = ("x_feat", "Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")
        ode = [gr[k] for k in keys]
        lyap = torch._foreach_mul(ctx.lyap, go * (1.0 - ctx.p))
        ctx.lyap = None
        torch._foreach_add_(ode, lyap)
        return (ode[0], None) + tuple(ode[1:]) + (None, None, None, None, None, None)
    nb, ug = LY.LyapODELossFn.backward, GS.GraphTrainStep._unit_grad
    LY.LyapODELossFn.backward = staticmethod(old_backward)
    GS.GraphTrainStep._unit_grad = lambda self, loss: None
    RESTORE.append(lambda: setattr(LY.LyapODELossFn, "backward", staticmethod(nb)))
    RESTORE.append(lambda: setattr(GS.GraphTrainStep, "_unit_grad", ug))


def torch_norm(m):
    from fiode_amd import cayley as CY
    CY.DENSE_NORM_PARTIALS = False        # the dense maps' norm by torch.linalg.vector_norm
    RESTORE.append(lambda: setattr(CY, "DENSE_NORM_PARTIALS", True))


def late_scale(m):
    """The unit-seed backward with lyap * (1 - p) made in the backward, after the solve's backward."""
    from fiode_amd import lyapunov as LY, ops

    def late_backward(ctx, go):
        gunit, xo, w, oplan, ws = ctx.ode
        ctx.ode = None
        gr, _ = ops.odetrain_backward(gunit, xo, w, oplan["dyn"], oplan["cfg"], ws)
        keys = ("x_feat", "Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3")
        ode = [gr[k] for k in keys]
        lyap = torch._foreach_mul(ctx.lyap, 1.0 - ctx.p)
        ctx.lyap = ctx.lyap_unit = None
        torch._foreach_add_(ode, lyap)
        return (ode[0], None) + tuple(ode[1:]) + (None, None, None, None, None, None)
    nb = LY.LyapODELossFn.backward
    LY.LyapODELossFn.backward = staticmethod(late_backward)
    RESTORE.append(lambda: setattr(LY.LyapODELossFn, "backward", staticmethod(nb)))


def ms_213(m):
    m._map_streams = (2, 1, 3, 3)       # the 4096 -> 512 map on side stream 2, 512 -> 512 on 1


def ms_321(m):
    m._map_streams = (3, 2, 1, 1)


def ms_3222(m):
    m._map_streams = (3, 2, 2, 2)


def ms_0(m):
    m._map_streams = (0, 2, 3, 3)       # the 4096 -> 512 map on the conv maps' stream


def first_ab(m):
    m._prefetch_first_lins = 2  # the 4096 -> 512 and 512 -> 512 maps before the conv stack


def first_dyn(m):
    m._prefetch_dyn_first = True   # the dynamics' maps before the conv stack too


def late2_first_ab(m):
    m._prefetch_first_lins = 2
    m._prefetch_dyn_first = True


def all_first(m):
    m._prefetch_late_at = None  # every map prefetched right after the input kernels (before r04bc)


def late0(m):
    m._prefetch_late_at = 0     # the 4096 -> 512 map before the conv stack, the other maps after conv 0


def late1(m):
    m._prefetch_late_at = 1


def late2(m):
    m._prefetch_late_at = 2


def late3(m):
    m._prefetch_late_at = 3     # ... after the last conv layer


def head_autograd(m):
    from fiode_amd import cayley as CY
    CY.HEAD_WGRAD_SIDE = False    # the linear head module by module (autograd's addmm backward)
    RESTORE.append(lambda: setattr(CY, "HEAD_WGRAD_SIDE", True))


def conv_wgrad_main(m):
    from fiode_amd import cayley as CY
    CY.CONV_WGRAD_SIDE = False    # the conv layers' weight / bias gradients after the input gradient, one stream
    RESTORE.append(lambda: setattr(CY, "CONV_WGRAD_SIDE", True))








def cap_hi(m):
    from fiode_amd import graph_step as GS
    GS.CAPTURE_PRIORITY = -1          # the step captured on a high-priority stream
    RESTORE.append(lambda: setattr(GS, "CAPTURE_PRIORITY", 0))


def ode_lo(m):
    m._ode_prio = 0                   # the train_ode solve's stream at normal priority










def norm_unfused(m):
    m.init_coordinates.param_map.fused_input = False   # Normalize's own kernel before conv 1 (before r05bm)


def nchw_last_off(m):
    m.init_coordinates.param_map[1].nchw_last = False    # the flatten's permute copies (before r05bo)




def qx_off(m):
    from fiode_amd import cayley as CY
    CY.SCONV_QX_MAX_K = 0         # conv 1's product by fiode_cgemm + the plain inverse transform (before r05cb)
    RESTORE.append(lambda: setattr(CY, "SCONV_QX_MAX_K", 4))


def head_out_lib(m):
    from fiode_amd import cayley as CY
    CY.HEAD_OUT_KERNEL = False    # the head's output layer by addmm, g Q3 + GroupSort backward (before r05cg)
    RESTORE.append(lambda: setattr(CY, "HEAD_OUT_KERNEL", True))


def lib_gemm(m):
    from fiode_amd import ops as OPS
    OPS.MM_LIBRARY = True         # every fiode_gemm product by torch.matmul (hipBLASLt) -- round 5's GEMMs
    RESTORE.append(lambda: setattr(OPS, "MM_LIBRARY", False))


def _lib_site(site):
    def f(m):
        from fiode_amd import ops as OPS
        OPS.MM_LIBRARY_SITES.add(site)
        RESTORE.append(lambda: OPS.MM_LIBRARY_SITES.discard(site))
    return f


def head_join_early(m):
    from fiode_amd import cayley as CY
    CY.HEAD_LATE_JOIN = False     # the head joins all three maps before its first layer (before r06)
    RESTORE.append(lambda: setattr(CY, "HEAD_LATE_JOIN", True))


def all_first_side(m):
    all_first(m)                  # every map prefetched at the step start: their nodes rank last ...
    dense_bwd_side(m)             # ... and each dense map's backward on its own prefetch stream


def _prio(mask):
    def v(m):
        import ctypes
        from fiode_amd import _lib as L
        f = L.lib().fiode_debug_set_prio_mask
        f.argtypes, f.restype = [ctypes.c_uint], ctypes.c_uint
        f(mask)                   # launch-time knob: this variant's capture keeps it
        RESTORE.append(lambda: f(3))     # (the library's default mask)
    return v


def no_warm(m):
    m._no_warm = True


def head_wg1(m):
    from fiode_amd import cayley as CY
    CY.HEAD_WGRAD_STREAMS = 1     # the head's three weight gradients in sequence on one stream (before r06)
    RESTORE.append(lambda: setattr(CY, "HEAD_WGRAD_STREAMS", 3))


def h0_copy(m):
    from fiode_amd import lyapunov as LY
    LY.H0_CACHE = False
    RESTORE.append(lambda: setattr(LY, "H0_CACHE", True))


def own_gemm(m):
    from fiode_amd import ops as OPS, cayley as CY
    sites = set(OPS.MM_LIBRARY_SITES)
    OPS.MM_LIBRARY_SITES.clear()         # fiode_gemm at every site, fiode_cgemm for the conv wgrad
    CY.CONV_WGRAD_LIB = False
    RESTORE.append(lambda: OPS.MM_LIBRARY_SITES.update(sites))
    RESTORE.append(lambda: setattr(CY, "CONV_WGRAD_LIB", True))


def lib3(m):
    for site in ("dense_fwd", "dense_bwd", "head"):
        _lib_site(site)(m)


def wgrad_lib(m):
    from fiode_amd import cayley as CY
    CY.CONV_WGRAD_LIB = True      # the conv weight gradient w G X^H by torch.matmul + scale (round 5)
    RESTORE.append(lambda: setattr(CY, "CONV_WGRAD_LIB", False))


def r05_gemms(m):
    lib_gemm(m)
    wgrad_lib(m)


def dyn_wgrad_main(m):
    from fiode_amd import lyapunov as LY
    LY.DYN_WGRAD_SIDE = False     # the dynamics weights' gradients inside LyapODELossFn's backward
    RESTORE.append(lambda: setattr(LY, "DYN_WGRAD_SIDE", True))


def ws_fill(m):
    from fiode_amd import ops as OPS
    OPS.WS_FILL_IN_CAPTURE = True     # GEMM workspaces made in the capture zeroed by a captured fill
    RESTORE.append(lambda: setattr(OPS, "WS_FILL_IN_CAPTURE", False))


def no_pair(m):
    from fiode_amd import ops as OPS
    OPS.MM_PAIR = False           # the dense maps' backward A and P2 as two launches (before r06)
    RESTORE.append(lambda: setattr(OPS, "MM_PAIR", True))


# variants of paths removed from the product after their A/B (the conv weight gradients on the map
# streams, fiode_cgemm for w G X^H, the library for thin / Q^H G products, h0 repeat, the pre-solve
# zero fill, one shared conv map stream) are kept only as records in DESIGN.md section 11
ALL = {"default": default, "ws_fill": ws_fill, "no_pair": no_pair, "lib_gemm": lib_gemm, "wgrad_lib": wgrad_lib, "r05_gemms": r05_gemms, "lib_dense_fwd": _lib_site("dense_fwd"),
       "lib_dense_bwd": _lib_site("dense_bwd"), "lib_head": _lib_site("head"), "lib3": lib3, "own_gemm": own_gemm, "h0_copy": h0_copy, "head_wg1": head_wg1, "no_warm": no_warm, "prio_otf": _prio(1), "prio_otb": _prio(2), "prio_small": _prio(4),
       "prio_pinv": _prio(8), "prio_all": _prio(15), "prio_ot": _prio(3),
       "prio_none": _prio(0), "all_first_side": all_first_side, "head_join_early": head_join_early, "head_autograd": head_autograd, "conv_wgrad_main": conv_wgrad_main,
       "cap_hi": cap_hi, "ode_lo": ode_lo, "norm_unfused": norm_unfused, "nchw_last_off": nchw_last_off, "dyn_wgrad_main": dyn_wgrad_main, "qx_off": qx_off, "head_out_lib": head_out_lib, "all_first": all_first, "first_ab": first_ab, "first_dyn": first_dyn,
       "late2_first_ab": late2_first_ab, "late0": late0, "late1": late1, "late2": late2, "late3": late3, "late3b": late3,
       "default_b": default, "ms_213": ms_213, "ms_321": ms_321, "ms_3222": ms_3222, "ms_0": ms_0, "torch_norm": torch_norm, "late_scale": late_scale, "after_ode": after_ode, "no_ahead": no_ahead, "torch_adam": torch_adam,
       "unfused_loss": unfused_loss, "ode_on_main": ode_on_main, "seed1000": seed1000, "pf_conv0": pf_conv0,
       "pf_conv1": pf_conv1, "dense_bwd_side": dense_bwd_side, "lib_gmn": lib_gmn, "old_seed": old_seed}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["default", "no_ahead"]
VARIANTS = {k: ALL[k] for k in names}
steps = {}
for k, f in VARIANTS.items():
    steps[k] = make(f)          # captured in GraphTrainStep.__init__
    while RESTORE:
        RESTORE.pop()()
times = {k: [] for k in VARIANTS}
for r in range(rounds):
    for k, gs in steps.items():
        for _ in range(3):
            gs.step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            gs.step()
        torch.cuda.synchronize()
        times[k].append((time.perf_counter() - t) / 20 * 1e3)
print(json.dumps({k: round(statistics.median(v), 4) for k, v in times.items()} |
                 {k + "_all": [round(t, 3) for t in v] for k, v in times.items()}), flush=True)
