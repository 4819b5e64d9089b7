"""Interleaved A/B of step variants (not a test): every variant's hipGraph step is captured first,
then replayed round-robin (R rounds x K steps each), so box-level drift hits all variants alike.

python tools/ab_step.py [rounds] [variant,variant,...]  ->  one JSON line: median ms per step per variant
"""
import json
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
    mod = bench.build_module(dev, train_ode=True)
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
                          maps_ahead_linear=getattr(mod, "_ahead_lin", False),
                          refresh_after_backward=getattr(mod, "_late_refresh", False))


def nogroup(m):
    m.group_lin_maps = False


def after_ode(m):
    m.lyap_after_ode = True


def grouped(m):
    m.group_lin_maps = True


def unfused_normalize(m):
    m.init_coordinates.param_map[0].fused_hwcb = False


def no_small_cayley(m):
    from fiode_amd import cayley
    cayley.SMALL_FUSED = False      # (module-global: restored by the next variant's build)


def small_cayley_on(m):
    from fiode_amd import cayley
    cayley.SMALL_FUSED = True


def maps_after_input(m):
    m.prefetch_schedule = {"after_input": True}


def sched(**kw):
    def f(m):
        m.prefetch_schedule = {"after_input": True, **kw}
    return f


def at_start(m):
    m.prefetch_schedule = {}


def grouped_ai(m):
    m.group_lin_maps = True


def grouped_ai_linfirst(m):
    m.group_lin_maps = True
    m.prefetch_schedule = {"after_input": True, "order": "lin_first"}


def lin_first(m):
    m.prefetch_schedule = {"after_input": True, "order": "lin_first"}


def dense_bwd_main(m):
    from fiode_amd import cayley
    cayley.DENSE_BWD_ON_MAIN = True


def dense_bwd_side(m):
    from fiode_amd import cayley
    cayley.DENSE_BWD_ON_MAIN = False


def both_bwd_main(m):
    from fiode_amd import cayley
    cayley.DENSE_BWD_ON_MAIN = True
    cayley.SPECTRAL_BWD_ON_MAIN = True


def reset(m):
    from fiode_amd import cayley
    cayley.DENSE_BWD_ON_MAIN = False
    cayley.SPECTRAL_BWD_ON_MAIN = False


def dense_bwd_side(m):
    reset(m)


def reset2(m):
    from fiode_amd import cayley
    cayley.DENSE_BWD_ON_MAIN = True
    cayley.SPECTRAL_BWD_ON_MAIN = False
    cayley.SMALL_BWD_ON_MAIN = False


def small_bwd_main(m):
    from fiode_amd import cayley
    cayley.SMALL_BWD_ON_MAIN = True


def ode_on_main(m):
    m.ode_side_stream = False


def conv_first_split(m):
    m.prefetch_schedule = {"after_input": True, "order": "conv_first", "conv_streams": "split"}


def lin_first_split(m):
    m.prefetch_schedule = {"after_input": True, "order": "lin_first", "conv_streams": "split"}


def conv_first(m):
    m.prefetch_schedule = {"after_input": True, "order": "conv_first"}


def lin_one(m):
    m.prefetch_schedule = {"after_input": True, "order": "lin_first", "lin_streams": "one"}


def lin_one_conv_first(m):
    m.prefetch_schedule = {"after_input": True, "order": "conv_first", "lin_streams": "one"}


def ode_bwd_side(m):
    from fiode_amd import lyapunov
    lyapunov.ODE_BWD_ON_MAIN = False


def ode_bwd_main(m):
    from fiode_amd import lyapunov
    lyapunov.ODE_BWD_ON_MAIN = True


def blas_rocblas(m):
    torch.backends.cuda.preferred_blas_library("cublas")       # rocBLAS on ROCm


def blas_lt(m):
    torch.backends.cuda.preferred_blas_library("cublaslt")     # hipBLASLt on ROCm


def no_split(m):
    m.split_ode_wgrad = False


def split_own(m):
    m.split_ode_wgrad = "own"


def split_ode(m):
    m.split_ode_wgrad = "ode"


def conv_maps_cached(m):
    """probe only: the conv layers' spectral maps computed once (detached), no map forward or
    backward in the step -- the upper bound of hiding them entirely"""
    import types
    from fiode_amd.cayley import CayleyConv

    def prefetch(self, stream):
        if self._n is None or not self._alpha_init:
            return CayleyConv.prefetch(self, stream)
        if getattr(self, "_cachedQ", None) is None:
            with torch.no_grad():
                self._cachedQ = self.spectral_weight(self._n, self.weight.device).detach().clone()
        ev = torch.cuda.Event()
        ev.record()
        self._pre = (self._cachedQ, ev)
    for c in m.modules():
        if isinstance(c, CayleyConv):
            c.prefetch = types.MethodType(prefetch, c)


def no_ahead(m):
    m._no_ahead = True


def ahead_lin(m):
    m._ahead_lin = True


def late_refresh(m):
    m._late_refresh = True


def warm_inverse(m):
    from fiode_amd import cayley
    cayley.WARM_INVERSE = True


def newton3(m):
    from fiode_amd import cayley
    cayley.WARM_INVERSE = True
    cayley.NEWTON_ITERS = 3


def warm_square(m):
    from fiode_amd import cayley
    cayley.WARM_INVERSE = True
    cayley.WARM_WIDE = False


def ahead_small(m):
    m._ahead_lin = "small"


def seed1000(m):
    m.seed = 1000


def torch_adam(m):
    m._torch_adam = True


def unfused_loss(m):
    m.fused_ode_loss = False


ALL = {"default": reset2, "torch_adam": torch_adam, "no_split": no_split, "ahead_lin": ahead_lin, "seed1000": seed1000, "ahead_small": ahead_small, "warm_square": warm_square, "newton3": newton3, "warm_inverse": warm_inverse, "late_refresh": late_refresh, "lin0": sched(lin=[0, 0, 0], dyn=0), "lin1": sched(lin=[1, 1, 1], dyn=1), "lin2": sched(lin=[2, 2, 2], dyn=2), "at_start": at_start, "no_ahead": no_ahead, "conv_maps_cached": conv_maps_cached, "split_own": split_own, "split_ode": split_ode, "dense_bwd_side": dense_bwd_side, "unfused_loss": unfused_loss, "blas_rocblas": blas_rocblas, "ode_bwd_side": ode_bwd_side, "lin_one": lin_one, "lin_one_conv_first": lin_one_conv_first, "conv_first_split": conv_first_split, "lin_first_split": lin_first_split,
       "conv_first": conv_first, "small_bwd_main": small_bwd_main, "ode_on_main": ode_on_main, "grouped": grouped,
       "grouped_linfirst": grouped_ai_linfirst, "lin_first": lin_first}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["default", "small_bwd_main", "ode_on_main"]
VARIANTS = {k: ALL[k] for k in names}
steps = {}
for k, f in VARIANTS.items():
    steps[k] = make(f)
    reset2(None)                    # flags only matter at capture time (inside make)
    from fiode_amd import cayley as _c
    _c.WARM_INVERSE = False
    _c.NEWTON_ITERS = 2
    _c.WARM_WIDE = True
    ode_bwd_main(None)
    blas_lt(None)
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
