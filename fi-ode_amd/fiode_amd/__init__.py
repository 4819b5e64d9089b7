"""fiode_amd -- MI355X-native (gfx950 HIP) forward-invariance hot path of FI-ODE.

Host-side mirror of the reference's plugin surface (yjhuangcd/FI-ODE): the dynamics class,
QP projection, Lyapunov candidate, samplers/schedulers, IVP/odeint and LyapunovLearning keep
their names, constructor fields and state_dict keys; their per-sample work runs in
libfiode.so (fi-ode_amd/csrc, C-ABI in include/fiode.h).
"""
from . import _lib  # noqa: F401  (fails loudly if libfiode.so is missing -- no CPU fallback)

__all__ = ["_lib"]
__version__ = "0.1.0"
