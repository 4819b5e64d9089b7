"""Phase timing of k_ot_fwd (needs tools/libfiode_prof.so built with -DOT_PROFILE; not a test)."""
import ctypes as ct, os, sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
os.environ.setdefault("FIODE_LIB", str(ROOT / "tools" / "libfiode_prof.so"))
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np, torch
from fiode_amd import _lib as L, ops
from tests._util import make_params
dev = torch.device("cuda:0")
P = make_params(1)
w = {k: torch.from_numpy(np.ascontiguousarray(getattr(P, k))).to(dev) for k in ops.WEIGHT_KEYS}
for B, sn in ((128, False), (128, True), (1024, False)):
    x = torch.randn(B, 10, device=dev); h0 = torch.full((B, 10), 0.1, device=dev)
    cfg = ops.odetrain_config(B, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=3)
    dyn = ops.DynCfg(scale_nominal=sn, dropout=0.5)
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); y, st, ws = ops.odetrain_forward(x, h0, w, dyn, cfg); e1.record(); torch.cuda.synchronize()
    E = ops.odetrain_evals(cfg); nt = (B + 3) // 4   # the prof words follow E x 2 x (4-row tiles) granules
    off = ct.c_int64 * 8
    # prof array sits after the exchange granules
    lib = L.lib()
    offs = (ct.c_int64 * L.FIODE_ODETRAIN_NSAVED)()
    # xslots offset = gft offset + al(R*C*4)
    lib.fiode_odetrain_saved_offsets(ct.byref(cfg), ct.cast(offs, ct.c_void_p))
    al = lambda v: (v + 255) & ~255
    xs = offs[7] + al(B * E * 10 * 4)
    prof = ws[xs + (4 * 2 * nt * 16 + 8) * 8: xs + (2 * E * nt * 16 + 8 + 16 + E) * 8].view(torch.int64).cpu().numpy()
    # the backward's VJP phases (prof[10..15], accumulated over its E VJPs on top of the forward's)
    b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b0.record(); ops.odetrain_backward(torch.ones_like(y), x, w, dyn, cfg, ws); b1.record(); torch.cuda.synchronize()
    pb = ws[xs + (4 * 2 * nt * 16 + 8) * 8: xs + (2 * E * nt * 16 + 8 + 16) * 8].view(torch.int64).cpu().numpy()
    vj = (pb[10:16] - prof[10:16]) / E * 0.01
    print(f"  backward total {b0.elapsed_time(b1)*1e3:.0f} us, per VJP (us): row math {vj[0]:.2f} g_a2 {vj[1]:.2f} "
          f"g_a1 {vj[2]:.2f} g_h partial {vj[3]:.2f} barrier {vj[4]:.2f} sum {vj[5]:.2f}", flush=True)
    Ks = prof[16:16 + E].tolist()               # the last rep's exit K of every eval
    ticks = prof[:8] / E          # 100 MHz wall clock -> 10 ns per tick
    print(f"B={B} total {e0.elapsed_time(e1)*1e3:.0f} us, per eval (us): mlp {ticks[1]*0.01:.2f} "
          f"partial sums+nominal {ticks[5]*0.01:.2f} bisection+exit exchange {ticks[3]*0.01:.2f} "
          f"(bisection {ticks[6]*0.01:.2f}, exchange wait {ticks[7]*0.01:.2f}, resumes {int(prof[8])}/{E}) "
          f"finalize {ticks[4]*0.01:.2f}  status {st.cpu().numpy().tolist()} scale_nominal={sn}\n  exit K per eval: {Ks}", flush=True)
