"""How predictable is the train_ode solve's batch-global QP exit?  (not a test)

Runs k_ot_fwd on the bench's configs[1] state (B=128, random-init KWLarge backbone features) for
several Philox offsets and reads back the exit-exchange granules ({epoch, mask} per eval, phase and
tile) the forward leaves in its workspace.  Per eval: the global exit K = lowest set bit of the AND
of the tiles' masks; per tile: its local first converged iteration.  Prints how often a tile's own
first converged iteration equals K, and the distribution of K - K_prev.

Since round 4 the granules are a ring of OT_XRING = 4 eval sets (odetrain.hip), so only the last 4
evals of each solve are still in the workspace: the statistics cover those.  The probe arms the
native backtrace handler (tools/native/libsegv_bt.so) and faulthandler: round 3's run of it ended
in a host SIGSEGV at interpreter teardown, after all its output.
"""
import faulthandler
import collections
import ctypes as ct
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "fi-ode_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fiode_amd import _lib as L, ops  # noqa: E402

XRING = 4
faulthandler.enable()
_BT = ROOT / "tools" / "native" / "libsegv_bt.so"
if _BT.exists():
    ct.CDLL(str(_BT))


def main():
    dev = torch.device("cuda:0")
    mod = bench.build_module(dev, seed=0, train_ode=True)
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(128, 3, 32, 32, generator=g).to(dev)
    with torch.no_grad():
        feat = mod.init_coordinates.param_map(x).float().contiguous()
        w = {k: v.detach().float().contiguous() for k, v in mod.dyn_fun.effective_weights().items()}
    B = 128
    h0 = torch.full((B, 10), 0.1, device=dev)
    dyn = mod.dyn_fun.dyn_cfg()
    lib = L.lib()
    hits = tot = 0
    pred = collections.Counter()      # predictor -> correct guesses

    def lowest_ge(mask, k):
        m = mask & ~((1 << max(k, 0)) - 1)
        return (m & -m).bit_length() - 1 if m else -1
    dk = collections.Counter()
    kc = collections.Counter()
    resumes = 0
    for off in range(8):
        cfg = ops.odetrain_config(B, 0.0, 1.0, 0.1, L.FIODE_DROPOUT_PHILOX, seed=7, offset=off)
        y, st, ws = ops.odetrain_forward(feat, h0, w, dyn, cfg)
        torch.cuda.synchronize()
        E = ops.odetrain_evals(cfg)
        nt = (B + 3) // 4 if B <= 1024 else (B + 15) // 16   # k_ot_fwd4 tiles (k_ot_fwd beyond)
        offs = (ct.c_int64 * L.FIODE_ODETRAIN_NSAVED)()
        lib.fiode_odetrain_saved_offsets(ct.byref(cfg), ct.cast(offs, ct.c_void_p))
        xs = offs[7] + ((B * E * 10 * 4 + 255) & ~255)
        xst = 16 if B <= 1024 else 1    # granule stride of k_ot_fwd4 (one line per tile)
        slots = ws[xs: xs + XRING * 2 * nt * xst * 8].view(torch.int64).cpu().numpy().astype(np.uint64).reshape(
            XRING, 2, nt, xst)[..., 0]
        kprev = dyn.qp_max_iter - 1
        for e in range(E - XRING, E):
            tag = int(slots[e % XRING, 0, 0] >> np.uint64(32))
            assert tag == e + 1, (e, tag)
            m0 = (slots[e % XRING, 0] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            kspec = min(dyn.qp_max_iter - 1, kprev + 3)
            allm = np.bitwise_and.reduce(m0)
            lowm = (1 << (kspec + 1)) - 1
            bits = int(allm) & lowm
            if bits:
                K = (bits & -bits).bit_length() - 1
            else:
                resumes += 1
                m1 = (slots[e % XRING, 1] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
                a1 = int(np.bitwise_and.reduce(m1))
                K = (a1 & -a1).bit_length() - 1 if a1 else dyn.qp_max_iter - 1
                m0 = m1
            for t in range(nt):
                loc = int(m0[t])
                f = (loc & -loc).bit_length() - 1 if loc else -1
                hits += f == K
                tot += 1
                for name, k in (("local_first", 0), ("ge_kprev-1", kprev - 1), ("ge_kprev", kprev),
                                ("ge_kprev+1", kprev + 1)):
                    pred[name] += lowest_ge(loc, k) == K
                pred["ge_max(f,kprev)"] += lowest_ge(loc, max(f, kprev)) == K
            dk[K - kprev] += 1
            kc[K] += 1
            kprev = K
        print(f"offset {off}: y finite {bool(torch.isfinite(y).all())}, last K {int(st[2])}", flush=True)
    print(f"tile-local first converged == global K: {hits}/{tot} = {hits / tot:.3f}")
    print("predictor accuracy:", {k: round(v / tot, 3) for k, v in pred.items()})
    print(f"resumes {resumes}; K distribution {sorted(kc.items())}")
    print(f"K - K_prev distribution {sorted(dk.items())} (the first of each solve's 4 evals vs max_iter - 1)")
    print("probe done; interpreter teardown next", flush=True)


if __name__ == "__main__":
    main()
