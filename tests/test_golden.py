"""Golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU: the oracle reproduces its frozen vectors bit for bit, and agrees with the known answers
hand-derived from the reference's source text (reference_facts.json).  GPU: the HIP QP and the
fused Lyapunov step reproduce the same vectors (QP bit-exact; step within the tolerances of
tests/test_gpu_lyap.py, QP inputs pinned to the device's as there)."""
import json
import pathlib

import numpy as np
import pytest

from oracle import fiode_oracle as O

G = pathlib.Path(__file__).resolve().parent / "golden"


def _npz(name):
    return dict(np.load(G / name, allow_pickle=False))


def test_reference_facts():
    f = json.loads((G / "reference_facts.json").read_text())
    for ep, (s1, s2) in f["mixer_split_S256"].items():
        assert tuple(O.split_samples(256, O.cifar_train_mixer(int(ep)))) == (s1, s2)
    table = O.db_count_table(10, 40)
    assert table[40][10] == f["db_grid_G_10_40"]
    assert sum(f["db_grid_T40_count_by_max"].values()) == f["db_grid_G_10_40"]
    cb = O.certify_batches(f["db_grid_G_10_40"], f["certify_batches_G_10_40"]["batches"])
    assert len(cb) == f["certify_batches_G_10_40"]["n_slices"] and list(cb[-1]) == f["certify_batches_G_10_40"]["last"]
    for case in f["qp_hand_cases"]:
        r = O.qp_forward(np.array([case["lower"]], np.float32), np.array([case["nominal"]], np.float32))
        assert np.allclose(r.v[0], case["v"], atol=case["atol"])


def test_oracle_reproduces_qp_fixture():
    d = _npz("oracle_qp.npz")
    r = O.qp_forward(d["lower"], d["nominal"])
    assert r.iters == int(d["iters"])
    assert np.array_equal(r.v, d["v"]) and np.array_equal(r.mu, d["mu"])
    gl, gn = O.qp_backward(d["g"], r.v, r.mu, d["lower"], d["nominal"])
    assert np.array_equal(gl, d["g_lower"]) and np.array_equal(gn, d["g_nominal"])


def test_oracle_reproduces_lyap_fixture():
    d = _npz("oracle_lyap_step.npz")
    P = O.DynParams(**{k[2:]: d[k] for k in d if k.startswith("P_")})
    inp = O.StepInputs(x_feat=d["x_feat"], y=d["y"], h=d["h"], S=d["h"].shape[0] // d["x_feat"].shape[0],
                       mask1=d["mask1"], mask2=d["mask2"], lmask1=d["lmask1"], lmask2=d["lmask2"],
                       kappa=float(d["kappa"]))
    out = O.lyapunov_step(inp, P, O.DynConfig())
    assert np.float32(out.loss) == d["loss"] and np.float32(out.eff) == d["eff"]
    assert np.array_equal(out.V, d["V"]) and np.array_equal(out.Vdot, d["Vdot"])
    for k, v in out.grads.items():
        assert np.array_equal(v, d["grad_" + k]), k


@pytest.mark.gpu
def test_gpu_qp_matches_fixture():
    import torch
    from fiode_amd.barrier_projection import FastBarrierProjectionNoUpper
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device("cuda:0")
    d = _npz("oracle_qp.npz")
    lower = torch.from_numpy(d["lower"]).to(dev).requires_grad_(True)
    nominal = torch.from_numpy(d["nominal"]).to(dev).requires_grad_(True)
    v = FastBarrierProjectionNoUpper(30, 1e-4)(lower, nominal)
    v.backward(torch.from_numpy(d["g"]).to(dev))
    assert np.array_equal(v.detach().cpu().numpy(), d["v"])
    assert np.array_equal(lower.grad.cpu().numpy(), d["g_lower"])
    assert np.array_equal(nominal.grad.cpu().numpy(), d["g_nominal"])


@pytest.mark.gpu
def test_gpu_lyap_step_matches_fixture():
    """The fused step on the fixture's samples and masks.  V is a function of h only: bit-exact vs
    the fixture.  The fixture's MLP outputs ride on the oracle's float64 matmul, and the reference's
    QP active-set test is float32 rounding noise, so V-dot, the loss, eff and
    the gradients are checked against the oracle re-run on the fixture's inputs with the QP inputs
    pinned to the device's (lower, nominal): V-dot and eff bit-exact, the loss within 1e-6, the
    gradients within 2e-5 of each tensor's max."""
    import torch
    from fiode_amd import ops, _lib as L
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    dev = torch.device("cuda:0")
    d = _npz("oracle_lyap_step.npz")
    B, S = d["x_feat"].shape[0], d["h"].shape[0] // d["x_feat"].shape[0]
    w = {k: torch.from_numpy(np.ascontiguousarray(d["P_" + k])).to(dev) for k in ops.WEIGHT_KEYS}
    masks = torch.from_numpy(np.stack([d["mask1"], d["mask2"], d["lmask1"], d["lmask2"]])).to(dev)
    sc, gr, dbg = ops.lyap_step(torch.from_numpy(d["x_feat"]).to(dev), torch.from_numpy(d["y"]).to(dev), w,
                                ops.DynCfg(), sample_size=S, n_uniform=S, sampler=L.FIODE_SAMPLER_GIVEN,
                                dropout_mode=L.FIODE_DROPOUT_GIVEN, kappa=float(d["kappa"]),
                                h=torch.from_numpy(d["h"]).to(dev), masks=masks, debug=True)
    torch.cuda.synchronize()
    s = sc.cpu().numpy()
    db = {k: v.cpu().numpy() for k, v in dbg.items()}
    assert np.array_equal(db["V"], d["V"])
    P = O.DynParams(**{k: np.ascontiguousarray(d["P_" + k]) for k in ops.WEIGHT_KEYS})
    inp = O.StepInputs(x_feat=d["x_feat"], y=d["y"], h=d["h"], S=S, mask1=d["mask1"], mask2=d["mask2"],
                       lmask1=d["lmask1"], lmask2=d["lmask2"], kappa=float(d["kappa"]))
    free = O.lyapunov_step(inp, P, O.DynConfig())
    inp.qp_inputs = (db["qp_lower"], db["qp_nominal"][0])
    inp.qp_inputs_log = (db["qp_lower"], db["qp_nominal"][1])
    out = O.lyapunov_step(inp, P, O.DynConfig())
    assert np.array_equal(db["Vdot"], out.Vdot)
    assert int(s[1]) == int(out.eff)
    assert abs(s[0] - out.loss) <= 1e-6 * max(1.0, abs(out.loss)), (s[0], out.loss)
    for k in ("Q1", "b1", "Qx", "bx", "Q2", "b2", "Q3", "b3", "x_feat"):
        a, b = gr[k].cpu().numpy(), out.grads[k]
        assert np.abs(a - b).max() <= 2e-5 * max(1e-6, float(np.abs(b).max())), k
    # the unpinned oracle (the fixture's own values): same forward up to the MLP's rounding
    assert abs(free.loss - float(d["loss"])) <= 1e-6 * max(1.0, abs(float(d["loss"])))