"""Checkpoint compatibility: Lightning-layout .ckpt files with the
reference's state_dict keys (classification.py:44-83, init_coordinates.py:38-44, models.py:195-199)
round-trip through save_checkpoint / load_from_checkpoint, read with weights_only=True."""
import pathlib
import sys

import pytest
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "fi-ode_amd"))

from bench import build_module  # noqa: E402
from fiode_amd import checkpoint as C  # noqa: E402

# keys the reference's LyapunovLearning state_dict holds for the dynamics / init / IVP (read from
# classification.py:44-83 -- CayleyLinear weight/bias/alpha --, init_coordinates.py:38-44, models.py:195-199)
REF_KEYS = [f"model.dyn_fun.{l}.{p}" for l in ("hidden_to_mlp", "mlp_to_mlp", "mlp_to_hidden", "U_x")
            for p in ("weight", "bias", "alpha")] + ["model.init_coordinates.h0_0", "model.ts"]


def _mod(seed):
    return build_module(torch.device("cpu"), seed=seed)


def test_reference_keys_present():
    sd = _mod(0).state_dict()
    for k in REF_KEYS:
        assert k in sd, k
    assert "model.dyn_fun.static_state" not in sd        # None buffer, as in the reference


def test_roundtrip_lightning_layout(tmp_path):
    a, b = _mod(0), _mod(1)
    opt = torch.optim.Adam(a.parameters(), lr=1e-3)
    path = tmp_path / "model.ckpt"
    C.save_checkpoint(a, path, epoch=37, global_step=1234, optimizers=[opt])
    ck = torch.load(path, weights_only=True)              # plain containers only
    assert set(ck) >= {"epoch", "global_step", "pytorch-lightning_version", "state_dict", "optimizer_states"}
    assert any(not torch.equal(a.state_dict()[k], b.state_dict()[k]) for k in REF_KEYS[:3])
    info = C.load_from_checkpoint(b, path, strict=True)
    assert info["missing_keys"] == [] and info["unexpected_keys"] == []
    assert info["epoch"] == 37 and info["global_step"] == 1234
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), k


def test_nonstrict_partial_and_shape_errors(tmp_path):
    a = _mod(0)
    sd = {k: v for k, v in a.state_dict().items() if k.startswith("model.dyn_fun.")}
    sd["model.dyn_fun.extra_buffer"] = torch.zeros(3)
    path = tmp_path / "partial.ckpt"
    torch.save({"state_dict": sd, "epoch": 5, "global_step": 10}, path)
    b = _mod(2)
    info = C.load_from_checkpoint(b, path, strict=False)    # hydra_conf_load_from_checkpoint_nonstrict
    assert "model.dyn_fun.extra_buffer" in info["unexpected_keys"]
    assert all(not k.startswith("model.dyn_fun.") for k in info["missing_keys"])
    assert torch.equal(b.dyn_fun.mlp_to_mlp.weight, a.dyn_fun.mlp_to_mlp.weight)
    with pytest.raises(RuntimeError):
        C.load_from_checkpoint(_mod(2), path, strict=True)
    sd["model.dyn_fun.mlp_to_mlp.weight"] = torch.zeros(3, 3)
    torch.save({"state_dict": sd}, path)
    with pytest.raises(C.CheckpointError, match="shape mismatch"):
        C.load_from_checkpoint(_mod(2), path)


def test_refuses_pickled_objects(tmp_path):
    import argparse
    path = tmp_path / "evil.ckpt"        # an arbitrary (non-allow-listed) object needs unpickling
    torch.save({"state_dict": {}, "hyper_parameters": argparse.Namespace(x=1)}, path)
    with pytest.raises(C.CheckpointError, match="weights_only"):
        C.read_checkpoint(path)


def test_resume_restores_optimizer_and_counters(tmp_path):
    a = _mod(0)
    opt = torch.optim.Adam(a.parameters(), lr=1e-3)
    for p in a.parameters():
        p.grad = torch.ones_like(p)
    opt.step()
    path = tmp_path / "resume.ckpt"
    C.save_checkpoint(a, path, epoch=21, global_step=99, optimizers=[opt])
    b = _mod(3)
    opt_b = torch.optim.Adam(b.parameters(), lr=1e-3)
    C.restore_training_state(b, path, optimizers=[opt_b])
    assert b.current_epoch == 21 and b.global_step == 99
    sa, sb = opt.state_dict()["state"], opt_b.state_dict()["state"]
    assert sa.keys() == sb.keys()
    for i in sa:
        assert torch.equal(sa[i]["exp_avg"], sb[i]["exp_avg"])


def test_classmethod_load(tmp_path):
    import bench
    a = _mod(0)
    path = tmp_path / "m.ckpt"
    C.save_checkpoint(a, path)
    b = _mod(4)
    cls = type(b)
    # the classmethod builds the module from the config kwargs, as Lightning does
    kw = dict(order=1, h_sample_size=bench.H_SAMPLE, h_dist_lim=15.0, sampler=b.sampler,
              sampler_scheduler=b.sampler_scheduler, dynamics=b.dyn_fun, init_fun=b.model.init_coordinates,
              lya_cand=b.lya_cand, t_max=1.0, simplex=True)
    c = cls.load_from_checkpoint(path, strict=True, **kw)
    assert torch.equal(c.dyn_fun.U_x.alpha, a.dyn_fun.U_x.alpha)


def test_sgd_fix_backbone_optimizes_dynamics_only():
    """pl_modules.py:110-118: with opt_name='SGD', fix_backbone=True optimizes the dynamics'
    parameters only; False optimizes every parameter."""
    m = _mod(0)
    m.opt_name, m.momentum = "SGD", 0.9
    dyn_ids = {id(p) for p in m.dyn_fun.parameters()}
    m.fix_backbone = True
    opt = m.configure_optimizers()[0]
    opt = opt[0] if isinstance(opt, list) else opt
    got = {id(p) for g in opt.param_groups for p in g["params"]}
    assert got == dyn_ids
    m.fix_backbone = False
    opt = m.configure_optimizers()[0]
    opt = opt[0] if isinstance(opt, list) else opt
    assert {id(p) for g in opt.param_groups for p in g["params"]} == {id(p) for p in m.parameters()}
