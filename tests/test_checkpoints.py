"""Checkpoint interoperability (model/checkpoints.py:9-120,
train.py:62-76, 255-274): the reference's key layout, CheckpointIO round trips, and the
torch.optim.Adam state format of HipAdam.  CPU only (no kernels run)."""
import os
import pickle

import pytest
import torch

import model as mdl
from model.optim import HipAdam
from oracle import nerf_oracle as orc
from tests.helpers import make_cfg


def _nope_nerf(hidden=64, seed=0):
    cfg = make_cfg(hidden=hidden, S=32)
    torch.manual_seed(seed)
    net = mdl.OfficialStaticNerf(cfg)
    rnd = mdl.Renderer(net, cfg["rendering"])
    return mdl.get_model(rnd, cfg), net, cfg


def test_state_dict_keys_match_reference_layout():
    """train.py:62 saves nope_nerf.state_dict(): renderer.model.<official_nerf keys>."""
    m, net, _ = _nope_nerf()
    ref_keys = {"renderer.model." + k for k in orc.OracleNerf(hidden_dim=64).state_dict()}
    assert set(m.state_dict()) == ref_keys
    shapes = {k: v.shape for k, v in orc.OracleNerf(hidden_dim=64).state_dict().items()}
    for k, v in net.state_dict().items():
        assert v.shape == shapes[k], k


def test_checkpoint_io_round_trip(tmp_path):
    m, net, _ = _nope_nerf(seed=1)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    io = mdl.CheckpointIO(str(tmp_path), model=m, optimizer=opt)
    io.save("model.pt", epoch_it=3, it=1200, loss_val_best=-25.5, scheduling_start=0, patient_count=2)
    assert os.path.exists(tmp_path / "model.pt")
    m2, _, _ = _nope_nerf(seed=2)
    opt2 = torch.optim.Adam(m2.parameters(), lr=1e-3)
    io2 = mdl.CheckpointIO(str(tmp_path), model=m2, optimizer=opt2)
    scalars = io2.load("model.pt")
    assert scalars == {"epoch_it": 3, "it": 1200, "loss_val_best": -25.5, "scheduling_start": 0,
                       "patient_count": 2}
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    s1, s2 = opt.state_dict()["state"], opt2.state_dict()["state"]
    assert s1.keys() == s2.keys() and all(torch.equal(s1[i]["exp_avg"], s2[i]["exp_avg"]) for i in s1)
    only = mdl.CheckpointIO(str(tmp_path), model=m2).load("model.pt", load_model_only=True)
    assert only == {}
    with pytest.raises(FileExistsError):
        io2.load("missing.pt")
    with pytest.raises(RuntimeError):
        io2.load("https://example.invalid/model.pt")


class _Payload:
    def __reduce__(self):
        return (print, ("executed",))


def test_checkpoint_loader_refuses_pickled_code(tmp_path):
    """Loading is weights_only: a file carrying an arbitrary object is refused."""
    path = tmp_path / "bad.pt"
    torch.save({"model": {}, "evil": _Payload()}, path)
    m, _, _ = _nope_nerf()
    with pytest.raises(pickle.UnpicklingError):
        mdl.CheckpointIO(str(tmp_path), model=m).load("bad.pt")


def test_hip_adam_state_dict_is_torch_adam_format():
    """A torch.optim.Adam state (3 steps) loads into HipAdam and comes back unchanged,
    and the group hyper-parameters travel; so reference optimizer states resume here."""
    m, _, _ = _nope_nerf(seed=3)
    ref_opt = torch.optim.Adam(m.parameters(), lr=5e-4, betas=(0.8, 0.99), eps=1e-7)
    for _ in range(3):
        for p in m.parameters():
            p.grad = torch.randn_like(p)
        ref_opt.step()
    sd = ref_opt.state_dict()
    m2, _, _ = _nope_nerf(seed=4)
    hip = HipAdam(m2.parameters(), lr=1e-3)
    hip.load_state_dict(sd)
    assert hip.param_groups[0]["lr"] == 5e-4 and tuple(hip.param_groups[0]["betas"]) == (0.8, 0.99)
    assert hip._hyper[0].item() == 3.0 and abs(hip._hyper[1].item() - 5e-4) < 1e-9
    back = hip.state_dict()
    assert back["state"].keys() == sd["state"].keys()
    for i, st in sd["state"].items():
        assert float(back["state"][i]["step"]) == float(st["step"])
        assert torch.equal(back["state"][i]["exp_avg"], st["exp_avg"])
        assert torch.equal(back["state"][i]["exp_avg_sq"], st["exp_avg_sq"])
    # and torch.optim.Adam accepts what HipAdam writes
    ref2 = torch.optim.Adam(m.parameters(), lr=1e-3)
    ref2.load_state_dict(back)
    assert ref2.param_groups[0]["lr"] == 5e-4
