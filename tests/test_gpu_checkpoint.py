"""Checkpoint / resume on the GPU (reference
model/checkpoints.py:29-120, train.py:62-76, 255-262): a HIP training run saved with
CheckpointIO and resumed in a fresh Trainer + HipAdam takes the next step bit for bit as the
uninterrupted run does, and a torch.optim.Adam state loaded into HipAdam steps as torch's
Adam does."""
import pytest
import torch

import model as mdl
from model.optim import HipAdam
from model.synthetic import make_cfg, vkitti_scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from model import _hip
    _hip.load_library()
    return torch.device("cuda", 0)


def _trainer(dev, c2w, cfg):
    torch.manual_seed(42)                                   # train.py:23-24
    net = mdl.OfficialStaticNerf(cfg)
    nn_model = mdl.get_model(mdl.Renderer(net, cfg["rendering"], device=dev), cfg, device=dev)
    opt = HipAdam(nn_model.parameters(), lr=cfg["training"]["learning_rate"])
    pose = mdl.LearnPose(1, False, False, cfg, init_c2w=c2w.unsqueeze(0).to(dev)).to(dev)
    return mdl.Trainer(nn_model, opt, cfg["training"], device=dev, pose_param_net=pose), nn_model, opt


@pytest.mark.parametrize("hidden,rays", [(256, 1024), (64, 256)])
def test_resume_is_bit_identical(dev, tmp_path, hidden, rays):
    """k HIP steps, CheckpointIO.save (model + optimizer + scalars, train.py:255-262), a fresh
    Trainer / HipAdam loading it (train.py:62-76), one more step: every parameter equals the
    uninterrupted run's bit for bit.  hidden 256 / 1024 rays runs the production path (the
    training chain, the native backward); hidden 64 the per-layer kernels."""
    cfg = make_cfg(hidden=hidden, S=128)
    cfg["training"]["n_training_points"] = rays
    cfg["training"]["pc_weight"] = [0.0, 0.0]
    cfg["training"]["rgb_s_weight"] = [0.0, 0.0]
    data, c2w = vkitti_scene(dev, 0)
    tr, m, opt = _trainer(dev, c2w, cfg)
    k = 3
    for i in range(k):
        tr.train_step(data, it=i, epoch=0, scheduling_start=0)
    io = mdl.CheckpointIO(str(tmp_path), model=m, optimizer=opt)
    io.save("model.pt", epoch_it=0, it=k, loss_val_best=1.0)
    rng = (torch.get_rng_state(), torch.cuda.get_rng_state(dev))
    tr.train_step(data, it=k, epoch=0, scheduling_start=0)
    torch.cuda.synchronize()
    want = {n: p.detach().clone() for n, p in m.named_parameters()}

    tr2, m2, opt2 = _trainer(dev, c2w, cfg)
    io2 = mdl.CheckpointIO(str(tmp_path), model=m2, optimizer=opt2)
    scalars = io2.load("model.pt", device=dev)
    assert scalars["it"] == k and scalars["epoch_it"] == 0
    torch.set_rng_state(rng[0])
    torch.cuda.set_rng_state(rng[1], dev)
    tr2.train_step(data, it=k, epoch=0, scheduling_start=0)
    torch.cuda.synchronize()
    for n, p in m2.named_parameters():
        assert torch.equal(p.detach(), want[n]), (n, (p.detach() - want[n]).abs().max().item())


def _cfg3_trainer(dev):
    """Config 3 (pose + distortion learned, pc + rgb_s losses) as bench.cfg3_setup builds it,
    with the three optimizers of train.py:59, :100, :118."""
    from model.synthetic import vkitti_pair_scene
    cfg = make_cfg(hidden=256, S=128)
    t = cfg["training"]
    t["n_training_points"] = 1024
    t["annealing_epochs"], t["scheduling_start"] = 2000, 0
    datas, c2w = vkitti_pair_scene(dev)
    torch.manual_seed(42)
    net = mdl.OfficialStaticNerf(cfg)
    nn_model = mdl.get_model(mdl.Renderer(net, cfg["rendering"], device=dev), cfg, device=dev)
    opt = HipAdam(nn_model.parameters(), lr=1e-3)
    pose = mdl.LearnPose(2, True, True, cfg, init_c2w=c2w.clone()).to(dev)
    distn = mdl.Learn_Distortion(2, True, True, cfg).to(dev)
    opt_pose = torch.optim.Adam(pose.parameters(), lr=5e-4, fused=True)
    opt_dist = torch.optim.Adam(distn.parameters(), lr=5e-4, fused=True)
    tr = mdl.Trainer(nn_model, opt, t, device=dev, optimizer_pose=opt_pose, pose_param_net=pose,
                     optimizer_distortion=opt_dist, distortion_net=distn)
    mods = {"model.pt": (nn_model, opt), "model_pose.pt": (pose, opt_pose),
            "model_distortion.pt": (distn, opt_dist)}
    return tr, datas, mods


def test_resume_cfg3_with_pose_and_distortion_files(dev, tmp_path):
    """Config 3 resume: model.pt, model_pose.pt and model_distortion.pt written as train.py:
    255-262 writes them (each module with its optimizer), loaded into a fresh config-3 trainer
    (train.py:62, :101, :119); the next step (the other camera) leaves the field, the learned
    poses and the distortion parameters bit for bit where the uninterrupted run leaves them."""
    tr, datas, mods = _cfg3_trainer(dev)
    k = 3
    for i in range(k):
        tr.train_step(datas[i % 2], it=i + 1, epoch=0, scheduling_start=0)
    for name, (m, o) in mods.items():
        mdl.CheckpointIO(str(tmp_path), model=m, optimizer=o).save(name, epoch_it=0, it=k)
    rng = (torch.get_rng_state(), torch.cuda.get_rng_state(dev))
    tr.train_step(datas[k % 2], it=k + 1, epoch=0, scheduling_start=0)
    torch.cuda.synchronize()
    want = {name: {n: p.detach().clone() for n, p in m.named_parameters()} for name, (m, _) in mods.items()}

    tr2, _, mods2 = _cfg3_trainer(dev)
    for name, (m, o) in mods2.items():
        scalars = mdl.CheckpointIO(str(tmp_path), model=m, optimizer=o).load(name, device=dev)
        assert scalars["it"] == k and scalars["epoch_it"] == 0
    torch.set_rng_state(rng[0])
    torch.cuda.set_rng_state(rng[1], dev)
    tr2.train_step(datas[k % 2], it=k + 1, epoch=0, scheduling_start=0)
    torch.cuda.synchronize()
    for name, (m, _) in mods2.items():
        assert want[name], name
        for n, p in m.named_parameters():
            assert torch.equal(p.detach(), want[name][n]), (name, n, (p.detach() - want[name][n]).abs().max().item())


def test_torch_adam_state_steps_like_torch_adam(dev):
    """A torch.optim.Adam state (the reference's optimizer, train.py:59) loaded into HipAdam:
    one HIP step from it equals torch Adam's step from the same state bit for bit."""
    cfg = make_cfg(hidden=256, S=128)
    torch.manual_seed(3)
    a = mdl.OfficialStaticNerf(cfg).to(dev)
    b = mdl.OfficialStaticNerf(cfg).to(dev)
    b.load_state_dict(a.state_dict())
    ref = torch.optim.Adam(a.parameters(), lr=1e-3)
    g = torch.Generator(device=dev).manual_seed(5)
    for _ in range(3):
        for p in a.parameters():
            p.grad = torch.randn(p.shape, device=dev, generator=g) * 1e-2
        ref.step()
    b.load_state_dict(a.state_dict())
    hip = HipAdam(b.parameters(), lr=1e-3)
    hip.load_state_dict(ref.state_dict())
    grads = [torch.randn(p.shape, device=dev, generator=g) * 1e-2 for p in a.parameters()]
    for p, gr in zip(a.parameters(), grads):
        p.grad = gr.clone()
    for p, gr in zip(b.parameters(), grads):
        p.grad = gr.clone()
    ref.step()
    hip.step()
    torch.cuda.synchronize()
    # k_adam is torch's foreach Adam op for op with torch's scalars (ABI 13): the parameters and
    # the state HipAdam now holds (step count, moments) equal torch Adam's bit for bit
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(pa.detach(), pb.detach()), (n, (pa.detach() - pb.detach()).abs().max().item())
    sa, sb = ref.state_dict()["state"], hip.state_dict()["state"]
    for i in sa:
        assert float(sa[i]["step"]) == float(sb[i]["step"]) == 4.0
        for key in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[i][key], sb[i][key]), (i, key, (sa[i][key] - sb[i][key]).abs().max().item())
