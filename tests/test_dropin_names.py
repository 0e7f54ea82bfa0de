"""The drop-in surface the reference's drivers import (CPU).

Every name the reference's train.py and vis/render.py pull from the ``model`` package
resolves against this package, and the host-side helpers behind them behave as the
reference's (model/common.py:492-615, model/intrinsics.py).  Parity of the trajectory
helpers is unpinned upstream (the reference has no tests or fixtures); they are checked
through properties the reference's algorithms guarantee."""
import importlib
import os

import numpy as np
import pytest
import torch

# (reference file:line, module, names) -- the imports of the reference's drivers
DRIVER_IMPORTS = [
    ("train.py:15", "model", ["OfficialStaticNerf", "Renderer", "get_model", "CheckpointIO", "LearnPose",
                              "Learn_Distortion", "LearnFocal", "Trainer"]),   # mdl.* at train.py:50-158
    ("train.py:17", "model.common", ["backup", "mse2psnr"]),
    ("vis/render.py:11", "model.checkpoints", ["CheckpointIO"]),
    ("vis/render.py:12", "model.common", ["convert3x4_4x4", "interp_poses", "interp_poses_bspline",
                                          "generate_spiral_nerf"]),
    ("vis/render.py:13", "model.extracting_images", ["Extract_Images"]),
    ("vis/render.py:14", "model", ["OfficialStaticNerf", "Renderer", "get_model", "LearnPose", "CheckpointIO",
                                   "LearnFocal"]),                               # mdl.* at vis/render.py:36-79
    ("evaluation/eval.py:13,21", "model.common", ["compute_errors", "mse2psnr"]),
]


@pytest.mark.parametrize("where,module,names", DRIVER_IMPORTS, ids=[d[0] for d in DRIVER_IMPORTS])
def test_driver_imports_resolve(where, module, names):
    mod = importlib.import_module(module)
    missing = [n for n in names if not hasattr(mod, n)]
    assert not missing, f"{where}: {module} lacks {missing}"


def _poses(n, seed=0):
    from scipy.spatial.transform import Rotation
    g = np.random.default_rng(seed)
    c2w = np.tile(np.eye(4, dtype=np.float32), (n, 1, 1))
    c2w[:, :3, :3] = Rotation.from_rotvec(0.3 * g.standard_normal((n, 3))).as_matrix()
    c2w[:, :3, 3] = g.standard_normal((n, 3))
    return torch.tensor(c2w)


def test_interp_poses_hits_inputs_and_is_rigid():
    from model.common import interp_poses
    c2w = _poses(5)
    out = interp_poses(c2w, 5)                      # same count: slerp knots + identity interpolation
    assert out.shape == (5, 4, 4)
    assert torch.allclose(out, c2w, atol=1e-5)
    out = interp_poses(c2w, 17)
    R = out[:, :3, :3]
    assert torch.allclose(R @ R.transpose(1, 2), torch.eye(3).expand(17, 3, 3), atol=1e-5)
    assert torch.equal(out[:, 3], torch.tensor([0.0, 0, 0, 1]).expand(17, 4))


def test_interp_poses_bspline_clamped_ends():
    from model.common import interp_poses_bspline, scipy_bspline
    c2w = _poses(6, 1)
    times = np.arange(6, dtype=np.float64)
    out = interp_poses_bspline(c2w, 25, times, 3)
    assert out.shape == (25, 4, 4)
    # a clamped (open) B-spline starts and ends on its first / last control vertex
    assert torch.allclose(out[0, :3, 3], c2w[0, :3, 3], atol=1e-5)
    assert torch.allclose(out[-1, :3, 3], c2w[-1, :3, 3], atol=1e-5)
    assert torch.allclose(out[0, :3, :3], c2w[0, :3, :3], atol=1e-5)
    # degree 1 is the polyline through the vertices
    pts = np.array([[0.0, 0, 0], [1, 0, 0], [1, 2, 0]])
    lin = scipy_bspline(pts, n=5, degree=1)
    assert np.allclose(lin, [[0, 0, 0], [0.5, 0, 0], [1, 0, 0], [1, 1, 0], [1, 2, 0]])


def test_get_poses_at_times_blend():
    from model.common import get_poses_at_times, interp_t
    c2w = _poses(3, 2)
    times = np.array([0.0, 1.0, 2.0])
    t = interp_t(c2w[:, :3, 3:], times, np.array([0.25]))
    # the reference weights: (t - t0)/(t1 - t0) on the earlier camera, (t1 - t)/(t1 - t0) on the later
    assert torch.allclose(t[0], 0.25 * c2w[0, :3, 3:] + 0.75 * c2w[1, :3, 3:], atol=1e-6)
    out = get_poses_at_times(c2w, times, np.array([0.25, 1.5]))
    assert out.shape == (2, 4, 4)


def test_generate_spiral_nerf_shape_and_frames():
    from model.common import generate_spiral_nerf
    c2w = _poses(4, 3)
    hwf = np.tile(np.array([[188.0], [621.0], [362.5]]), (4, 1, 1))
    out = generate_spiral_nerf(c2w, np.array([2.0, 4.0]), 12, hwf)
    assert out.shape == (12, 3, 4)
    R = out[:, :3, :3].double()
    assert torch.allclose(R @ R.transpose(1, 2), torch.eye(3, dtype=torch.float64).expand(12, 3, 3), atol=1e-5)
    # the spiral circles the average camera: its centre is the mean of the path's centres
    # only approximately, but every camera stays within the 90th-percentile radii box
    assert torch.isfinite(out).all()


def test_mse2psnr_and_compute_errors():
    from model.common import compute_errors, mse2psnr
    assert mse2psnr(np.float32(0.01)) == pytest.approx(20.0)
    assert mse2psnr(np.float32(0.0)) == pytest.approx(100.0)         # clamp at 1e-10
    gt = np.array([1.0, 2.0, 4.0])
    e = compute_errors(gt, gt.copy())
    assert e[:4] == (0.0, 0.0, 0.0, 0.0) and e[4:] == (1.0, 1.0, 1.0)


def test_backup_copies_config_and_sources(tmp_path, monkeypatch):
    from model.common import backup
    work = tmp_path / "ref"
    (work / "model").mkdir(parents=True)
    (work / "dataloading").mkdir()
    (work / "configs").mkdir()
    (work / "train.py").write_text("# train")
    (work / "configs" / "default.yaml").write_text("a: 1")
    (work / "model" / "x.py").write_text("x = 1")
    (work / "dataloading" / "y.py").write_text("y = 1")
    cfg = work / "run.yaml"
    cfg.write_text("b: 2")
    monkeypatch.chdir(work)
    out = tmp_path / "out"
    backup(str(out), str(cfg))
    b = out / "backup"
    assert (b / "config.yaml").read_text() == "b: 2"
    assert (b / "train.py").exists() and (b / "default.yaml").exists()
    assert (b / "model" / "x.py").exists() and (b / "dataloading" / "y.py").exists()


def test_learn_focal_parameterisations():
    from model import LearnFocal
    f = LearnFocal(True, True, order=2, init_focal=400.0)
    assert torch.allclose(f(0), torch.tensor([400.0, 400.0]))
    f = LearnFocal(True, False, order=1, init_focal=[300.0, 310.0])
    assert torch.allclose(f(), torch.tensor([300.0, 310.0]))
    f = LearnFocal(False, False)
    assert torch.allclose(f(), torch.tensor([1.0, 1.0])) and not f.fx.requires_grad
    assert sorted(n for n, _ in LearnFocal(True, False).named_parameters()) == ["fx", "fy"]


def test_small_helpers():
    from model.common import convert2mip, normalize_tensor, skew_symmetric, taylor_A, taylor_B, taylor_C
    x = torch.tensor([0.3, 1.1])
    assert torch.allclose(taylor_A(x), torch.sin(x) / x, atol=1e-6)
    assert torch.allclose(taylor_B(x), (1 - torch.cos(x)) / x ** 2, atol=1e-6)
    assert torch.allclose(taylor_C(x), (x - torch.sin(x)) / x ** 3, atol=1e-5)
    w = torch.tensor([[1.0, 2.0, 3.0]])
    assert torch.allclose(skew_symmetric(w)[0] @ torch.tensor([4.0, 5, 6]), torch.linalg.cross(w[0], torch.tensor([4.0, 5, 6])))
    p = torch.tensor([[0.5, 0, 0], [3.0, 0, 0]])
    assert torch.allclose(convert2mip(p), torch.tensor([[0.5, 0, 0], [2 - 1 / 3, 0, 0]]))
    assert torch.allclose(normalize_tensor(torch.tensor([[3.0, 4.0]])), torch.tensor([[0.6, 0.8]]))
