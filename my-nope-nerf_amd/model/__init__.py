"""MI355X-native drop-in for the reference's ``model`` package (model/__init__.py).

``sys.path.insert(0, '<repo>/my-nope-nerf_amd'); import model as mdl`` exposes the
names the reference's train.py and vis/render.py use (mdl.OfficialStaticNerf,
mdl.Renderer, mdl.get_model, mdl.LearnPose, mdl.Learn_Distortion, mdl.LearnFocal,
mdl.Trainer, mdl.CheckpointIO), backed by the nerf_hip kernels; the submodules
``model.common`` and ``model.extracting_images`` carry the names those drivers import
(tests/test_dropin_names.py).  Out of scope: Trainer_pose
(test-time pose refinement), DPT.
"""
from .checkpoints import CheckpointIO
from .config import get_model
from .distortions import Learn_Distortion
from .intrinsics import LearnFocal
from .network import nope_nerf
from .official_nerf import OfficialStaticNerf
from .poses import LearnPose
from .rendering import Renderer
from .training import Trainer

__all__ = ["CheckpointIO", "get_model", "Learn_Distortion", "LearnFocal", "nope_nerf", "OfficialStaticNerf", "LearnPose", "Renderer",
           "Trainer"]
