"""Checkpoint I/O interoperable with the reference (model/checkpoints.py:9-120).

Same class, method names and on-disk layout: ``save(filename, **scalars)`` writes one
``torch.save`` dict holding each registered module's ``state_dict()`` under its
registration name (train.py:62: ``model``, ``optimizer``; :101/:119: the pose and
distortion files) next to the scalars (``epoch_it``, ``it``, ``loss_val_best``,
``scheduling_start``, ``patient_count``, train.py:255-274).  ``load`` restores the
modules and returns the scalars.  Because the MI355X modules keep the reference
parameter names (``renderer.model.layers0.0.weight`` ...) and HipAdam reads and writes
``torch.optim.Adam``'s state_dict format, reference ``model.pt`` files load here and
files written here resume in the reference's train.py.

Differences: loading uses ``torch.load(..., weights_only=True)`` (tensors, numbers and
containers only -- a checkpoint is never executed), and URL loading
(checkpoints.py:92-101, ``model_zoo``) is not available offline.
"""
from __future__ import annotations

import datetime
import os
import shutil
import urllib.parse

import torch


def is_url(url) -> bool:
    """checkpoints.py:113-120."""
    return urllib.parse.urlparse(str(url)).scheme in ("http", "https")


class CheckpointIO:
    def __init__(self, checkpoint_dir="./chkpts", **kwargs):
        self.module_dict = kwargs
        self.checkpoint_dir = checkpoint_dir
        os.makedirs(checkpoint_dir, exist_ok=True)

    def register_modules(self, **kwargs):
        self.module_dict.update(kwargs)

    def _path(self, filename):
        return filename if os.path.isabs(filename) else os.path.join(self.checkpoint_dir, filename)

    def save(self, filename, **kwargs):
        """checkpoints.py:29-41: the registered state_dicts plus the given scalars."""
        outdict = dict(kwargs)
        for k, v in self.module_dict.items():
            outdict[k] = v.state_dict()
        torch.save(outdict, self._path(filename))

    def backup_model_best(self, filename, **kwargs):
        """checkpoints.py:43-52."""
        filename = self._path(filename)
        if os.path.exists(filename):
            backup_dir = os.path.join(self.checkpoint_dir, "backup_model_best")
            os.makedirs(backup_dir, exist_ok=True)
            ts = datetime.datetime.now().timestamp()
            shutil.copy(filename, os.path.join(backup_dir, "%s.pt" % ts))

    def load(self, filename, device=None, load_model_only=False):
        """checkpoints.py:54-65."""
        if is_url(filename):
            raise RuntimeError("CheckpointIO: loading from a URL needs network access (not available)")
        return self.load_file(filename, device, load_model_only)

    def load_file(self, filename, device=None, load_model_only=False):
        """checkpoints.py:67-90 (safe loader: weights_only=True)."""
        filename = self._path(filename)
        if not os.path.exists(filename):
            raise FileExistsError(filename)          # the reference raises this type too
        state_dict = torch.load(filename, map_location=device, weights_only=True)
        if load_model_only:
            state_dict = {"model": state_dict["model"]}
        return self.parse_state_dict(state_dict)

    def parse_state_dict(self, state_dict):
        """checkpoints.py:103-111: load the registered modules, return the rest."""
        for k, v in self.module_dict.items():
            if k in state_dict:
                v.load_state_dict(state_dict[k])
            else:
                print("Warning: Could not find %s in checkpoint!" % k)
        return {k: v for k, v in state_dict.items() if k not in self.module_dict}
