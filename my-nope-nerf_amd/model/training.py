"""Trainer (drop-in for model/training.py:16-416).

Same constructor, ``train_step`` / ``render_visdata`` / ``compute_loss`` signatures and
loss-dict keys.  The step itself is the reference algorithm; what changes is where it
runs and what it waits for:
  * the render + its backward are the fused nerf_hip path (rendering.Renderer);
  * the step is free of device->host syncs: the depth-loss mask stays a dense weight,
    the distortion clamp is a ``torch.where``, the "any valid depth among the sampled
    rays" resampling loop (training.py:280-283) only runs when the image's valid-pixel
    count (known on the host from the data dict) does not already guarantee it;
  * with torch.distributed initialised (one process per GPU, RCCL), every rank renders
    its own rays and the NeRF / pose / distortion gradients are averaged by ONE
    all-reduce over a flat bucket before the optimiser steps.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.distributed as dist
from torch.nn import functional as F

from .common import arange_pixels, get_tensor_values, inv, project_to_cam, transform_to_world
from .rays import can_sample_on_device, depth_affine, mat4_mul
from .rays import sample_rays as sample_rays_dev
from .losses import Loss
from .pair import pair_losses


class Trainer(object):
    def __init__(self, model, optimizer, cfg, device=None, optimizer_pose=None, pose_param_net=None,
                 optimizer_focal=None, focal_net=None, optimizer_distortion=None, distortion_net=None, **kwargs):
        self.model = model
        self.optimizer = optimizer
        self.device = device
        self.optimizer_pose = optimizer_pose
        self.pose_param_net = pose_param_net
        self.focal_net = focal_net
        self.optimizer_focal = optimizer_focal
        self.distortion_net = distortion_net
        self.optimizer_distortion = optimizer_distortion

        self.n_training_points = cfg["n_training_points"]
        self.rendering_technique = cfg["type"]
        self.vis_geo = cfg.get("vis_geo", False)
        self.detach_gt_depth = cfg["detach_gt_depth"]
        self.pc_ratio = cfg["pc_ratio"]
        self.match_method = cfg["match_method"]
        self.shift_first = cfg["shift_first"]
        self.detach_ref_img = cfg["detach_ref_img"]
        self.scale_pcs = cfg["scale_pcs"]
        self.detach_rgbs_scale = cfg["detach_rgbs_scale"]
        self.vis_reprojection_every = cfg["vis_reprojection_every"]
        self.nearest_limit = cfg["nearest_limit"]
        self.annealing_epochs = cfg["annealing_epochs"]
        for w in ("pc_weight", "rgb_s_weight", "rgb_weight", "depth_weight", "weight_dist_2nd_loss",
                  "weight_dist_1st_loss", "depth_consistency_weight", "t_cycle_weight"):
            setattr(self, w, cfg[w])
        self.loss = Loss(cfg)
        self._pix_cache = {}
        # test hook: (ray_idx, noise) replaces the next draws of compute_loss (the
        # reference's randperm / torch.rand), so a step can be replayed on the oracle
        self.inject = None
        self.world_size = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world_size > 1 else 0
        # graph-capture mode (enable_graph_rng): the ray draw keys on a device step counter
        self.seed_counter = None
        # fixed gradient-bucket layout for the data-parallel all-reduce (bucket_params)
        self._bucket = None
        self._flat = None               # persistent all-reduce bucket (_bucket_buffer)
        self._offsets = []
        self._n_inplace = 0
        self._flag_cache = {}
        self._submodules = {}      # module -> its submodule list, for the per-step train-mode check
        self._comm_timer = None    # time_collectives: the all-reduces' (start, end) hipEvents / CPU seconds
        self._seed_one = None      # the backward's persistent d loss / d loss seed (train_step)

    def time_collectives(self, on=True):
        """Time every gradient all-reduce from now on (hipEvents on the launch stream around
        dist.all_reduce; perf_counter on CPU tensors) until switched off; collective_ms() sums
        them.  The event time includes the wait for the slowest rank.  Off: no events."""
        self._comm_timer = [] if on else None

    def collective_ms(self):
        """Milliseconds of the all-reduces timed since time_collectives(True) (synchronises on
        the last event)."""
        if not self._comm_timer:
            return 0.0
        total = 0.0
        for rec in self._comm_timer:
            if isinstance(rec, tuple):
                rec[1].synchronize()
                total += rec[0].elapsed_time(rec[1])
            else:
                total += 1e3 * rec
        return total

    def enable_graph_rng(self):
        """Make a step replayable from a captured hipGraph with fresh randomness: the ray
        sampler keys on a device counter it advances itself (stratified noise comes from
        torch.rand, whose Philox offsets graph replays already advance)."""
        self.seed_counter = torch.zeros(1, dtype=torch.int64, device=self.device)

    # ------------------------------------------------------------------ step
    def _modules_and_optims(self):
        mods = [(self.model, self.optimizer), (self.pose_param_net, self.optimizer_pose),
                (self.focal_net, self.optimizer_focal), (self.distortion_net, self.optimizer_distortion)]
        return [(m, o) for m, o in mods if m is not None]

    def train_step(self, data, it=None, epoch=None, scheduling_start=None, render_path=None):
        """training.py:70-100."""
        for m, o in self._modules_and_optims():
            subs = self._submodules.get(id(m))
            if subs is None or subs[0] is not m:     # the module walk, once per module (~50 us of host per step)
                subs = self._submodules[id(m)] = (m, list(m.modules()))
            if not all(sub.training for sub in subs[1]):   # train() walks and sets every submodule
                m.train()
            if o is not None:
                o.zero_grad()
        if self.world_size > 1 and self._flat is None:
            self._bucket_buffer(self.device)   # before the first backward: the field writes its gradients into it
        runner = self._field_runner() if self._n_inplace else None
        if runner is not None:
            runner.release_grad_buffer()       # the step's first field backward may take the bucket
        loss_dict = self.compute_loss(data, it=it, epoch=epoch, scheduling_start=scheduling_start,
                                      out_render_path=render_path)
        loss = loss_dict["loss"]
        # the backward's seed d loss / d loss = 1 from a persistent tensor: loss.backward() would
        # fill a fresh one with a kernel launch every step (the same value, so the same gradients;
        # 1.8700 vs 1.8762 ms per cfg2 step, profiles/r06/backward_seed_ab.txt)
        seed = self._seed_one
        if seed is None or seed.device != loss.device or seed.dtype != loss.dtype or seed.shape != loss.shape:
            seed = self._seed_one = torch.ones_like(loss)
        loss.backward(seed)
        if self.world_size > 1:
            self.allreduce_grads()
        for _, o in self._modules_and_optims():
            if o is not None:
                o.step()
        return loss_dict

    def bucket_params(self):
        """The fixed gradient-bucket layout: every trainable parameter of the NeRF, pose,
        focal and distortion modules, in module order.  It depends on the model alone, so
        every rank sends the same element count whatever gradients it produced."""
        if self._bucket is None:
            self._bucket = [p for m, _ in self._modules_and_optims() for p in m.parameters() if p.requires_grad]
        return self._bucket

    def _field_runner(self):
        """The HIP field runner whose backward produces the NeRF gradients (model.renderer.model)."""
        field = getattr(getattr(self.model, "renderer", None), "model", None)
        return field.hip_runner() if hasattr(field, "hip_runner") else None

    def _bucket_buffer(self, dev):
        """The persistent flat all-reduce bucket: [gradients of bucket_params() | one presence
        flag per parameter].  When the NeRF field's parameters lead the bucket in the runner's
        order, the runner's backward writes their gradients straight into it (FieldRunner.
        grad_buffer), so ~2.4 MB of the ~2.4 MB bucket is reduced in place -- no gather, no
        copy-back.  The pose / distortion gradients (a few floats) are copied in."""
        params = self.bucket_params()
        if self._flat is not None and self._flat.device == dev:
            return self._flat
        n = sum(p.numel() for p in params)
        self._flat = torch.zeros(n + len(params), device=dev, dtype=torch.float32)
        self._offsets, off = [], 0
        for p in params:
            self._offsets.append(off)
            off += p.numel()
        self._n_inplace = 0
        runner = self._field_runner()
        if runner is not None:
            pl = runner.param_list()
            if len(pl) <= len(params) and all(a is b for a, b in zip(pl, params)):
                runner.grad_buffer = self._flat[:sum(p.numel() for p in pl)]
                self._n_inplace = len(pl)
        return self._flat

    def allreduce_grads(self):
        """Average every gradient over the ranks with ONE flat all-reduce (RCCL on the GPU),
        in place on the persistent bucket (``_bucket_buffer``).

        The bucket has a fixed layout (``bucket_params``) plus one presence flag per
        parameter: a parameter without a gradient on this rank contributes zeros (DDP's
        convention), so the ranks always agree on the collective's size.  After the
        reduction every parameter some rank produced a gradient for holds the average over
        ``world_size`` as a view of the bucket; one no rank produced a gradient for stays
        ``None`` (torch Adam then skips it on every rank alike).  Only a rank that lacked a
        gradient reads the flags back (one host sync); the common all-present case stays
        sync-free."""
        params = self.bucket_params()
        if not params:
            return
        dev = next((p.grad.device for p in params if p.grad is not None), params[0].device)
        flat = self._bucket_buffer(dev)
        n = len(params)
        missing = tuple(p.grad is None for p in params)
        flags = self._flag_cache.get(missing)
        if flags is None:
            flags = torch.tensor([0.0 if m else 1.0 for m in missing], dtype=torch.float32, device=dev)
            self._flag_cache[missing] = flags
        views = [flat[o:o + p.numel()].view_as(p) for o, p in zip(self._offsets, params)]
        dst, src, zero = [], [], []
        for i, (p, v) in enumerate(zip(params, views)):
            g = p.grad
            if g is None:
                zero.append(v)
            elif not (i < self._n_inplace and g.data_ptr() == v.data_ptr() and g.is_contiguous()):
                dst.append(v)           # pose / distortion (or a field gradient not written in place)
                src.append(g)
        if dst:
            torch._foreach_copy_(dst, src)
        if zero:
            torch._foreach_zero_(zero)
        flat[-n:].copy_(flags)
        timer = self._comm_timer
        if timer is not None:
            if flat.is_cuda:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            else:
                t0 = time.perf_counter()
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        if timer is not None:
            if flat.is_cuda:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                timer.append((e0, e1))
            else:
                timer.append(time.perf_counter() - t0)
        flat[:-n].mul_(1.0 / self.world_size)
        present = flat[-n:].tolist() if any(missing) else None
        runner = self._field_runner() if self._n_inplace else None
        if runner is not None:
            runner.release_grad_buffer()
        for i, (p, v) in enumerate(zip(params, views)):
            if p.grad is None:
                if present[i] > 0:
                    p.grad = v
            elif p.grad.data_ptr() != v.data_ptr():
                p.grad = v              # the averaged gradient, as a view of the bucket (no copy back)

    # ------------------------------------------------------------------ data
    def process_data_dict(self, data):
        """training.py:166-183."""
        dev = self.device
        img = data.get("img").to(dev, non_blocking=True)
        img_idx = data.get("img.idx")
        depth = data.get("img.dpt")
        if depth is None:
            depth = data.get("img.depth")
        depth = depth.to(dev, non_blocking=True).unsqueeze(1)
        depth_mask = data.get("img.depth_mask")
        camera_mat = data.get("img.camera_mat").to(dev, non_blocking=True)
        scale_mat = data.get("img.scale_mat").to(dev, non_blocking=True)
        pose_gt = data.get("img.pose_gt").to(dev, non_blocking=True)
        return (img, depth, camera_mat, scale_mat, img_idx, pose_gt, depth_mask)

    def process_data_reference(self, data):
        dev = self.device
        ref_imgs = data.get("img.ref_imgs").to(dev, non_blocking=True)
        ref_depths = data.get("img.ref_dpts")
        if ref_depths is None:
            ref_depths = data.get("img.ref_depths")
        ref_depths = ref_depths.to(dev, non_blocking=True).unsqueeze(1)
        ref_pose_gt = data.get("img.ref_pose_gt").to(dev, non_blocking=True)
        return (ref_imgs, ref_depths, data.get("img.ref_idxs"), ref_pose_gt)

    def anneal(self, start_weight, end_weight, anneal_start_epoch, anneal_epoches, current):
        """training.py:204-212."""
        if current <= anneal_start_epoch:
            return start_weight
        if current >= anneal_start_epoch + anneal_epoches:
            return end_weight
        return start_weight + (end_weight - start_weight) * (current - anneal_start_epoch) / anneal_epoches

    def _pixels(self, h, w, device):
        key = (h, w, str(device))
        if key not in self._pix_cache:
            self._pix_cache[key] = arange_pixels((h, w), 1, device=device)[1]
        return self._pix_cache[key]

    def sample_rays(self, n_pix, depth_mask, need_valid, img=None, hw=None):
        """training.py:277-283 plus the colour / pixel gathers of :284-287: a random subset
        of R pixels, resampled while none of them has a valid depth.  Returns (ray_idx,
        pixels [B,R,2], rgb_gt [B,R,3]).

        On the device one HIP launch draws the subset and gathers both (rays.sample_rays;
        ``randperm`` sorts n_pix keys to keep R of them).  The validity check is a
        device->host sync per step in the reference; here it runs only when an all-invalid
        draw is plausible: with n_invalid of n_pix pixels invalid that probability is
        <= (n_invalid / n_pix) ** R, computed on the host from the data dict's CPU mask
        (5 % holes at 1024 rays: 1e-1332)."""
        dev = self.device
        R = self.n_training_points
        h, w = hw
        B = img.shape[0]
        on_dev = img.is_cuda and B == 1 and can_sample_on_device(n_pix, R)

        def draw():
            if on_dev:
                if self.seed_counter is not None:
                    # graph-capture mode: a fixed per-rank key and a device step counter, so a
                    # replayed step draws new rays without a host-side seed
                    seed = (0x2545F4914F6CDD1D + self.rank * 0x632BE59BD9B4E019) & 0xFFFFFFFFFFFFFFFF
                    return sample_rays_dev(n_pix, R, w, h, img[0], seed=seed, seed_counter=self.seed_counter)
                # host-generator seed (reproducible under torch.manual_seed), decorrelated per
                # rank so data-parallel ranks render different rays
                seed = int(torch.randint(0, 2 ** 62, (1,)).item()) + self.rank * 0x632BE59BD9B4E019
                return sample_rays_dev(n_pix, R, w, h, img[0], seed=seed & 0xFFFFFFFFFFFFFFFF)
            ray_idx = torch.randperm(n_pix, device=dev)[:R]
            rgb_gt = img.view(B, 3, n_pix).permute(0, 2, 1)[:, ray_idx]
            return ray_idx, self._pixels(h, w, dev)[:, ray_idx], rgb_gt

        ray_idx, p, rgb_gt = draw()
        if need_valid and depth_mask is not None:
            if depth_mask.is_cuda:
                risky = True
            else:
                n_invalid = n_pix - int(depth_mask.sum())
                risky = n_invalid > 0 and (n_invalid / n_pix) ** R > 1e-9
            if risky and self.seed_counter is not None:
                # graph-capture mode: the resample-until-valid loop needs the host to look at
                # the draw (a sync inside capture) and a replay could never re-decide it
                raise RuntimeError(
                    "Trainer: graph-capture mode (enable_graph_rng) needs a depth mask on the host whose "
                    "valid-pixel count rules out an all-invalid draw (training.py:280-283 resampling)")
            if risky:
                m = depth_mask.flatten().to(dev)
                while not m[ray_idx].any():
                    ray_idx, p, rgb_gt = draw()
        return ray_idx, p, rgb_gt

    # ------------------------------------------------------------------ loss
    def compute_loss(self, data, eval_mode=False, it=None, epoch=None, scheduling_start=None,
                     out_render_path=None):
        """training.py:214-416."""
        names = ["rgb_weight", "depth_weight", "pc_weight", "rgb_s_weight", "depth_consistency_weight",
                 "weight_dist_2nd_loss", "weight_dist_1st_loss", "t_cycle_weight"]
        weights = {n: self.anneal(getattr(self, n)[0], getattr(self, n)[1], scheduling_start,
                                  self.annealing_epochs, epoch) for n in names}
        rgb_loss_type = "l1" if epoch < self.annealing_epochs + scheduling_start else "l2"
        render_model = weights["rgb_weight"] != 0.0 or weights["depth_weight"] != 0.0
        use_ref_imgs = (weights["pc_weight"] != 0.0 or weights["rgb_s_weight"] != 0.0
                        or weights["t_cycle_weight"] != 0.0)
        nl = self.nearest_limit
        img, depth_input, camera_mat_gt, scale_mat, img_idx, pose_gt, depth_mask = self.process_data_dict(data)
        if use_ref_imgs:
            ref_img, depth_ref, ref_idx, ref_pose_gt = self.process_data_reference(data)
        dev = self.device
        B, _, h, w = img.shape
        _, _, h_depth, w_depth = depth_input.shape
        kwargs = {"weights": weights, "rgb_loss_type": rgb_loss_type}
        if self.pose_param_net is not None:
            kwargs["t_list"] = self.pose_param_net.get_t()
        # the ground-truth relative pose only feeds the t-cycle term (losses.py:161-162)
        world_mat_gt = inv(pose_gt).unsqueeze(0) if (use_ref_imgs and weights["t_cycle_weight"] != 0.0) else None
        num_cams = self.pose_param_net.num_cams if self.pose_param_net is not None else None
        c2w = self.pose_param_net(img_idx) if self.pose_param_net is not None else pose_gt.reshape(4, 4)
        world_mat = inv(c2w).unsqueeze(0)
        scale_input = shift_input = None
        affine_in = None
        if self.distortion_net is not None:
            scale_input, shift_input = self.distortion_net(img_idx)
            if depth_input.is_cuda and tuple(depth_input.shape[-2:]) == (h, w):
                # training.py:259-264's elementwise scale / shift commutes with the gathers that
                # consume the prior (the ray gather of network.py:24-26, the nearest resize of
                # training.py:346-347): apply it after them, to 1024 + 7285 values instead of the
                # H x W map, so its backward never materialises a dense gradient of the map
                affine_in = self._affine(scale_input, shift_input)
            elif self.shift_first:
                depth_input = (depth_input + shift_input) * scale_input
            else:
                depth_input = depth_input * scale_input + shift_input
        if self.optimizer_focal:
            fxfy = self.focal_net(0)
            pad = torch.zeros(4, device=dev)
            one = torch.ones(1, device=dev)
            camera_mat = torch.cat([fxfy[0:1], pad, -fxfy[1:2], pad, -one, pad, one]).view(1, 4, 4)
        else:
            camera_mat = camera_mat_gt

        extra = {}
        if self.inject is not None:
            ray_idx, noise = self.inject
            ray_idx = ray_idx.to(dev)
            rgb_gt = img.view(B, 3, h * w).permute(0, 2, 1)[:, ray_idx]
            p = self._pixels(h, w, dev)[:, ray_idx]
            extra["noise"] = noise.to(dev)
        else:
            ray_idx, p, rgb_gt = self.sample_rays(h * w, depth_mask, data.get("img.dpt") is None, img=img,
                                                  hw=(h, w))

        rendered_rgb = rendered_depth = gt_depth = dmask = None
        if render_model:
            out = self.model(p, ray_idx, camera_mat, world_mat, scale_mat, self.rendering_technique, it=it,
                             eval_mode=eval_mode, depth_img=depth_input, img_size=(h, w), depth_affine=affine_in,
                             dense_depth=not eval_mode, **extra)
            rendered_rgb, rendered_depth, gt_depth = out["rgb"], out["depth_pred"], out["depth_gt"]
            dmask = out.get("depth_mask")

        if use_ref_imgs:
            kwargs.update(self._reference_terms(weights, img, ref_img, depth_input, depth_ref, img_idx, ref_idx,
                                                ref_pose_gt, world_mat, world_mat_gt, camera_mat, scale_input, affine_in,
                                                num_cams, h_depth, w_depth, nl, it, out_render_path))
        if render_model and self.detach_gt_depth:
            gt_depth = gt_depth.detach()
        loss_dict = self.loss(rendered_rgb, rgb_gt, rendered_depth, gt_depth, depth_mask=dmask, **kwargs)
        if self.optimizer_focal:
            loss_dict["focalx"] = fxfy[0] / camera_mat_gt[0, 0, 0]
            loss_dict["focaly"] = fxfy[1] / camera_mat_gt[0, 1, 1]
        loss_dict["scale"] = scale_input
        loss_dict["shift"] = shift_input
        return loss_dict

    def _affine(self, scale, shift):
        """The depth-prior distortion of training.py:259-264 / :325-329 as a function of the
        (gathered) prior values, optionally followed by the nearest_limit clamp (one HIP launch
        each way, rays.depth_affine)."""
        return lambda d, lo=float("-inf"): depth_affine(d, scale, shift, self.shift_first, lo)

    def _reference_terms(self, weights, img, ref_img, depth_input, depth_ref, img_idx, ref_idx, ref_pose_gt,
                         world_mat, world_mat_gt, camera_mat, scale_input, affine_in, num_cams, h_depth, w_depth,
                         nl, it,
                         out_render_path):
        """training.py:305-405: point clouds of the image pair, relative pose, reprojection."""
        B = img.shape[0]
        want_gt = world_mat_gt is not None
        ref_Rt_gt = inv(ref_pose_gt).unsqueeze(0) if want_gt else None
        c2w_ref = self.pose_param_net(ref_idx)
        scale_ref = shift_ref = None
        affine_ref = None
        if self.distortion_net is not None:
            scale_ref, shift_ref = self.distortion_net(ref_idx)
            if self.detach_ref_img:
                scale_ref, shift_ref = scale_ref.detach(), shift_ref.detach()
            if affine_in is not None:
                affine_ref = self._affine(scale_ref, shift_ref)     # after the resize (see compute_loss)
            elif self.shift_first:
                depth_ref = scale_ref * (depth_ref + shift_ref)
            else:
                depth_ref = scale_ref * depth_ref + shift_ref
        if self.detach_ref_img:
            c2w_ref = c2w_ref.detach()
            depth_ref = depth_ref.detach()
        ref_Rt = inv(c2w_ref).unsqueeze(0)
        if int(img_idx) < num_cams - 1:
            d1, d2, img1, img2 = depth_input, depth_ref, img, ref_img
            a1, a2 = affine_in, affine_ref
            Rt_rel_12 = mat4_mul(ref_Rt, inv(world_mat))
            Rt_rel_12_gt = mat4_mul(ref_Rt_gt, inv(world_mat_gt)) if want_gt else None
            scale1 = scale_input
        else:
            d1, d2, img1, img2 = depth_ref, depth_input, ref_img, img
            a1, a2 = affine_ref, affine_in
            Rt_rel_12 = mat4_mul(world_mat, inv(ref_Rt))
            Rt_rel_12_gt = mat4_mul(world_mat_gt, inv(ref_Rt_gt)) if want_gt else None
            scale1 = scale_ref
        res = (int(h_depth / self.pc_ratio), int(w_depth / self.pc_ratio))
        d1 = F.interpolate(d1, res, mode="nearest")
        d2 = F.interpolate(d2, res, mode="nearest")
        if a1 is not None:                                             # distortion, then d[d < nl] = nl
            d1, d2 = a1(d1, nl), a2(d2, nl)
        else:
            d1, d2 = d1.clamp_min(nl), d2.clamp_min(nl)
        if (img.is_cuda and not camera_mat.requires_grad and not self.loss.cfg.get("with_ssim", False)
                and self.match_method == "dense"):
            # pair.hip: point clouds, chamfer and reprojection terms in 4 + 4 launches
            want_rgbs = weights["rgb_s_weight"] != 0.0
            i1 = F.interpolate(img1, res, mode="bilinear") if want_rgbs else None
            i2 = F.interpolate(img2, res, mode="bilinear") if want_rgbs else None
            s = scale1 if (self.scale_pcs and scale1 is not None) else None
            l_pc, l_rgbs = pair_losses(d1, d2, camera_mat, Rt_rel_12, s, i1, i2, res, nl, self.detach_rgbs_scale)
            return {"pair_losses": (l_pc, l_rgbs), "sample_resolution": res, "rt_12": Rt_rel_12,
                    "rt_12_gt": Rt_rel_12_gt}
        R_rel_12, t_rel_12 = Rt_rel_12[:, :3, :3], Rt_rel_12[:, :3, 3]
        pixel_locations, p_pc = arange_pixels(resolution=res, device=img.device)
        pc1 = transform_to_world(p_pc, d1.view(1, -1, 1), camera_mat)
        pc2 = transform_to_world(p_pc, d2.view(1, -1, 1), camera_mat)
        out = {}
        if weights["rgb_s_weight"] != 0.0:
            i1 = F.interpolate(img1, res, mode="bilinear")
            i2 = F.interpolate(img2, res, mode="bilinear")
            rgb_pc1 = get_tensor_values(i1, p_pc, mode="bilinear", scale=False, detach=False, detach_p=False,
                                        align_corners=True)
            src = pc1.detach().clone() if self.detach_rgbs_scale else pc1
            pc1_rot = src @ R_rel_12.transpose(1, 2) + t_rel_12
            bad = (-pc1_rot[:, :, 2:] < nl).expand_as(pc1_rot)
            pc1_rot = torch.where(bad, torch.full_like(pc1_rot, nl), pc1_rot)
            p_reproj, valid = project_to_cam(pc1_rot, camera_mat)
            rgb_proj = get_tensor_values(i2, p_reproj, mode="bilinear", scale=False, detach=False,
                                         detach_p=False, align_corners=True)
            out["rgb_pc1"] = rgb_pc1.view(B, res[0], res[1], 3)
            out["rgb_pc1_proj"] = rgb_proj.view(B, res[0], res[1], 3)
            out["valid_points"] = valid.view(B, res[0], res[1], 1)
        if self.scale_pcs and scale1 is not None:
            pc1 = pc1 / scale1
            pc2 = pc2 / scale1
        out["X"] = pc1 @ R_rel_12.transpose(1, 2) + t_rel_12
        out["Y"] = pc2
        out["sample_resolution"] = res
        out["p_2d"] = pixel_locations
        out["rt_12"] = Rt_rel_12
        out["rt_12_gt"] = Rt_rel_12_gt
        return out

    # ------------------------------------------------------------------ render
    def render_visdata(self, data, resolution, it, out_render_path):
        """training.py:103-165: colour + depth PNGs at ``resolution`` and, with ``vis_geo``,
        the Phong-shaded occupancy surface (``%04d_geo.png``, Renderer.phong_renderer)."""
        from PIL import Image
        img, depth_input, camera_mat, scale_mat, img_idx, *_ = self.process_data_dict(data)
        h, w = resolution
        c2w = self.pose_param_net(img_idx)
        world_mat = inv(c2w).unsqueeze(0)
        if self.optimizer_focal:
            fxfy = self.focal_net(0)
            camera_mat = torch.tensor([[[fxfy[0], 0, 0, 0], [0, -fxfy[1], 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]]],
                                      device=self.device)
        pixels = self._pixels(h, w, self.device)
        p_idx = torch.arange(h * w, device=self.device)
        with torch.no_grad():
            out = self.model(pixels, p_idx, camera_mat, world_mat, scale_mat, self.rendering_technique,
                             add_noise=False, eval_mode=True, it=it, depth_img=depth_input, img_size=(h, w))
            rgb = out["rgb"].view(h, w, 3).cpu().numpy()
            depth = out["depth_pred"].view(h, w).cpu().numpy()
        img_out = (rgb * 255).astype(np.uint8)
        if out_render_path:
            dimg = np.clip(255.0 / depth.max() * (depth - depth.min()), 0, 255).astype(np.uint8)
            Image.fromarray(dimg).save(os.path.join(out_render_path, "%04d_depth.png" % int(img_idx)))
            Image.fromarray(img_out).convert("RGB").save(os.path.join(out_render_path, "%04d_img.png" % int(img_idx)))
        if self.vis_geo:                                       # training.py:144-163
            with torch.no_grad():
                geo = torch.cat([self.model(pix_i, None, camera_mat, world_mat, scale_mat, "phong_renderer",
                                            add_noise=False, eval_mode=True, it=it, depth_img=depth_input,
                                            img_size=(h, w))["rgb"] for pix_i in torch.split(pixels, 1024, dim=1)],
                                dim=1)
                img_out = (geo.view(h, w, 3).cpu().numpy() * 255).astype(np.uint8)
            if out_render_path:
                Image.fromarray(img_out).convert("RGB").save(os.path.join(out_render_path, "%04d_geo.png" % int(img_idx)))
        return img_out
