"""Full-frame rendering sharded over GPUs.

The render callers (training.py:103-165 render_visdata, extracting_images.py:40-133,
vis/render.py:86-121) render every pixel of a frame in eval mode.  Rays are
independent, so the frame is cut into G contiguous ray tiles of ceil(H*W / G) rays
(the last one padded), each rank renders its tile through the HIP path, and one RCCL
all-gather of (rgb, depth) -- 16 B per ray, ~1.9 MB for a 188x621 frame -- assembles
the frame on every rank.  No other collective is involved.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def tile_bounds(n_rays: int, rank: int, world: int) -> Tuple[int, int, int]:
    """(start, end, tile) of this rank's contiguous ray tile; tile = ceil(n / world)."""
    tile = (n_rays + world - 1) // world
    start = min(rank * tile, n_rays)
    return start, min(start + tile, n_rays), tile


def render_frame_sharded(render_tile: Callable[[int, int], Tuple[torch.Tensor, torch.Tensor]], n_rays: int,
                         device, group: Optional[dist.ProcessGroup] = None):
    """render_tile(start, end) -> (rgb [n,3], depth [n]) for rays [start, end).
    Returns (rgb [n_rays,3], depth [n_rays]) of the whole frame on every rank."""
    if not (dist.is_available() and dist.is_initialized()):
        rgb, depth = render_tile(0, n_rays)
        return rgb, depth
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    start, end, tile = tile_bounds(n_rays, rank, world)
    local = torch.zeros(tile, 4, device=device, dtype=torch.float32)
    if end > start:
        rgb, depth = render_tile(start, end)
        local[:end - start, :3] = rgb.reshape(-1, 3)
        local[:end - start, 3] = depth.reshape(-1)
    full = torch.empty(world * tile, 4, device=device, dtype=torch.float32)
    dist.all_gather_into_tensor(full, local, group=group)
    full = full[:n_rays]
    return full[:, :3].contiguous(), full[:, 3].contiguous()


def render_image(renderer, pixels, camera_mat, world_mat, scale_mat, depth_img=None, group=None):
    """Eval-mode render of every pixel (pixels [1, H*W, 2] in [-1,1], depth prior
    optional: ones as in extracting_images.py), sharded over the process group.
    Returns (rgb [H*W,3], depth [H*W]) with the reference's eval depth (z-depth,
    rendering.py:144-148)."""
    n = pixels.shape[1]
    dev = pixels.device
    depth_flat = None if depth_img is None else depth_img.reshape(1, -1, 1)

    def tile(start, end):
        d = None if depth_flat is None else depth_flat[:, start:end]
        if d is None:
            d = torch.ones(1, end - start, 1, device=dev)
        with torch.no_grad():
            out = renderer.nope_nerf(pixels[:, start:end], d, camera_mat, world_mat, scale_mat, add_noise=False,
                                     eval_=True)
        return out["rgb"].reshape(-1, 3), out["depth_pred"].reshape(-1)

    return render_frame_sharded(tile, n, dev, group)
