"""Multi-GPU image-tile rendering: one process per GPU, torch.distributed over RCCL.

SURVEY §8e: pixels are independent and every RNG seed is a pure function of the global
pixel coordinate, so the image shards with no data-path exchange.  Bands of
RT_STRIPE_ROWS rows are dealt round-robin (band b -> rank b % world), which balances the
sky/ground cost between ranks.  Each rank renders its bands into a compact local buffer
(rt_render_stripes); the only collective is ONE gather of the finished tiles to rank 0
(RCCL over xGMI), followed by the de-interleave kernel on the root.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .compute_shader import ComputeShaderPipeline, stripe_local_rows


def padded_rows(height: int, world: int) -> int:
    """Rows of every rank's send buffer (rank 0 holds the most bands)."""
    return stripe_local_rows(height, 0, world)


def gather_stripes(local: torch.Tensor, world: int, rank: int, dst: int = 0,
                   group=None, out: torch.Tensor | None = None) -> torch.Tensor | None:
    """Gather equal-shaped (rows0, W, 4) tiles to `dst` as one (world*rows0, W, 4) tensor
    (into `out`, shaped (world, rows0, W, 4), when given).

    One collective (dist.gather; RCCL on GPU, gloo on CPU — device tensors under gloo are
    staged through host memory, which gloo's gather requires)."""
    if world == 1:
        return local
    if local.is_cuda and dist.get_backend(group) == "gloo":
        host = gather_stripes(local.cpu(), world, rank, dst, group)
        if host is None:
            return None
        if out is None:
            return host.to(local.device)
        out.copy_(host.reshape(out.shape))
        return out.reshape((world * local.shape[0],) + tuple(local.shape[1:]))
    if rank == dst:
        if out is None:
            out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype,
                              device=local.device)
        dist.gather(local, gather_list=list(out.unbind(0)), dst=dst, group=group)
        return out.reshape((world * local.shape[0],) + tuple(local.shape[1:]))
    dist.gather(local, gather_list=None, dst=dst, group=group)
    return None


class StripeRenderer:
    """One rank's share of a width x height progressive render."""

    def __init__(self, pipeline: ComputeShaderPipeline, width: int, height: int, rank: int,
                 world: int):
        self.pipe, self.width, self.height = pipeline, width, height
        self.rank, self.world = rank, world
        self.rows = stripe_local_rows(height, rank, world)
        self.rows0 = padded_rows(height, world)
        # ping-pong local accumulators, padded to rows0 so the gather is uniform
        self.buf = [pipeline.new_image(width, self.rows0), pipeline.new_image(width, self.rows0)]
        self.cur = 0
        # the root's gather and output buffers, allocated up front (finish() then runs only
        # the collective and the de-interleave kernel)
        self._gathered = self._image = None
        if world > 1 and rank == 0:
            dev = self.buf[0].device
            self._gathered = torch.empty((world, self.rows0, width, 4), dtype=torch.float32,
                                         device=dev)
            self._image = torch.empty((height, width, 4), dtype=torch.float32, device=dev)

    def frame(self, camera, spheres, seeds) -> None:
        """One progressive `update` (or len(seeds) fused frames) over this rank's bands."""
        src, dst = self.buf[self.cur], self.buf[1 - self.cur]
        if self.rows:
            self.pipe.render_stripes(src, dst, self.width, self.height, self.rank, self.world,
                                     camera, spheres, seeds)
        self.cur = 1 - self.cur

    def frames(self, camera, spheres, seeds) -> None:
        """len(seeds) progressive frames, one `update` dispatch each, from a single call."""
        if self.rows:
            a, b = self.buf[self.cur], self.buf[1 - self.cur]
            newest = self.pipe.update_frames(a, b, self.width, self.height, camera, spheres,
                                             seeds, self.rank, self.world)
            if newest == 1:
                self.cur = 1 - self.cur
        elif len(seeds) % 2:
            self.cur = 1 - self.cur

    def frames_per_launch(self, camera) -> int:
        """Frames rt_update_frames fuses per launch for this pipeline and camera."""
        return self.pipe.frames_per_launch(camera)

    @property
    def local(self) -> torch.Tensor:
        return self.buf[self.cur]

    def finish(self, dst: int = 0, group=None) -> torch.Tensor | None:
        """Gather the finished tiles; returns the full image on `dst`, None elsewhere."""
        if self.world == 1:
            return self.local[: self.height]
        pre = dst == 0 and self._gathered is not None
        gathered = gather_stripes(self.local, self.world, self.rank, dst, group,
                                  out=self._gathered if pre else None)
        if gathered is None:
            return None
        # (the de-interleave writes every pixel: no zero fill needed)
        out = self._image if pre else torch.empty((self.height, self.width, 4),
                                                  dtype=torch.float32, device=gathered.device)
        self.pipe.deinterleave(gathered, out, self.width, self.height, self.world)
        return out
