"""Multi-GPU image-tile rendering: one process per GPU, torch.distributed over RCCL.

SURVEY §8e: pixels are independent and every RNG seed is a pure function of the global
pixel coordinate, so the image shards with no data-path exchange.  Bands of
RT_STRIPE_ROWS rows are dealt round-robin (band b -> rank b % world), which balances the
sky/ground cost between ranks — or, given a partition (one band set per rank, e.g.
rt_partition_bands' cost-balanced contiguous ranges), by that.  Each rank renders its bands
into a compact local buffer (rt_update_frames / rt_update_frames_bands); the only collective
is ONE gather of the finished tiles to rank 0 (RCCL over xGMI), followed by the
de-interleave kernel on the root.  The gather runs either behind the C ABI (StripeComm:
rt_comm_* + rt_gather_stripes / rt_gather_bands, ncclGather inside librt_hip.so — what a
non-Python host binds) or through torch.distributed (gather_stripes).
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from . import _lib
from .compute_shader import (RT_STRIPE_ROWS, ComputeShaderPipeline, _check_image,
                             stripe_local_rows)


class StripeComm:
    """An RCCL communicator of librt_hip.so (rt_comm_create) on a pipeline's device: the
    stripe gather behind the C ABI (rt_gather_stripes = one ncclGather + the root's
    de-interleave)."""

    def __init__(self, pipeline: ComputeShaderPipeline, uid: bytes, nranks: int, rank: int):
        if len(uid) != _lib.RT_COMM_ID_BYTES:
            raise ValueError(f"unique id must be {_lib.RT_COMM_ID_BYTES} bytes")
        self.pipe = pipeline
        buf = (ctypes.c_uint8 * _lib.RT_COMM_ID_BYTES).from_buffer_copy(uid)
        comm = ctypes.c_void_p()
        _lib.call("rt_comm_create", pipeline._ctx, buf, nranks, rank, ctypes.byref(comm))
        self._comm = comm
        self.rank, self.nranks, self.device = self.info()

    @staticmethod
    def unique_id() -> bytes:
        """rt_comm_unique_id (ncclGetUniqueId): call on one rank, share with all."""
        buf = (ctypes.c_uint8 * _lib.RT_COMM_ID_BYTES)()
        _lib.call("rt_comm_unique_id", buf)
        return bytes(buf)

    @classmethod
    def from_process_group(cls, pipeline: ComputeShaderPipeline, group=None, src: int = 0):
        """Every rank of an initialised torch.distributed group calls this together: `src`
        draws the unique id, it is broadcast over the group, and each rank creates its
        communicator (rank and size as in the group)."""
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        box = [cls.unique_id() if rank == src else None]
        dist.broadcast_object_list(box, src=src, group=group)
        return cls(pipeline, box[0], world, rank)

    def info(self) -> tuple[int, int, int]:
        r, n, d = _lib.U32(0), _lib.U32(0), ctypes.c_int(-1)
        _lib.call("rt_comm_info", self._comm, ctypes.byref(r), ctypes.byref(n), ctypes.byref(d))
        return int(r.value), int(n.value), int(d.value)

    def gather(self, local: torch.Tensor, width: int, height: int, root: int = 0,
               gathered: torch.Tensor | None = None,
               out: torch.Tensor | None = None) -> torch.Tensor | None:
        """rt_gather_stripes on the current stream: the full image on `root` (into `out`
        when given), None elsewhere."""
        rows0 = stripe_local_rows(height, 0, self.nranks)
        _check_image(local, width, rows0, "local")
        gptr = outp = None
        if self.rank == root:
            if out is None:
                out = torch.empty((height, width, 4), dtype=torch.float32, device=local.device)
            _check_image(out, width, height, "out")
            outp = ctypes.c_void_p(out.data_ptr())
            if gathered is not None:
                _check_image(gathered, width, rows0 * self.nranks, "gathered")
                gptr = ctypes.c_void_p(gathered.data_ptr())
        _lib.call("rt_gather_stripes", self.pipe._ctx, self._comm,
                  ctypes.c_void_p(local.data_ptr()), gptr, outp, width, height, root,
                  self.pipe._stream())
        return out if self.rank == root else None

    def gather_bands(self, local: torch.Tensor, width: int, height: int, sets, root: int = 0,
                     gathered: torch.Tensor | None = None,
                     out: torch.Tensor | None = None) -> torch.Tensor | None:
        """rt_gather_bands for a partition (sets[r] = rank r's band set): the full image on
        `root`, None elsewhere; every rank's `local` padded to the largest share's rows."""
        rows = max(int(c) for _, _, c in sets) * RT_STRIPE_ROWS
        _check_image(local, width, rows, "local")
        gptr = outp = None
        if self.rank == root:
            if out is None:
                out = torch.empty((height, width, 4), dtype=torch.float32, device=local.device)
            _check_image(out, width, height, "out")
            outp = ctypes.c_void_p(out.data_ptr())
            if gathered is not None:
                _check_image(gathered, width, rows * self.nranks, "gathered")
                gptr = ctypes.c_void_p(gathered.data_ptr())
        _lib.call("rt_gather_bands", self.pipe._ctx, self._comm,
                  ctypes.c_void_p(local.data_ptr()), gptr, outp, width, height,
                  _lib.band_sets(sets), root, self.pipe._stream())
        return out if self.rank == root else None

    def close(self) -> None:
        if getattr(self, "_comm", None) and self._comm.value:
            _lib.call("rt_comm_destroy", self._comm)
            self._comm = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


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
                 world: int, comm: StripeComm | None = None, partition=None):
        """comm: gather through the C ABI's RCCL communicator (rt_gather_stripes /
        rt_gather_bands) instead of torch.distributed.  partition: one band set (first, step,
        count) per rank, identical on every rank and covering every band once (e.g.
        partition_bands' cost-balanced ranges); None = round-robin stripes."""
        if comm is not None and (comm.rank, comm.nranks) != (rank, world):
            raise ValueError("the communicator's rank/size differ from the renderer's")
        self.pipe, self.width, self.height = pipeline, width, height
        self.rank, self.world = rank, world
        self.comm = comm
        self.partition = None
        if partition is not None:
            self.partition = [tuple(int(v) for v in bs) for bs in partition]
            if len(self.partition) != world:
                raise ValueError("a partition holds one band set per rank")
            self.bands = self.partition[rank]
            self.rows = self.bands[2] * RT_STRIPE_ROWS
            self.rows0 = max(bs[2] for bs in self.partition) * RT_STRIPE_ROWS
        else:
            nb = (height + RT_STRIPE_ROWS - 1) // RT_STRIPE_ROWS
            self.bands = (rank, world, (nb - rank + world - 1) // world if nb > rank else 0)
            self.rows = stripe_local_rows(height, rank, world)
            self.rows0 = padded_rows(height, world)
        # ping-pong local accumulators, padded to rows0 so the gather is uniform
        self.buf = [pipeline.new_image(width, self.rows0), pipeline.new_image(width, self.rows0)]
        self.cur = 0
        self._runs = None   # bound update_frames calls, per ping-pong direction
        # the root's gather and output buffers, allocated up front (finish() then runs only
        # the collective and the de-interleave kernel)
        self._gathered = self._image = None
        if world > 1 and rank == 0:
            dev = self.buf[0].device
            self._gathered = torch.empty((world, self.rows0, width, 4), dtype=torch.float32,
                                         device=dev)
            self._image = torch.empty((height, width, 4), dtype=torch.float32, device=dev)

    def band_list(self) -> list[int]:
        """This rank's global bands in local order."""
        f, st, c = self.bands
        return [f + j * st for j in range(c)]

    def frame(self, camera, spheres, seeds) -> None:
        """One progressive `update` (or len(seeds) fused frames) over this rank's bands."""
        if self.partition is not None:
            raise ValueError("a partitioned renderer runs frames() (rt_update_frames_bands)")
        src, dst = self.buf[self.cur], self.buf[1 - self.cur]
        if self.rows:
            self.pipe.render_stripes(src, dst, self.width, self.height, self.rank, self.world,
                                     camera, spheres, seeds)
        self.cur = 1 - self.cur

    def frames(self, camera, spheres, seeds) -> None:
        """len(seeds) progressive frames, one `update` dispatch each, from a single call."""
        if self.rows and self.partition is not None:
            newest = self.pipe.update_frames_bands(self.buf[self.cur], self.buf[1 - self.cur],
                                                   self.width, self.height, self.bands, camera,
                                                   spheres, seeds)
            if newest == 1:
                self.cur = 1 - self.cur
        elif self.rows:
            bind = getattr(self.pipe, "bind_update_frames", None)
            if self._runs is None and bind is not None:
                # both ping-pong directions bound at the first call (the buffers are this
                # renderer's own), so that no later call — a timed one — pays for a binding
                self._runs = [bind(self.buf[k], self.buf[1 - k], self.width, self.height,
                                   self.rank, self.world) for k in (0, 1)]
            run = self._runs[self.cur] if self._runs else None
            if run is not None:
                newest = run(camera, spheres, seeds)
            else:
                newest = self.pipe.update_frames(self.buf[self.cur], self.buf[1 - self.cur],
                                                 self.width, self.height, camera, spheres,
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
        if self.comm is not None:
            if group is not None:
                raise ValueError("a renderer with a communicator gathers over it, not a group")
            pre = dst == 0 and self._gathered is not None
            g = self._gathered.reshape(-1, self.width, 4) if pre else None
            if self.partition is not None:
                return self.comm.gather_bands(self.local, self.width, self.height,
                                              self.partition, dst, gathered=g,
                                              out=self._image if pre else None)
            return self.comm.gather(self.local, self.width, self.height, dst, gathered=g,
                                    out=self._image if pre else None)
        if self.world == 1 and self.partition is None:
            return self.local[: self.height]
        pre = dst == 0 and self._gathered is not None
        gathered = gather_stripes(self.local, self.world, self.rank, dst, group,
                                  out=self._gathered if pre else None)
        if gathered is None:
            return None
        # (the de-interleave writes every pixel: no zero fill needed)
        out = self._image if pre else torch.empty((self.height, self.width, 4),
                                                  dtype=torch.float32, device=gathered.device)
        if self.partition is not None:
            self.pipe.deinterleave_bands(gathered, out, self.width, self.height,
                                         self.partition, self.rows0)
        else:
            self.pipe.deinterleave(gathered, out, self.width, self.height, self.world)
        return out
