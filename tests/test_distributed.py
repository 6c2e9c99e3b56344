"""Multi-process (world_size 2, gloo, CPU) test of the stripe partition + single gather.

Each rank renders its bands with the CPU oracle (test infrastructure standing in for the
GPU kernel, which needs a device), the product's gather_stripes() moves them to rank 0,
and the de-interleaved image must equal the oracle's full render bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, w, h, q):
    sys.path[:0] = [str(PKG_DIR), str(ROOT)]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gpu_ray_tracing import distributed as D
        from gpu_ray_tracing import stripe_local_rows
        from oracle import host_ref as H
        from oracle import oracle as O
        spheres = H.generate_scene(1, 0, 4)
        seeds = H.frame_seeds(3, 2)
        cam = H.scene_camera_from(max_depth=3, width=w, height=h, random_seed=float(seeds[0]))
        rows, rows0 = stripe_local_rows(h, rank, world), D.padded_rows(h, world)
        local = np.zeros((rows0, w, 4), np.float32)
        # this rank's bands, global coordinates
        ys = [b * 8 + r for b in range(rank, (h + 7) // 8, world) for r in range(8)
              if b * 8 + r < h]
        assert len(ys) <= rows
        yy = np.repeat(np.array(ys, np.uint32), w)
        xx = np.tile(np.arange(w, dtype=np.uint32), len(ys))
        st, _ = O.render_pixels(np.zeros((yy.size, 4), np.float32), xx, yy, cam, spheres, seeds)
        local[: len(ys)] = st.reshape(len(ys), w, 4)
        g = D.gather_stripes(torch.from_numpy(local), world, rank)
        if rank == 0:
            g = g.numpy().reshape(world, rows0, w, 4)
            img = np.empty((h, w, 4), np.float32)
            for y in range(h):
                band = y // 8
                img[y] = g[band % world, (band // world) * 8 + y % 8]
            full, _ = O.render(np.zeros((h, w, 4), np.float32), cam, spheres, seeds)
            q.put(bool(np.array_equal(img.view(np.uint32), full.view(np.uint32))))
        else:
            assert g is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h", [(2, 24, 40), (2, 17, 21), (3, 16, 33)])
def test_stripe_gather_gloo(world, w, h):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert q.get(timeout=5) is True
