"""Multi-rank path of bench.py on CPU with the gloo backend (world_size 2 and 4).

Each rank builds its shard exactly as bench.py does (shard_spec + host_shard), checksums it
with the oracle, and the test gathers the per-rank results and checks that they equal the
single-process checksum of the whole global batch -- i.e. the shards are disjoint and
together cover the batch, with no data-path collective in the product path (the gather
here is the test's own). Also checks the max-over-ranks timing reduction bench.py uses.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, Oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, config, n, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    spec = bench.shard_spec(config, rank, world, n=n)
    host = bench.host_shard(spec)
    orc = Oracle()
    if spec["layout"] == "strided":
        res = orc.batch_strided(host, spec["plen"], spec["plen"], n)
    else:
        res = orc.batch_csr(host, spec["offsets"])
    gathered = [torch.zeros(n, dtype=torch.int32) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(res.astype(np.int32)))
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)     # bench.py's max-over-ranks time
    dist.barrier()
    if rank == 0:
        q.put((np.concatenate([g.numpy() for g in gathered]).astype(np.uint16), float(t.item()),
               spec["byte_offset"]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("config,n", [("A", 3000), ("B", 500), ("C", 4000)])
def test_shards_compose_global_batch(world, config, n):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, config, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, tmax, off0 = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == float(world) and off0 == 0
    # the whole global batch in one process
    whole = bench.shard_spec(config, 0, 1, n=n * world)
    host = bench.host_shard(whole)
    orc = Oracle()
    if whole["layout"] == "strided":
        want = orc.batch_strided(host, whole["plen"], whole["plen"], n * world)
    else:
        want = orc.batch_csr(host, whole["offsets"])
    assert np.array_equal(got, want)


def test_shard_specs_are_disjoint_and_contiguous():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    for config in ("A", "C"):
        specs = [bench.shard_spec(config, r, 4, n=1000) for r in range(4)]
        for a, b in zip(specs, specs[1:]):
            assert b["byte_offset"] == a["byte_offset"] + a["total"]
            assert b["first_packet"] == a["first_packet"] + a["n"]
