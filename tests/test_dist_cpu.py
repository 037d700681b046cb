"""The split-shard (multi-GPU) control plane on CPU: partition math, the torch.distributed
bootstrap of the RCCL unique id, and the XOR combine of partition answers -- checked with
world_size-2/4 gloo process groups against the oracle's whole-shard answer.  (The device-side
combine is the same XOR fold over an RCCL all-gather, csrc/pir_engine.cpp.)"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import _oracle as O
from erasurecodedpir_amd.dist import log2_exact, partition


def test_partition_math():
    assert partition(0, 1, 20) == (0, 0, 0, 1 << 20)
    assert partition(3, 8, 27) == (3, 3, 3 << 24, 1 << 24)
    assert log2_exact(8) == 3
    with pytest.raises(ValueError):
        log2_exact(6)
    with pytest.raises(ValueError):
        partition(0, 16, 3)
    # the rows of all partitions tile the shard exactly
    rows = sorted(partition(r, 4, 10)[2:] for r in range(4))
    assert [a for a, _ in rows] == [0, 256, 512, 768] and all(b == 256 for _, b in rows)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, q):
    import torch.distributed as dist
    from erasurecodedpir_amd.dist import broadcast_bytes, xor_fold_allgather

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p, n, efs, nq, party1, key, shard = case
        uid = broadcast_bytes(os.urandom(128) if rank == 0 else None)
        g, prefix, row0, rows = partition(rank, world, n)
        # this rank's partition answer (the oracle stands in for the partition engine)
        part = O.answer_slice(p, party1, n, efs, nq, key, shard, prefix, world)
        full = xor_fold_allgather(part)
        q.put((rank, uid, full.tobytes(), row0, rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_split_shard_xor_combine_gloo(world):
    p, n, efs, nq = 3, 10, 48, 2
    rng = np.random.default_rng(world)
    fcw = O.final_cw(p, nq, 1)
    keys = O.gen_keys(n, 700, fcw, p, nq, rng.integers(0, 256, 16 * p, dtype=np.uint8).tobytes())
    shard = rng.integers(0, 256, (1 << n) * efs, dtype=np.uint8)
    case = (p, n, efs, nq, 2, keys[1], shard)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    want = O.answer(p, 2, n, efs, nq, keys[1], shard).tobytes()
    uids = {r[1] for r in res}
    assert len(uids) == 1  # every rank got rank 0's communicator id
    for rank, _, full, row0, rows in res:
        assert full == want, rank
        assert rows == (1 << n) // world and row0 == rank * rows
