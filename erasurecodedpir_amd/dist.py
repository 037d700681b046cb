"""Split-shard layout across GPUs: one logical PIR server's 2^n-row shard is
partitioned into G = 2^g contiguous row ranges, one per rank (= one GPU, one process).  Rank r
evaluates the DPF subtree under node r of tree level g (a prefix descent, the decomposition the
reference's evalAllOptimizedDPFThread attempts at src/c/dpf_tree.cpp:657-684) and scans its
own rows; the per-rank answers are XOR-combined.  RCCL has no XOR reduction, so the engine
all-gathers the NR x EFS partials over RCCL and XOR-folds them on the device
(csrc/pir_engine.cpp).  This module only bootstraps the communicator through
torch.distributed (which carries the 128-byte RCCL unique id) and holds the partition math.
"""
import numpy as np


def log2_exact(v):
    if v <= 0 or v & (v - 1):
        raise ValueError(f"{v} is not a power of two")
    return v.bit_length() - 1


def partition(rank, world_size, n):
    """-> (log_parts, prefix, first_row, num_rows) of rank's share of a 2^n-row shard."""
    g = log2_exact(world_size)
    if g > n:
        raise ValueError(f"{world_size} partitions of a 2^{n}-row shard")
    rows = 1 << (n - g)
    return g, rank, rank * rows, rows


def broadcast_bytes(payload, group=None):
    """Rank 0's bytes on every rank (torch.distributed object broadcast)."""
    import torch.distributed as dist

    obj = [payload if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


def make_split_engine(num_parties, party_index, n, record_bytes, num_rounds=1, device=None,
                      group=None):
    """Create this rank's partition engine and attach the RCCL communicator.  Call inside an
    initialised torch.distributed job (one process per GPU)."""
    import torch.distributed as dist

    from .engine import Engine, comm_unique_id

    rank, world = dist.get_rank(), dist.get_world_size()
    g, prefix, _, _ = partition(rank, world, n)
    if device is None:
        import os

        device = int(os.environ.get("LOCAL_RANK", rank))
    eng = Engine(num_parties, party_index, n, record_bytes, num_rounds, device=device,
                 log_num_partitions=g, partition_index=prefix)
    uid = broadcast_bytes(comm_unique_id() if rank == 0 else None, group)
    if world > 1:
        eng.attach_comm(uid, world, rank)
    return eng


def xor_fold_allgather(partial, group=None):
    """Host-side reference of the engine's combine step: all-gather the per-rank partial
    answers (uint8 arrays of equal shape) and XOR-fold them (used on CPU / gloo)."""
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.ascontiguousarray(partial, dtype=np.uint8))
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    out = np.zeros_like(partial)
    for p in parts:
        out ^= p.numpy()
    return out
