"""Sharded corpus search: per-shard top-k + one all-gather + merge.

Replaces the sequential per-document loop of BatchProcessor.search_similar
(batch_operations.py:268-284). Every rank owns a contiguous range of global
document indices (index.json insertion order, encrypted_storage.py:136-141),
computes encrypted compares and its local top-k by (acc desc, index asc) —
the order Python's stable sort gives batch_operations.py:282 on a monotone
dequantisation — and the ranks exchange k (acc, index) pairs with ONE
all-gather (RCCL over xGMI on MI355X; gloo in the CPU tests). Because rank r's
indices all precede rank r+1's, merging by (acc desc, position asc) over the
rank-ordered concatenation is exactly (acc desc, global index asc).
"""
from __future__ import annotations

import numpy as np
import torch


def sharded_topk(acc: torch.Tensor, below: torch.Tensor | None, k: int, base_idx: int, topk_fn,
                 world: int = 1, group=None):
    """topk_fn(acc, below, k, base_idx) -> (acc_k, idx_k), missing slots idx -1.

    Returns the global top-k (identical on every rank). The exchange runs
    whenever a process group exists, a one-rank group included (so a
    one-GPU launcher run executes the RCCL all-gather too), and world must
    then equal the group's size (ValueError otherwise); without one, world
    must be 1."""
    oa, oi = topk_fn(acc, below, k, base_idx)
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        if world != 1:
            raise RuntimeError(f"sharded_topk: world {world} without a process group")
        return oa, oi
    if world != torch.distributed.get_world_size(group):
        # a caller meaning a local (replicated) search inside a multi-rank job
        # would otherwise merge every rank's duplicates, or hang when the
        # other ranks do not join: refuse instead of overriding the argument
        raise ValueError(f"sharded_topk: world {world} but the process group has "
                         f"{torch.distributed.get_world_size(group)} ranks")
    # one collective: the k (acc, index) pairs travel packed as [k, 2] int64.
    # RCCL gathers device tensors in place; other backends (gloo rehearsals)
    # go through host copies
    dev = oa.device
    host = dev.type != "cpu" and torch.distributed.get_backend(group) != "nccl"
    pairs = torch.stack([oa.to(torch.int64), oi.to(torch.int64)], dim=1)
    if host:
        pairs = pairs.cpu()
    gathered = [torch.empty_like(pairs) for _ in range(world)]
    torch.distributed.all_gather(gathered, pairs, group=group)
    cat = torch.cat(gathered).to(dev)
    cat_a, cat_i = cat[:, 0].contiguous(), cat[:, 1].contiguous()
    ma, pos = topk_fn(cat_a, (cat_i < 0).to(torch.int64), k, 0)
    mi = torch.where(pos >= 0, cat_i[pos.clamp(min=0)], pos)
    return ma, mi


def host_topk(acc: torch.Tensor, below: torch.Tensor | None, k: int, base_idx: int):
    """Host (numpy) twin of fhe_topk for the clear search modes: entries with
    below == 0 ordered by (acc desc, index asc); indices are base_idx +
    position; missing slots acc = INT64_MIN, idx = -1."""
    a = acc.cpu().numpy().astype(np.int64)
    keep = np.arange(a.size) if below is None else np.flatnonzero(below.cpu().numpy() == 0)
    order = keep[np.lexsort((keep, -a[keep]))][:k]
    oa = np.full(k, np.iinfo(np.int64).min, dtype=np.int64)
    oi = np.full(k, -1, dtype=np.int64)
    oa[:order.size] = a[order]
    oi[:order.size] = order + base_idx
    return torch.from_numpy(oa), torch.from_numpy(oi)
