"""Multi-GPU sharding of the multi-bin emulator over output k-bins.

One process per GPU.  The P output bins are split into contiguous blocks, one per
rank; every rank trains an independent multi-bin model (its own theta) on its
block — the reference's shared Gram makes a bin only an extra right-hand side, so
this is the "embarrassing" per-shard-theta mode.  Collectives happen only at the
edges: ONE broadcast of the packed inputs from rank 0 before training and one
gather of the posterior blocks after it; nothing inside the training loop.
Backend "nccl" is RCCL over xGMI on ROCm; "gloo" is used for CPU tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def bin_block(p: int, rank: int, world: int):
    """Contiguous [b0, b1) block of the p bins owned by `rank`."""
    edges = np.linspace(0, p, world + 1).round().astype(int)
    return int(edges[rank]), int(edges[rank + 1])


def broadcast_arrays(arrays, rank: int, world: int, device):
    """Rank 0 passes a list of float64 arrays; every rank gets copies.  One
    broadcast of the shape header and ONE broadcast of the packed payload."""
    if rank == 0:
        shapes = [np.shape(a) for a in arrays]
        hdr = [len(shapes)] + [len(s) for s in shapes] + [d for s in shapes for d in s]
        hdr_t = torch.tensor([len(hdr)] + hdr, dtype=torch.int64, device=device)
    else:
        hdr_t = torch.zeros(64, dtype=torch.int64, device=device)
    if rank == 0:
        pad = torch.zeros(64, dtype=torch.int64, device=device)
        pad[:hdr_t.numel()] = hdr_t
        hdr_t = pad
    if world > 1:
        dist.broadcast(hdr_t, 0)
    h = hdr_t.tolist()
    k = h[1]
    ndims = h[2:2 + k]
    dims = h[2 + k:2 + k + sum(ndims)]
    shapes, o = [], 0
    for nd in ndims:
        shapes.append(tuple(dims[o:o + nd]))
        o += nd
    size = sum(int(np.prod(s)) for s in shapes)
    if rank == 0:
        buf = torch.tensor(np.concatenate([np.asarray(a, dtype=np.float64).ravel() for a in arrays]),
                           dtype=torch.float64, device=device)
    else:
        buf = torch.empty(size, dtype=torch.float64, device=device)
    if world > 1:
        dist.broadcast(buf, 0)
    flat = buf.cpu().numpy()
    out, o = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(flat[o:o + n].reshape(s))
        o += n
    return out


def gather_bin_blocks(block: torch.Tensor, p: int, rank: int, world: int) -> torch.Tensor:
    """All-gather [n, p_r] column blocks into the full [n, p] array (bins in order)."""
    if world == 1:
        return block
    widths = [bin_block(p, r, world)[1] - bin_block(p, r, world)[0] for r in range(world)]
    wmax = max(widths)
    padded = torch.zeros((block.shape[0], wmax), dtype=block.dtype, device=block.device)
    padded[:, :block.shape[1]] = block
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded)
    return torch.cat([parts[r][:, :widths[r]] for r in range(world)], dim=1)
