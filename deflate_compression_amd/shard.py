"""Multi-GPU sharding of one DEFLATE stream.

Blocks are independent, so rank r of N encodes a contiguous, block-aligned range
of the input with no collective on the data path.  Shard framing makes the pieces
concatenable: rank 0 writes the zlib header, every non-final shard ends with an
empty stored block (sync flush, byte-aligned), the last shard carries BFINAL; the
Adler-32 trailer is combined on the host from the per-shard Adler values
(RFC 1950 arithmetic, dmx_adler32_combine).  The exchange step is a gather of the
variable-size compressed chunks to one rank (or all ranks) over RCCL/xGMI.

With the cross-block dictionary (DMX_F_DICT) the first block of a shard
needs the block before it, which the previous rank holds: exchange_history is that
neighbour halo exchange (one sw-byte point-to-point message per rank boundary).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import DMX_F_FINAL, DMX_F_HEADER, adler32_combine

BLOCK = 32768


def shard_range(n: int, rank: int, world: int, sw: int = BLOCK) -> tuple[int, int]:
    """Block-aligned [lo, hi) of rank's share of an n-byte input."""
    nblk = (n + sw - 1) // sw
    b0 = nblk * rank // world
    b1 = nblk * (rank + 1) // world
    return min(b0 * sw, n), min(b1 * sw, n)


def shard_flags(rank: int, world: int) -> int:
    return (DMX_F_HEADER if rank == 0 else 0) | (DMX_F_FINAL if rank == world - 1 else 0)


def combine_adler(adlers, lengths) -> int:
    a = 1
    for ad, ln in zip(adlers, lengths):
        a = adler32_combine(a, int(ad), int(ln))
    return a


def trailer(adler: int) -> bytes:
    return int(adler).to_bytes(4, "big")


def gather_chunks(chunk: torch.Tensor, length: int, root: int | None = 0, group=None):
    """Gather variable-size uint8 chunks (first `length` bytes of `chunk`) from every
    rank.  root=None -> all-gather (every rank gets every chunk, max-size padded);
    root=r -> point-to-point sends to r only (uses all of r's xGMI links at once).
    Returns (list of chunk tensors or None on non-root ranks, list of lengths)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = chunk.device
    ln = torch.tensor([length], dtype=torch.int64, device=dev)
    lens = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(lens, ln, group=group)
    lens = [int(x.item()) for x in lens]
    if root is None:
        m = max(lens) if lens else 0
        buf = torch.zeros(m, dtype=torch.uint8, device=dev)
        buf[:length] = chunk[:length]
        outs = [torch.empty(m, dtype=torch.uint8, device=dev) for _ in range(world)]
        dist.all_gather(outs, buf, group=group)
        return [o[:l] for o, l in zip(outs, lens)], lens
    if rank == root:
        outs = [None] * world
        ops = []
        for r in range(world):
            if r == root:
                outs[r] = chunk[:length]
            else:
                outs[r] = torch.empty(lens[r], dtype=torch.uint8, device=dev)
                if lens[r]:
                    ops.append(dist.P2POp(dist.irecv, outs[r], r, group=group))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        return outs, lens
    if length:
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, chunk[:length].contiguous(), root, group=group)]):
            w.wait()
    return None, lens


def shard_lengths(n: int, dev, group=None) -> list:
    """Every rank's shard length (one all_gather)."""
    world = dist.get_world_size(group)
    ln = torch.tensor([n], dtype=torch.int64, device=dev)
    lens = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(lens, ln, group=group)
    return [int(x.item()) for x in lens]


def exchange_history(d_in: torch.Tensor, n: int, sw: int = BLOCK, group=None, lens=None,
                     out: torch.Tensor | None = None) -> torch.Tensor | None:
    """DMX_F_DICT across shards: the history of this rank's first block is the last block
    of the nearest lower rank with a non-empty shard (shards are block-aligned, so that
    is its last min(sw, len) bytes).  One all_gather of the lengths, then point-to-point
    sends of each tail to the rank(s) that follow it.  Returns the received bytes (a
    uint8 tensor on d_in's device) or None when there is no earlier data.  `lens` (all
    shard lengths, from an earlier call's shard_lengths) and `out` (a receive buffer
    of the right size) let a repeated exchange skip the length all_gather."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = d_in.device
    if lens is None:
        lens = shard_lengths(n, dev, group)

    def src_of(t):
        for r in range(t - 1, -1, -1):
            if lens[r] > 0:
                return r
        return None

    ops = []
    if n > 0:
        tail = d_in[n - min(sw, n):n].contiguous()
        for t in range(rank + 1, world):
            if lens[t] > 0 and src_of(t) == rank:
                ops.append(dist.P2POp(dist.isend, tail, t, group=group))
    src = src_of(rank) if n > 0 else None
    if src is None:
        out = None
    else:
        if out is None or out.numel() != min(sw, lens[src]):
            out = torch.empty(min(sw, lens[src]), dtype=torch.uint8, device=dev)
        ops.append(dist.P2POp(dist.irecv, out, src, group=group))
    for w in dist.batch_isend_irecv(ops) if ops else []:
        w.wait()
    return out
