"""Multi-GPU sharding of one DEFLATE stream.

Blocks are independent, so rank r of N encodes a contiguous, block-aligned range
of the input with no collective on the data path.  Shard framing makes the pieces
concatenable: rank 0 writes the zlib header, every non-final shard ends with an
empty stored block (sync flush, byte-aligned), the last shard carries BFINAL; the
Adler-32 trailer is combined on the host from the per-shard Adler values
(RFC 1950 arithmetic, dmx_adler32_combine).  The exchange step is a gather of the
variable-size compressed chunks to one rank (or all ranks) over RCCL/xGMI.
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
