"""Batch sharding across the GPUs of one node (one process per GPU).

Problems are independent, so a batch of N splits into
contiguous rank-major blocks and every rank solves its own block with no data-path
collective.  Inputs are generated on each rank from the counter-based stream
(offset = the block's first element), so no scatter is needed either.  The only
collectives are the optional split / gather a caller with host- or rank-0-resident data
needs: scatter_blocks hands each rank its block of one rank's batch, gather_blocks
collects every H block on one rank, both as paired send/recv over RCCL
(torch.distributed "nccl" == RCCL on ROCm) -- reported separately by bench.py.

A batch that lives in HOST memory needs neither: SharedHostBatch puts src/tar/H in one
shared-memory file every rank maps, and each rank's GPU reads its block and writes its H
rows over its own PCIe link (ops.solve_host, zero-copy) -- N links in parallel, no xGMI
traffic, no rank-0 bottleneck.
"""
from __future__ import annotations

import mmap
import os
from typing import Callable, List, Optional, Tuple

import torch


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of rank's contiguous block; sizes differ by at most one problem."""
    if world < 1 or not 0 <= rank < world or n_total < 0:
        raise ValueError(f"bad shard request n={n_total} world={world} rank={rank}")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def gather_blocks(block: torch.Tensor, n_total: int, world: int, rank: int, dst: int = 0,
                  group=None) -> Optional[torch.Tensor]:
    """Gathers each rank's (n_r, 9) H block into one (n_total, 9) tensor on ``dst``.

    Uses paired send/recv (a gather, not an all-gather: rank ``dst``'s ingress is the
    bound, ~7 xGMI links).  Returns the full tensor on ``dst``, None elsewhere.
    """
    import torch.distributed as dist

    lo, hi = shard_range(n_total, world, rank)
    if block.shape[0] != hi - lo:
        # checked before any send/recv: a wrong-sized block would leave a peer waiting
        raise ValueError(f"rank {rank} holds {block.shape[0]} rows, its block is [{lo},{hi})")
    if world == 1:
        return block
    if rank == dst:
        full = torch.empty((n_total,) + tuple(block.shape[1:]), dtype=block.dtype,
                           device=block.device)
        ops: List = []
        for r in range(world):
            lo, hi = shard_range(n_total, world, r)
            if r == dst:
                full[lo:hi].copy_(block)
            elif hi > lo:
                ops.append(dist.P2POp(dist.irecv, full[lo:hi], r, group))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        return full
    if hi > lo:
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, block.contiguous(), dst, group)]):
            w.wait()
    return None


def scatter_blocks(full: Optional[torch.Tensor], n_total: int, world: int, rank: int,
                   like: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    """Splits ``full`` ((n_total, ...) on rank ``src``; None elsewhere) into the contiguous
    rank-major blocks of shard_range and returns this rank's block (shaped like
    ``like``'s rows).  Paired send/recv: rank ``src``'s egress is the bound."""
    import torch.distributed as dist

    lo, hi = shard_range(n_total, world, rank)
    if rank == src and (full is None or full.shape[0] != n_total):
        raise ValueError(f"rank {src} must hold the whole ({n_total}, ...) batch")
    if world == 1:
        return full
    if rank == src:
        ops: List = []
        for r in range(world):
            rlo, rhi = shard_range(n_total, world, r)
            if r != src and rhi > rlo:
                ops.append(dist.P2POp(dist.isend, full[rlo:rhi].contiguous(), r, group))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        return full[lo:hi]
    block = torch.empty((hi - lo,) + tuple(like.shape[1:]), dtype=like.dtype, device=like.device)
    if hi > lo:
        for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, block, src, group)]):
            w.wait()
    return block


class SharedHostBatch:
    """An (n, 8) src, (n, 8) tar and (n, 9) H float32 batch in one shared-memory file
    (``/dev/shm/<name>``) that every rank of the node maps.  Rank ``owner`` creates it
    (``posix_fallocate`` reserves the pages up front, so a full /dev/shm fails here with
    OSError instead of a SIGBUS later), the others attach after ``barrier()``.  Each rank
    then solves its block with ``solve_block`` (the GPU reads and writes the shared pages
    directly).  ``close()`` unmaps; the owner also unlinks."""

    def __init__(self, name: str, n: int, rank: int, barrier: Callable[[], None],
                 owner: int = 0, directory: str = "/dev/shm"):
        if n < 0:
            raise ValueError(f"n must be >= 0, got {n}")
        self.n, self.rank, self.owner = n, rank, owner
        self.path = os.path.join(directory, name)
        nbytes = max(n * (8 + 8 + 9) * 4, 4096)
        self._mm = None
        err = None
        if rank == owner:
            try:
                fd = os.open(self.path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o600)
                try:
                    os.posix_fallocate(fd, 0, nbytes)
                    self._mm = mmap.mmap(fd, nbytes)
                finally:
                    os.close(fd)
            except OSError as e:  # reported after the barrier, so no peer waits forever
                err = e
                try:
                    os.unlink(self.path)
                except OSError:
                    pass
        barrier()
        if rank == owner and err is not None:
            raise err
        if rank != owner:
            fd = os.open(self.path, os.O_RDWR)
            try:
                if os.fstat(fd).st_size < nbytes:
                    raise OSError(f"{self.path} holds fewer than {nbytes} bytes")
                self._mm = mmap.mmap(fd, nbytes)
            finally:
                os.close(fd)
        flat = torch.frombuffer(self._mm, dtype=torch.float32, count=nbytes // 4)
        self.src = flat[:n * 8].view(n, 8)
        self.tar = flat[n * 8:n * 16].view(n, 8)
        self.H = flat[n * 16:n * 25].view(n, 9)

    def block(self, world: int, rank: Optional[int] = None) -> Tuple[int, int]:
        return shard_range(self.n, world, self.rank if rank is None else rank)

    def solve_block(self, world: int, algo: str = "aca", normalize: bool = True,
                    device=None) -> Tuple[int, int]:
        """Solves this rank's block in place (H rows of the shared file); returns it."""
        from .ops import solve_host

        lo, hi = self.block(world)
        if hi > lo:
            solve_host(algo, self.src[lo:hi], self.tar[lo:hi], normalize=normalize,
                       out=self.H[lo:hi], device=device)
        return lo, hi

    def close(self) -> None:
        self.src = self.tar = self.H = None
        if self._mm is not None:
            try:
                self._mm.close()
            except BufferError:  # a caller still holds a view: leave the mapping to GC
                pass
            self._mm = None
        if self.rank == self.owner:
            try:
                os.unlink(self.path)
            except OSError:
                pass
