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
rows over its own PCIe link (ops.solve_host with register=True, zero-copy) -- N links in parallel, no xGMI
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
    (``/dev/shm/<name>``) that every rank of the node maps.  Rank ``owner`` creates it; the
    others attach after ``barrier()``.  Each rank then solves its block with ``solve_block``
    (the GPU reads and writes the shared pages directly).  ``close()`` unmaps; the owner
    also unlinks.

    Page placement.  With ``world`` given, the owner only sizes the file and every rank
    allocates the pages of its OWN block (its src, tar and H rows) with ``posix_fallocate``
    -- on tmpfs the pages are allocated by the calling process, so under the default
    first-touch policy they land on that rank's NUMA node (bench.py binds each rank to its
    GPU's node before anything else).  A full /dev/shm fails there with OSError, not a
    SIGBUS later; ``agree(ok) -> all_ok`` (e.g. a max-reduction over ranks) lets every rank
    learn of another's failure.  Without ``world`` the owner allocates the whole file (one
    process, or placement does not matter)."""

    def __init__(self, name: str, n: int, rank: int, barrier: Callable[[], None],
                 owner: int = 0, directory: str = "/dev/shm", world: Optional[int] = None,
                 agree: Optional[Callable[[bool], bool]] = None):
        if n < 0:
            raise ValueError(f"n must be >= 0, got {n}")
        if world is not None and not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.n, self.rank, self.owner = n, rank, owner
        self.path = os.path.join(directory, name)
        nbytes = max(n * (8 + 8 + 9) * 4, 4096)
        self.nbytes = nbytes
        self._mm = None
        err = None
        if rank == owner:
            try:
                fd = os.open(self.path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o600)
                try:
                    if world is None:
                        os.posix_fallocate(fd, 0, nbytes)
                    else:
                        os.ftruncate(fd, nbytes)  # sized, no pages yet: each rank allocates its own
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
            if world is not None and agree is not None:
                agree(False)
            raise err
        if rank != owner:
            try:
                fd = os.open(self.path, os.O_RDWR)
                try:
                    if os.fstat(fd).st_size < nbytes:
                        raise OSError(f"{self.path} holds fewer than {nbytes} bytes")
                    self._mm = mmap.mmap(fd, nbytes)
                finally:
                    os.close(fd)
            except OSError:
                if world is not None and agree is not None:
                    agree(False)  # every rank votes exactly once, failure or not
                raise
        if world is not None:
            ok, err = True, None
            try:
                self.allocate_block(world)
            except OSError as e:
                ok, err = False, e
            if agree is not None and not agree(ok) and ok:
                err = OSError("another rank could not allocate its block of the shared batch")
            if err is not None:
                self.close()
                raise err
        flat = torch.frombuffer(self._mm, dtype=torch.float32, count=nbytes // 4)
        self.src = flat[:n * 8].view(n, 8)
        self.tar = flat[n * 8:n * 16].view(n, 8)
        self.H = flat[n * 16:n * 25].view(n, 9)

    def block_byte_ranges(self, world: int, rank: Optional[int] = None) -> List[Tuple[int, int]]:
        """The file byte ranges of a rank's block: its src, tar and H rows."""
        lo, hi = self.block(world, rank)
        n = self.n
        return [(lo * 32, hi * 32), (n * 32 + lo * 32, n * 32 + hi * 32),
                (n * 64 + lo * 36, n * 64 + hi * 36)]

    def allocate_block(self, world: int) -> None:
        """Allocates the pages under this rank's block (posix_fallocate from this process)."""
        fd = os.open(self.path, os.O_RDWR)
        try:
            for a, b in self.block_byte_ranges(world):
                if b > a:
                    os.posix_fallocate(fd, a, b - a)
        finally:
            os.close(fd)

    def block(self, world: int, rank: Optional[int] = None) -> Tuple[int, int]:
        return shard_range(self.n, world, self.rank if rank is None else rank)

    def solve_block(self, world: int, algo: str = "aca", normalize: bool = True,
                    device=None) -> Tuple[int, int]:
        """Solves this rank's block in place (H rows of the shared file); returns it.  The
        pages are registered for the call (zero-copy, HG_FLAG_HOST_REGISTER): they belong to
        this object's own shared-memory mapping, never to the heap, and the driver drops any
        GPU mapping of them when close() unmaps the file."""
        from .ops import solve_host

        lo, hi = self.block(world)
        if hi > lo:
            solve_host(algo, self.src[lo:hi], self.tar[lo:hi], normalize=normalize,
                       out=self.H[lo:hi], device=device, register=True)
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
