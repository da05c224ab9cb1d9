"""Multi-process sharding of the observations.

One process per GPU; rank r owns the contiguous block [lo, hi) of the
observations (``shard_range``) and sweeps it on its own device.  The only
exchange per Gibbs sweep is ONE all-reduce (sum) of the int64 sufficient-
statistics block (2n + n^2 + 16 words, < 1 KB at n=10) over
torch.distributed — backend "nccl" (RCCL over xGMI) on the GPUs, "gloo" in
the CPU tests.  Integer sums are exact and order-free, so every rank gets the
identical block, draws the identical Gamma update from the identical host
stream, and the chain is bit-identical for every world size.

This replaces the reference's single-process loop over observations
(src/PHT_MCMC_Aslett.c:325-337); the reference has no distributed mode.
"""
from __future__ import annotations

import numpy as np


def shard_range(N: int, rank: int, world: int) -> tuple[int, int]:
    """Observations [lo, hi) owned by ``rank`` (global ids = Philox counters)."""
    return N * rank // world, N * (rank + 1) // world


def make_stats_allreduce(dist, n_words: int, device: str = "cpu"):
    """reduce(arr: int64 ndarray) -> None: in-place sum over all ranks.

    ``dist`` is ``torch.distributed`` (initialised); ``device`` is where the
    staging buffer lives ("cuda:<local>" for RCCL, "cpu" for gloo)."""
    import torch

    buf = torch.zeros(n_words, dtype=torch.int64, device=device)
    on_gpu = buf.device.type == "cuda"
    # GPU staging goes through one pinned host block: both copies are DMA
    # from page-locked memory, and only one stream sync per sweep.
    host = torch.zeros(n_words, dtype=torch.int64, pin_memory=on_gpu)
    host_np = host.numpy()

    def reduce(arr: np.ndarray) -> None:
        if arr.dtype != np.int64 or arr.shape != (n_words,):
            raise ValueError(f"stats block must be int64[{n_words}], got {arr.dtype}{arr.shape}")
        host_np[:] = arr
        if on_gpu:
            buf.copy_(host, non_blocking=True)
            dist.all_reduce(buf)
            host.copy_(buf, non_blocking=True)
            torch.cuda.current_stream(buf.device).synchronize()
        else:
            dist.all_reduce(host)
        arr[:] = host_np

    return reduce


def rccl_selftest_vector(rank: int, n_words: int) -> np.ndarray:
    """A rank-dependent int64 block exercising all 64 bits of the sum: large
    words (the z sums), small counts, zeros, and words whose total crosses
    2^32 (a 32-bit or float reduction would show)."""
    k = np.arange(n_words, dtype=np.int64)
    v = (k * 7919 + 13) * (rank + 1)
    v[::3] = (np.int64(1) << 50) + k[::3] * 1_000_003 + rank
    v[1::5] = 0
    v[2::7] = np.int64(0xFFFFFFFF) - rank
    return v


def attach_rccl(sweeper, dist, device: str, n_words: int = 256) -> bool:
    """The in-library alternative to make_stats_allreduce on GPUs: rank 0
    makes an RCCL unique id, torch.distributed broadcasts it, and every
    rank's Sweeper sums its statistics block with an RCCL all-reduce on its
    own sweep stream (no host callback, no staging copies per sweep).

    Self-test before use: the library's all-reduce of a rank-dependent int64
    block must equal torch.distributed's sum of the same block, bit for bit,
    on every rank (agreed by an all-reduce of the verdicts).  Returns True
    when the in-library reduce is attached and verified; False when the test
    failed — the caller must then use make_stats_allreduce (a context with a
    communicator refuses a callback, so the caller also needs a fresh
    Sweeper)."""
    import torch

    from . import RCCL_ID_BYTES, rccl_unique_id

    # every rank reaches every collective below whatever fails locally, so a
    # failure on one rank becomes a common "fall back" verdict, not a hang
    def agree(ok):
        v = torch.tensor([1 if ok else 0], dtype=torch.int64, device=device)
        dist.all_reduce(v, op=dist.ReduceOp.MIN)
        return bool(v.item())

    # local preconditions first (RCCL loadable, device, no communicator yet,
    # the self-test's staging buffer): a rank failing them must not enter
    # ncclCommInitRank, where its peers would wait for it forever
    try:
        sweeper.rccl_prepare(n_words)
        prepared = True
    except Exception:  # noqa: BLE001 - reported through the verdict
        prepared = False
    if not agree(prepared):
        return False
    t = torch.zeros(RCCL_ID_BYTES + 1, dtype=torch.uint8, device=device)  # id + "id made" byte
    if dist.get_rank() == 0:
        try:
            t[:RCCL_ID_BYTES].copy_(torch.frombuffer(bytearray(rccl_unique_id()), dtype=torch.uint8))
            t[RCCL_ID_BYTES] = 1
        except Exception:  # noqa: BLE001 - rank 0 has no RCCL: everyone falls back
            t[RCCL_ID_BYTES] = 0
    dist.broadcast(t, 0)
    host = t.cpu().numpy()
    if host[RCCL_ID_BYTES] == 0:
        return False
    try:
        sweeper.attach_rccl(bytes(host[:RCCL_ID_BYTES].tobytes()), dist.get_world_size(), dist.get_rank())
        attached = True
    except Exception:  # noqa: BLE001 - reported through the verdict
        attached = False
    if not agree(attached):
        return False
    mine = rccl_selftest_vector(dist.get_rank(), n_words)
    lib_sum = mine.copy()
    ok = 1
    try:
        sweeper.rccl_allreduce(lib_sum)
    except Exception:  # noqa: BLE001 - reported through the verdict
        ok = 0
    ref = torch.from_numpy(mine.copy()).to(device)
    dist.all_reduce(ref)
    if ok and not np.array_equal(lib_sum, ref.cpu().numpy()):
        ok = 0
    return agree(ok)


def max_over_ranks(dist, values, device: str = "cpu"):
    """Element-wise max of a few floats over ranks (bench timing)."""
    import torch

    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def sum_over_ranks(dist, values, device: str = "cpu"):
    """Element-wise sum of a few floats over ranks."""
    import torch

    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return [float(v) for v in t.cpu()]
