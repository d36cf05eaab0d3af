"""One-process-per-GPU plumbing around the C-ABI (torch.distributed, host side).

The data path never goes through torch: each rank's ``libcrossbow_sma``
context owns its RCCL communicator (ncclCommInitRank) and runs the all-reduce
of the SMA step itself.  torch.distributed (gloo, CPU) only carries the
control plane: the 128-byte RCCL unique id from rank 0 to every rank, the
barriers around the timed region and the max-over-ranks of the wall time.

Rank r drives global device r; replica i lives on device i % G, i.e. on rank
i % G (the reference's round-robin placement, clib-multigpu/modelmanager.c:51-64).
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Tuple


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(world: int, rank: int, backend: str = "gloo") -> None:
    import torch.distributed as dist
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend, rank=rank, world_size=world)


def share_unique_id(rank: int, world: int, make: Callable[[], bytes]) -> Optional[bytes]:
    """Rank 0 creates the RCCL unique id with ``make``; every rank returns it."""
    if world <= 1:
        return None
    import torch.distributed as dist
    obj = [make() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    uid = obj[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != 128:
        raise RuntimeError("bad RCCL unique id from rank 0")
    return bytes(uid)


def barrier(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(value: float, world: int) -> float:
    if world <= 1:
        return float(value)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def tune_buckets(gpu, n: int, world: int, step: Callable[[], None], candidates=(1, 2, 4, 8, 16),
                 steps: int = 10, warmup: int = 2, modes=(0, 1, 2), strides=(1, 2, 4), passes: int = 2,
                 group_candidates=(2, 4)):
    """Pick the bucket count of the G > 1 pipeline (kernel A / RCCL
    all-reduce / kernel B per bucket) by timing each candidate on the live
    communicator, the way a runtime tunes itself in its warm-up.

    More buckets hide more of the all-reduce behind kernel A, but each bucket
    costs fixed time (cross-queue waits, a shorter launch's ramp and drain:
    ~7 us per bucket on one MI355X with the bucket events on the kernel
    dispatches, profiles/r01/bench_force_split_tuned.json), so the best count
    depends on how long the all-reduce is, i.e. on G and the xGMI links.
    Every rank times every candidate, the times are max-reduced over ranks,
    and all ranks take the same argmin, so the RCCL call sequence stays
    identical on every rank.  ``step()`` runs one barrier step.
    With more than one bucket each count is also timed in every pipeline
    mode (``gpu.set_pipeline_mode``: 0 within a step, 1 across steps, 2 across
    steps with kernel B on the all-reduce's stream), and modes 1/2 with each
    cross-step wait stride below the bucket count (``gpu.set_cross_wait_stride``).
    The candidates are timed in ``passes`` interleaved passes and each keeps
    its best pass, so one noisy sample (a few percent on one GPU) does not
    decide.  Returns (bucket_elements, mode, stride, {key: ms_per_step}) with
    keys "<buckets>/<mode>" for stride 1 and "<buckets>/<mode>/s<stride>".
    """
    import time

    def combos(nb):
        if nb <= 1:
            return [(0, 1)]
        return [(m, s) for m in modes for s in ((1,) if m == 0 else strides) if s == 1 or s < nb]

    results = {}
    for _ in range(max(1, passes)):
        for nb in candidates:
            elems = (1 << 62) if nb <= 1 else max(1, -(-n // nb))
            for mode, stride in combos(nb):
                gpu.set_bucket_elements(elems)
                gpu.set_pipeline_mode(mode)
                gpu.set_cross_wait_stride(stride)
                for _ in range(warmup):
                    step()
                gpu.wait()
                barrier(world)
                t0 = time.perf_counter()
                for _ in range(steps):
                    step()
                gpu.wait()
                ms = max_over_ranks((time.perf_counter() - t0) * 1e3 / steps, world)
                key = (nb, mode, stride)
                results[key] = min(ms, results.get(key, ms))
    best = min(results, key=lambda k: (results[k], k))
    nb, mode, stride = best
    elems = (1 << 62) if nb <= 1 else max(1, -(-n // nb))
    gpu.set_bucket_elements(elems)
    gpu.set_pipeline_mode(mode)
    gpu.set_cross_wait_stride(stride)
    out = {tuning_key(*k): v for k, v in results.items()}
    # Then the all-reduce grouping of the winner (gpu.set_allreduce_group):
    # fewer comm-stream waits, later all-reduce starts.  On one GPU groups of
    # 2-4 cut 8-16-bucket mode-0 steps by 4-9 % (profiles/r01/allreduce_group_ab.json);
    # over xGMI the later start may cost more than the waits save, so it is timed.
    groups = [grp for grp in group_candidates if 1 < grp < nb]
    if groups:
        timed = {1: results[best]}
        for _ in range(max(1, passes)):
            for grp in groups:
                gpu.set_allreduce_group(grp)
                for _ in range(warmup):
                    step()
                gpu.wait()
                barrier(world)
                t0 = time.perf_counter()
                for _ in range(steps):
                    step()
                gpu.wait()
                ms = max_over_ranks((time.perf_counter() - t0) * 1e3 / steps, world)
                timed[grp] = min(ms, timed.get(grp, ms))
        for grp in groups:
            out[tuning_key(nb, mode, stride) + f"/g{grp}"] = timed[grp]
        gpu.set_allreduce_group(min(timed, key=lambda g: (timed[g], g)))
    return elems, mode, stride, out


def tuning_key(nb: int, mode: int, stride: int = 1) -> str:
    return f"{nb}/{mode}" if stride == 1 else f"{nb}/{mode}/s{stride}"


def local_replicas(size: int, world: int, rank: int):
    """Global replica ids this rank owns (round-robin placement)."""
    return [i for i in range(size) if i % world == rank]


def finalize(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
