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
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional, Tuple

from ._abi import ALLREDUCE_PEER, ALLREDUCE_RCCL, ALLREDUCE_RSAG, CbxError


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def rehearsal_env(rank: int) -> None:
    """Several ranks on ONE device with the real RCCL (rehearsals on a one-GPU
    box): RCCL refuses two ranks of one host on one device, so each rank
    claims a host of its own (NCCL_HOSTID) and the ranks connect through
    RCCL's socket transport over loopback.  Set before the first RCCL call."""
    os.environ["NCCL_HOSTID"] = f"cbx-rehearsal-rank-{rank}"
    os.environ["NCCL_SOCKET_IFNAME"] = "lo"
    os.environ["NCCL_IB_DISABLE"] = "1"
    os.environ["NCCL_NET"] = "Socket"


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


def setup_peer(gpu, world: int) -> Optional[str]:
    """One process per GPU: map every rank's buffers for the peer-read
    all-reduce.  Every rank exports its handles (cbx_peer_export), the blobs
    are all-gathered over the control group in rank order, and every rank
    imports them (cbx_peer_import).  Returns None when every rank succeeded,
    else why not; the ranks agree, so either all of them may use the form or
    none does."""
    if world <= 1:
        return "one rank"
    import torch.distributed as dist
    why = None
    blob = b""
    try:
        blob = gpu.peer_export()
    except CbxError as e:
        why = str(e)
    blobs = [None] * world
    dist.all_gather_object(blobs, blob)
    if why is None:
        if all(isinstance(b, (bytes, bytearray)) and b for b in blobs):
            try:
                gpu.peer_import([bytes(b) for b in blobs])
            except CbxError as e:
                why = str(e)
        else:
            why = "another rank could not export its handles"
    if max_over_ranks(0.0 if why is None else 1.0, world) > 0.0:
        return why or "failed on another rank"
    return None


@dataclass
class Tuning:
    """What ``tune_buckets`` chose (already set on the context) and why."""
    bucket_elements: int
    buckets: int
    mode: int
    stride: int
    group: int
    algorithm: int
    enqueue_threads: Optional[int]          # None: not timed (one local device)
    table: Dict[str, float] = field(default_factory=dict)   # key -> ms per step (max over ranks)
    errors: Dict[str, str] = field(default_factory=dict)    # key -> why the candidate was dropped


def tune_buckets(gpu, n: int, world: int, step: Callable[[], None], candidates=(1, 2, 4, 8),
                 steps: int = 10, warmup: int = 2, modes=(0, 1), strides=(1, 2, 4), passes: int = 2,
                 group_candidates=(2, 4), progress: Optional[Callable[[str], None]] = None,
                 ndev: Optional[int] = None, peer: bool = False, peer_only: bool = False,
                 peer_candidates=(1, 4, 8), threads: bool = False,
                 phase: Optional[Callable[[str], None]] = None,
                 refresh: Optional[Callable[[], None]] = None) -> Tuning:
    """Pick the configuration of the G > 1 pipeline (kernel A / collective /
    kernel B per bucket) by timing each candidate on the live communicator,
    the way a runtime tunes itself in its warm-up.

    More buckets hide more of the collective behind kernel A, but each bucket
    costs fixed time (cross-queue waits, a shorter launch's ramp and drain:
    ~7 us per bucket on one MI355X with the bucket events on the kernel
    dispatches, profiles/r01/bench_force_split_tuned.json), so the best count
    depends on how long the collective is, i.e. on G and the xGMI links.
    Every rank times every candidate, the times are max-reduced over ranks,
    and all ranks take the same argmin, so the RCCL call sequence stays
    identical on every rank.  ``step()`` runs one barrier step.

    The search keeps only the knobs the one-GPU A/B data showed to matter by
    more than 2 %: 1/2/4/8 buckets (16 was slower than 8 everywhere,
    profiles/r01/bench_force_split_tuned.json), pipeline mode 0 (within a
    step) and 1 (across steps, ``gpu.set_pipeline_mode``), mode 1 at each
    cross-step wait stride below the bucket count (``gpu.set_cross_wait_stride``,
    3-6 % at 8 buckets, profiles/r01/cross_wait_stride_ab.json), and the
    collective's form (``gpu.set_allreduce_algorithm``): one all-reduce, or,
    where G divides 1024, reduce-scatter + base momentum on the rank's shard
    + all-gather, which moves the same link bytes in two collectives per
    bucket and saves kernel B's momentum pass on (G-1)/G of the model; with
    one process over every device, or per rank after ``setup_peer``
    (``peer``), also the peer-read form at ``peer_candidates`` buckets
    (``peer_only``: that form alone, e.g. when RCCL refuses the device
    selection).  Then the all-reduce grouping of the
    winner (``gpu.set_allreduce_group``, 4-9 % in mode 0,
    profiles/r01/allreduce_group_ab.json) and, with ``threads`` (one process
    over several devices), the winner with one enqueue thread per device
    against the reference's one thread (``gpu.set_enqueue_threads``).  The
    group, the form and the threads are reset first, so an earlier setting
    never skews the sweep.  Candidates are timed in ``passes`` interleaved
    passes and each keeps its best pass, so one noisy sample (a few percent
    on one GPU) does not decide.

    A candidate whose step fails (``CbxError``: e.g. a collective form the
    communicator refuses) is dropped on every rank (the failure is
    max-reduced, so all ranks keep the same candidates) and recorded in
    ``Tuning.errors``; the sweep goes on.  ``phase(name)`` (if given) is
    called before each candidate, ``progress`` receives one line per timed
    candidate.  ``ndev`` is the number of GPUs (default ``world``: one
    process per GPU).  ``refresh()`` (if given) runs before each candidate's
    warm-up, outside its timing: bench.py puts the fresh synthetic state back
    there, so no candidate runs on values that many earlier steps drove far
    from it (a step's arithmetic per element does not depend on them).

    Keys: "<buckets>/<mode>" for stride 1, "<buckets>/<mode>/s<stride>", the
    same + "/rsag" or "/peer" for the other forms, "<key of the winner>/g<group>"
    and "<key of the final choice>/t1" (threaded enqueue).
    """
    import time

    def combos(nb):
        if nb <= 1:
            return [(0, 1)]
        return [(m, s) for m in modes for s in ((1,) if m == 0 else strides) if s == 1 or s < nb]

    errors: Dict[str, str] = {}

    def failed_anywhere(key: str, why: Optional[str]) -> bool:
        """Agree over ranks whether this candidate failed (every rank then
        drops it, and every rank reaches the same collectives next)."""
        if max_over_ranks(0.0 if why is None else 1.0, world) == 0.0:
            return False
        errors[key] = why or "failed on another rank"
        if progress:
            progress(f"tune {key}: dropped ({errors[key]})")
        return True

    def run_steps(k: int) -> Optional[str]:
        try:
            for _ in range(k):
                step()
            gpu.wait()
            return None
        except CbxError as e:
            try:
                gpu.wait()
            except CbxError:
                pass
            return str(e)

    def attempt(key: str) -> Optional[float]:
        """ms per step of the current setting (max over ranks), or None: the
        candidate failed on some rank and is dropped on every rank."""
        if phase:
            phase(f"tune {key}")
        if refresh:
            refresh()
        if failed_anywhere(key, run_steps(warmup)):
            return None
        barrier(world)
        t0 = time.perf_counter()
        why = run_steps(steps)
        el = (time.perf_counter() - t0) * 1e3 / steps
        if failed_anywhere(key, why):
            return None
        ms = max_over_ranks(el, world)
        if progress:
            progress(f"tune {key}: {ms:.4f} ms/step")
        return ms

    def elems_of(nb):
        return (1 << 62) if nb <= 1 else max(1, -(-n // nb))

    G = world if ndev is None else ndev
    algos = []
    if not peer_only:
        algos.append(ALLREDUCE_RCCL)
        if 1 < G <= 16 and 1024 % G == 0:
            algos.append(ALLREDUCE_RSAG)
    if (peer or peer_only) and 1 < G <= 16:
        algos.append(ALLREDUCE_PEER)
    gpu.set_allreduce_group(1)
    if threads:
        gpu.set_enqueue_threads(0)
    results = {}
    for _ in range(max(1, passes)):
        for algo in algos:
            gpu.set_allreduce_algorithm(algo)
            for nb in (peer_candidates if algo == ALLREDUCE_PEER else candidates):
                for mode, stride in combos(nb):
                    key = (nb, mode, stride, algo)
                    if tuning_key(*key) in errors:
                        continue
                    gpu.set_bucket_elements(elems_of(nb))
                    gpu.set_pipeline_mode(mode)
                    gpu.set_cross_wait_stride(stride)
                    ms = attempt(tuning_key(*key))
                    if ms is None:
                        results.pop(key, None)
                        continue
                    results[key] = min(ms, results.get(key, ms))
    if not results:
        raise CbxError(-1, f"every tuning candidate failed: {errors}")
    best = min(results, key=lambda k: (results[k], k))
    nb, mode, stride, algorithm = best
    gpu.set_allreduce_algorithm(algorithm)
    gpu.set_bucket_elements(elems_of(nb))
    gpu.set_pipeline_mode(mode)
    gpu.set_cross_wait_stride(stride)
    out = {tuning_key(*k): v for k, v in results.items()}
    # Then the all-reduce grouping of the winner: fewer comm-stream waits,
    # later collective starts.  Over xGMI the later start may cost more than
    # the waits save, so it is timed, not assumed.
    group = 1
    groups = [grp for grp in group_candidates if 1 < grp < nb]
    best_ms = results[best]
    if groups:
        timed = {1: best_ms}
        for _ in range(max(1, passes)):
            for grp in groups:
                key = tuning_key(*best) + f"/g{grp}"
                if key in errors:
                    continue
                gpu.set_allreduce_group(grp)
                ms = attempt(key)
                if ms is None:
                    timed.pop(grp, None)
                    continue
                timed[grp] = min(ms, timed.get(grp, ms))
        for grp in groups:
            if grp in timed:
                out[tuning_key(*best) + f"/g{grp}"] = timed[grp]
        group = min(timed, key=lambda g: (timed[g], g))
        best_ms = timed[group]
    gpu.set_allreduce_group(group)
    # Then who enqueues: the reference's one thread over every local device,
    # or one thread per device (host-bound at 8 devices on one thread,
    # DESIGN.md section 6; on 8 distinct devices unmeasured until now).
    enqueue_threads = None
    if threads:
        final = tuning_key(*best) + (f"/g{group}" if group > 1 else "")
        t_ms = None
        for _ in range(max(1, passes)):
            if final + "/t1" in errors:
                break
            gpu.set_enqueue_threads(1)
            ms = attempt(final + "/t1")
            if ms is not None:
                t_ms = ms if t_ms is None else min(t_ms, ms)
        if t_ms is not None:
            out[final + "/t1"] = t_ms
        enqueue_threads = 1 if t_ms is not None and t_ms < best_ms else 0
        gpu.set_enqueue_threads(enqueue_threads)
    return Tuning(bucket_elements=elems_of(nb), buckets=nb, mode=mode, stride=stride, group=group,
                  algorithm=algorithm, enqueue_threads=enqueue_threads, table=out, errors=errors)


def tuning_key(nb: int, mode: int, stride: int = 1, algo: int = ALLREDUCE_RCCL) -> str:
    key = f"{nb}/{mode}" if stride == 1 else f"{nb}/{mode}/s{stride}"
    return key + {ALLREDUCE_RSAG: "/rsag", ALLREDUCE_PEER: "/peer"}.get(algo, "")


def local_replicas(size: int, world: int, rank: int):
    """Global replica ids this rank owns (round-robin placement)."""
    return [i for i in range(size) if i % world == rank]


def finalize(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
