#!/usr/bin/env python3
"""bench.py -- SMA param-bucket reduce on MI355X (BASELINE.json metric).

A "step" is one ModelManager.trySynchronise (lockAny -> synchronise ->
unlockAny, ModelManager.java:293-353) over the full flat parameter buffer of
the workload, with every input already resident in HBM:

  N = 1 : configs[2] (C3) -- ResNet-50 fp32 parameters (n = 25,557,032),
          8 replicas on one MI355X, alpha 0.1, momentum 0.9: the fused kernel.
  N > 1 : the same 8 replicas per GPU on each of N GPUs (weak scaling):
          kernel A + RCCL all-reduce over xGMI + kernel B per GPU.

value = algorithmic bytes moved by all ranks / max-over-ranks wall time of
exactly K steps ((12R+8+8m)n per step at G = 1, and
(12R+8)n + (12+8m)n per GPU at G > 1; the all-reduce is reported apart).

Process forms at N > 1:
  per-rank  one process per GPU, launched by torch.distributed.run (each rank
            its own RCCL communicator, ncclCommInitRank).  RCCL's forms are
            tuned and timed first; the peer-read form (IPC-mapped buffers)
            after them, timed too if its best candidate is faster, and the
            faster timed block sets `value` (the other: `other_form`);
  single    one process over N devices, the form Crossbow itself takes
            (TheGPU.init -> ncclCommInitAll, executioncontext.c:185-201, grouped
            all-reduces from one host thread, synch/common.c:14-54): --gpus N
            without a torch.distributed.run environment, or --single-process.

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
      python bench.py --gpus N [--single-process]
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import math
import os
import re
import select
import signal
import socket
import statistics
import subprocess
import sys
import tempfile
import threading
import time

# ROCclr's hardware queues per device (GPU_MAX_HW_QUEUES, read once when the
# HIP runtime starts).  bench.py runs with the environment's value (HIP's
# default 4 when unset), the value a deployment gets unless it sets one:
# forcing 16 (round 4) slowed the replica optimiser step on a caller's
# stream by a third, while the pipeline at G > 1 measured
# within 3 % of 16 at 4.  `--hw-queues N` sets it for the
# run; config.hw_queues records the value and who set it.
HW_QUEUES_ENV = os.environ.get("GPU_MAX_HW_QUEUES")
HW_QUEUES_SET = None
if "--hw-queues" in sys.argv[:-1]:
    HW_QUEUES_SET = sys.argv[sys.argv.index("--hw-queues") + 1]
    os.environ["GPU_MAX_HW_QUEUES"] = HW_QUEUES_SET

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "GB/s device-resident SMA param-bucket reduce (ResNet-50, 8 replicas)"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
XGMI_LINK_GBS = 153.0  # per xGMI link (7 per MI355X, one to each peer on an 8-GPU node)
SEED = 20190701


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--model", choices=["resnet50", "lenet"], default="resnet50")
    p.add_argument("--replicas", type=int, default=8, help="replicas per GPU")
    p.add_argument("--alpha", type=float, default=0.1)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--block", type=int, default=64)
    p.add_argument("--blocks-per-cu", type=int, default=0)
    p.add_argument("--policy", type=int, default=1, help="0 plain, 1 nontemporal loads/stores")
    p.add_argument("--unroll", type=int, default=2)
    p.add_argument("--waves-per-cu", type=int, default=-1,
                   help="occupancy cap for the SMA kernels: -1 auto (library default), 0 none, else waves per CU")
    p.add_argument("--bucket-mb", type=float, default=0.0,
                   help="G>1 pipeline bucket (MB of fp32): 0 = tuned in the warm-up (dist.tune_buckets), "
                        "<0 = one bucket")
    p.add_argument("--calib-steps", type=int, default=10,
                   help="G>1: unpipelined steps before warm-up that time kernel A, the all-reduce and kernel B apart")
    p.add_argument("--tune-steps", type=int, default=10, help="G>1 tuner: timed steps per candidate and pass")
    p.add_argument("--tune-passes", type=int, default=2,
                   help="G>1 tuner: interleaved passes over the candidates (each keeps its best pass)")
    p.add_argument("--force-split", action="store_true", help="use kernel A + all-reduce + B even at G=1")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--cpu-elements", type=int, default=0,
                   help="elements of the CPU baseline's state (0 = the full workload, n)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-staged", action="store_true")
    p.add_argument("--no-copy-ceiling", action="store_true")
    p.add_argument("--staged-buckets", type=int, default=8,
                   help="buckets of the pipelined host-staged step (cbx_synchronise_staged)")
    p.add_argument("--no-optimiser", action="store_true", help="skip the replica optimiser-step measurement")
    p.add_argument("--no-seam", action="store_true", help="skip the sma.c seam measurement (caller-owned buffers)")
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="N > 1 rehearsal on a one-GPU box: every rank on device 0, each its own RCCL 'host' "
                        "(NCCL_HOSTID), so real RCCL links the ranks by sockets over loopback; the numbers say "
                        "nothing about xGMI, the run checks the N > 1 code path end to end")
    p.add_argument("--single-process", action="store_true",
                   help="N > 1 in one process over N devices (cbx_init -> ncclCommInitAll, Crossbow's own form); "
                        "the default when --gpus N > 1 runs without a torch.distributed.run environment. With "
                        "--rehearse-one-gpu every device is device 0 and the all-reduce is the peer-read form "
                        "(RCCL refuses a repeated device)")
    p.add_argument("--rccl-tuning-log", action="store_true",
                   help="N > 1 with RCCL: log RCCL's per-collective tuning choices (NCCL_DEBUG=INFO, "
                        "NCCL_DEBUG_SUBSYS=TUNING into a file) in THIS run for the allreduce.rccl_tuning field "
                        "(one log line per collective on the host's enqueue path, so off by default)")
    p.add_argument("--no-rccl-tuning-run", action="store_true",
                   help="N > 1 with RCCL: skip the separate short run (same configuration, RCCL's tuning log on) "
                        "that fills allreduce.rccl_tuning after the timed region")
    p.add_argument("--bucket-elements", type=int, default=0,
                   help="G>1 pipeline bucket in fp32 elements (overrides --bucket-mb; skips the tuner)")
    p.add_argument("--pipeline-mode", type=int, default=None, help="with an explicit bucket size: 0 or 1")
    p.add_argument("--wait-stride", type=int, default=None, help="with an explicit bucket size: cross-step wait stride")
    p.add_argument("--allreduce-group", type=int, default=None, help="with an explicit bucket size: all-reduce group")
    p.add_argument("--allreduce-algorithm", type=int, default=None,
                   help="with an explicit bucket size: 0 all-reduce, 1 peer-read, 2 reduce-scatter + all-gather")
    p.add_argument("--enqueue-threads", type=int, default=None,
                   help="one process over N devices, explicit bucket size: 0 one thread (the reference's), 1 per device")
    p.add_argument("--watchdog-scale", type=float, default=1.0,
                   help="multiplies every phase deadline of the watchdog (0 = off); on a missed deadline the run "
                        "writes every thread's stack to stderr and exits with code 3")
    p.add_argument("--watchdog-selftest", type=float, default=0.0, help=argparse.SUPPRESS)
    p.add_argument("--hw-queues", type=int, default=None,
                   help="GPU_MAX_HW_QUEUES for this run (default: the environment's, HIP's 4 when unset)")
    p.add_argument("--no-peer-ipc", action="store_true",
                   help="one process per GPU: skip the peer-read form's block (IPC mapping, its tuner candidates "
                        "and timed region), which otherwise runs after the RCCL forms' timed region")
    p.add_argument("--peer-ipc-deadline", type=float, default=300.0,
                   help="watchdog deadline (s, times --watchdog-scale) of the peer-read form's IPC mapping")
    p.add_argument("--watchdog-selftest-result", type=float, default=0.0, help=argparse.SUPPRESS)
    p.add_argument("--selftest-raise", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--selftest-sigterm", choices=("main", "thread", "unpublished", "launcher"), default=None,
                   help=argparse.SUPPRESS)
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes per launch (written by scripts/pmc_traffic.py)")
    return p.parse_args()


SYSCALLS = {"0": "read", "1": "write", "7": "poll", "16": "ioctl", "23": "select", "24": "sched_yield",
            "35": "nanosleep", "42": "connect", "43": "accept", "45": "recvfrom", "46": "sendmsg", "47": "recvmsg",
            "61": "wait4", "202": "futex", "230": "clock_nanosleep", "232": "epoll_wait", "270": "pselect6", "271": "ppoll",
            "281": "epoll_pwait"}


def thread_states() -> str:
    """Every thread of this process as the kernel sees it (/proc/self/task:
    name, wait channel, current system call): faulthandler shows Python
    frames only, so a thread stuck inside a native call (a HIP runtime call,
    a socket read) would otherwise leave no trace of where it waits."""
    lines = []
    try:
        tids = sorted(os.listdir("/proc/self/task"), key=int)
    except OSError as e:
        return f"  /proc/self/task unreadable: {e}\n"
    for tid in tids:
        def rd(name):
            try:
                with open(f"/proc/self/task/{tid}/{name}") as f:
                    return f.read().strip()
            except OSError as e:
                return f"?({e.errno})"
        sc = rd("syscall").split()
        call = sc[0] if sc else "?"
        call += f" ({SYSCALLS[call]})" if call in SYSCALLS else (" (user space)" if call == "running" else "")
        lines.append(f"  tid {tid} comm={rd('comm')} wchan={rd('wchan') or '0'} syscall={call}")
    return "\n".join(lines) + "\n"


class Watchdog:
    """Deadlines per phase of the run, so a run that stalls (a collective
    that never completes, a tuner candidate that hangs, a lost device) ends
    with a diagnosis instead of silently: a daemon thread checks the current
    phase's deadline and, once it passes, writes which phase and which tuner
    candidate were in flight, the last completed phase, every thread's state
    as the kernel sees it (wait channel, system call) and every thread's
    Python stack (faulthandler) to stderr, then leaves with os._exit (no
    restart, no exec).  Once the first timed region has produced the line
    (`publish`), a missed deadline prints that line on rank 0 first, with
    `incomplete_phase` naming what did not finish, and the exit code is 0;
    before that it is 3 and stdout stays empty.  Every phase is one stderr
    line on rank 0.  `catch_sigterm` extends the same to the launcher's
    SIGTERM.  Exactly one of these endings (or main's own print) prints."""

    def __init__(self, scale: float, rank: int):
        self.scale, self.rank = scale, rank
        self.phase, self.deadline, self.seconds, self.last_done = None, None, 0.0, None
        self.result, self.out = None, None
        self.ending, self.wake = False, None
        # reentrant: the main thread's SIGTERM handler may run inside a `with self.lock`
        self.lock = threading.RLock()
        if scale > 0:
            threading.Thread(target=self._watch, name="bench-watchdog", daemon=True).start()

    def catch_sigterm(self) -> None:
        """torch.distributed.run ends every rank with SIGTERM once one rank
        fails (SIGKILL after its grace period): on rank 0 that must not cost a
        line already assembled.  Python's C-level handler writes the signal's
        number to the wakeup fd in whichever thread the kernel picks, so the
        watchdog thread prints the line even while the main thread sits in a
        blocking native call (a HIP synchronize, a collective).  The
        Python-level handler (main thread, at any bytecode boundary, maybe in
        the middle of a write to stderr) only keeps the default action away.
        Before the line exists the rank ends as SIGTERM would (exit 143).
        Main thread only; needs the watchdog thread (scale > 0)."""
        if self.scale <= 0:
            return
        r, w = socket.socketpair()
        r.setblocking(False)
        w.setblocking(False)
        self.wake = (r, w)
        signal.set_wakeup_fd(w.fileno(), warn_on_full_buffer=False)
        signal.signal(signal.SIGTERM, lambda signum, frame: None)

    def _claim_end(self):
        """(phase, last done, published) for the one ending that prints, else None."""
        with self.lock:
            if self.ending:
                return None
            self.ending, self.deadline = True, None
            return self.phase, self.last_done, self.result is not None

    def finish(self) -> bool:
        """main is about to print the complete line: no other ending may."""
        return self._claim_end() is not None

    def _terminated(self) -> None:
        claim = self._claim_end()
        if claim is None:
            return  # another ending (or main's print) is already under way
        phase, done, published = claim
        sys.stderr.write(f"[bench] rank {self.rank}: SIGTERM in phase '{phase}'; thread states follow\n")
        sys.stderr.write(thread_states())
        sys.stderr.flush()
        if published and self.rank == 0:
            try:
                print(self._line(phase, 0.0, done, "SIGTERM", how="was ended by SIGTERM (the launcher ends every "
                                 "rank once one fails)"), file=self.out, flush=True)
            except Exception as e:  # noqa: BLE001 -- never let the line itself keep the rank alive
                sys.stderr.write(f"[bench] could not print the line: {e!r}\n")
                sys.stderr.flush()
        os._exit(0 if published else 128 + signal.SIGTERM)

    def enter(self, name: str, seconds: float) -> None:
        with self.lock:
            if self.phase is not None:
                self.last_done = self.phase
            self.phase, self.seconds = name, seconds * self.scale
            self.deadline = time.monotonic() + self.seconds if self.scale > 0 else None
        if self.rank == 0:
            log(f"[bench] phase {name}" + (f" (deadline {self.seconds:.0f} s)" if self.scale > 0 else ""))
        kill = os.environ.get("CBX_BENCH_FAULT_KILL")  # test switch "rank:phase": that rank crashes there
        if kill and kill.partition(":")[0] == str(self.rank) and kill.partition(":")[2] == name:
            os.kill(os.getpid(), signal.SIGKILL)

    def publish(self, result: dict, out) -> None:
        """The line as assembled so far (the main thread keeps adding to it)."""
        with self.lock:
            self.result, self.out = result, out

    def fail_now(self, exc: BaseException) -> None:
        """A phase after the first timed region raised `exc`: print the
        published line (rank 0) naming the phase and the error, and leave
        with 0, as for a missed deadline.  Before the line exists, re-raise."""
        with self.lock:
            published = self.result is not None
        if not published:
            raise exc
        claim = self._claim_end()
        if claim is None:  # a SIGTERM ending is printing: let it finish the process
            time.sleep(60)
            os._exit(0)
        phase, done, _ = claim
        error = f"{type(exc).__name__}: {exc}"
        sys.stderr.write(f"[bench] rank {self.rank}: phase '{phase}' failed: {error}\n")
        sys.stderr.flush()
        if self.rank == 0:
            print(self._line(phase, 0.0, done, error), file=self.out, flush=True)
        os._exit(0)

    def _line(self, phase, secs, done, error=None, how=None):
        """The published line with the phase that missed its deadline (or raised, or was ended)."""
        import copy
        for _ in range(5):  # the main thread may be adding a key right now
            try:
                r = copy.deepcopy(self.result)
                break
            except RuntimeError:
                time.sleep(0.05)
        else:
            r = {k: self.result[k] for k in ("metric", "value", "unit") if k in self.result}
        how = how or (f"raised {error}" if error else f"missed its {secs:.0f} s deadline")
        r["incomplete_phase"] = {
            "phase": phase, "deadline_s": None if error else round(secs, 1), "error": error, "last_completed": done,
            "note": f"this phase came after the timed region that set `value` and {how}; the run ended here "
                    "(bench.py), so later fields are absent"}
        c = r.get("config", {})
        if "IPC mapping" in str(phase) and c.get("peer_ipc") in ("mapping", "pending (after the timed region)", None):
            c["peer_ipc"] = f"failed: '{phase}' {how}" + ("" if error else " (watchdog)")
        return json.dumps(r)

    def _watch(self) -> None:
        while True:
            wake = self.wake
            if wake is None:
                time.sleep(0.2)
            elif select.select([wake[0]], [], [], 0.2)[0]:
                try:
                    got = wake[0].recv(256)
                except BlockingIOError:
                    got = b""
                if int(signal.SIGTERM) in got:
                    self._terminated()
            with self.lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                phase, secs, done = self.phase, self.seconds, self.last_done
                published = self.result is not None
            if late and self._claim_end() is not None:
                sys.stderr.write(f"[bench] WATCHDOG rank {self.rank}: phase '{phase}' missed its {secs:.0f} s "
                                 f"deadline; last completed phase: '{done}'; thread states and stacks follow\n")
                sys.stderr.write(thread_states())
                sys.stderr.flush()
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                if published and self.rank == 0:
                    try:
                        print(self._line(phase, secs, done), file=self.out, flush=True)
                    except Exception as e:  # never let the diagnosis itself hang or raise past _exit
                        sys.stderr.write(f"[bench] WATCHDOG could not print the line: {e!r}\n")
                        sys.stderr.flush()
                os._exit(0 if published else 3)


def free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def lib_buckets(n: int, bucket_elems: int, G: int) -> int:
    """The bucket count the library cuts n elements into (SplitStep::prepare_common)."""
    pad = 1024
    n4 = -(-(-(-n // 4)) // pad) * pad
    if bucket_elems <= 0:
        if G <= 1:
            return 1
        b4 = -(-(n4 // 8) // pad) * pad
    else:
        b4 = -(-(bucket_elems // 4) // pad) * pad
    if b4 <= 0 or b4 > n4:
        b4 = n4
    return -(-n4 // b4)


def alg_bytes(n, R, momentum, G):
    m = 1 if momentum > 0 else 0
    if G == 1:
        return (12 * R + 8 + 8 * m) * n, (12 * R + 8 + 8 * m) * n
    a = (12 * R + 8) * n
    return a + (12 + 8 * m) * n, a


def cpu_baseline_threads(args, n_full, threads):
    """Same replay with OpenBLAS on `threads` threads (no pinning): the
    'all cores' row of BASELINE.md 3, capped at the GPU box's CPU share."""
    from oracle import oracle as O
    n = min(args.cpu_elements, n_full) if args.cpu_elements > 0 else n_full
    O.blas_open()
    O.blas_set_threads(threads)
    st = O.make_state(n, 1, args.replicas, args.alpha, args.momentum, threads=threads)
    try:
        O.sma_step_blas(st)
        steps, t0 = 0, O.now()
        while True:
            O.sma_step_blas(st)
            steps += 1
            el = O.now() - t0
            if el >= args.cpu_seconds / 2:
                break
    finally:
        O.blas_set_threads(1)
    b, _ = alg_bytes(n, args.replicas, args.momentum, 1)
    return {"value": round(b * steps / el / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{n} fp32 elements x {args.replicas} replicas, {steps} steps in {el:.1f} s, "
                      f"OpenBLAS on {threads} threads"}


def cpu_c1(seconds=3.0):
    """BASELINE configs[0] (C1): LeNet (n = 1,111,946), 2 replicas, alpha 0.1,
    mu 0 -- the reference's own CPU-runnable case -- replayed on OpenBLAS,
    1 thread pinned to core 0, at full size."""
    from oracle import oracle as O
    n, R = 1_111_946, 2
    O.blas_open()
    O.blas_set_threads(1)
    st = O.make_state(n, 1, R, 0.1, 0.0)
    O.bind_core(0)
    try:
        O.sma_step_blas(st)
        steps, t0 = 0, O.now()
        while True:
            O.sma_step_blas(st)
            steps += 1
            el = O.now() - t0
            if el >= seconds:
                break
    finally:
        O.unbind()
    b = (12 * R + 8) * n
    return {"value": round(b * steps / el / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "ms_per_step": round(el * 1e3 / steps, 3),
            "sample": f"C1 LeNet n={n}, 2 replicas, mu 0, full size, {steps} steps in {el:.1f} s"}


def cpu_model() -> str:
    """The host CPU's model name (/proc/cpuinfo), for the baseline's record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, n_full):
    """The reference's call sequence (memset, memcpy + 3 saxpy per replica,
    momentum, apply) on OpenBLAS, 1 thread bound to core 0 like TheCPU.bind(0)
    (clib-multigpu/CPU.c:39-52, BLAS.c:32), on a bounded sample."""
    from oracle import oracle as O
    n = min(args.cpu_elements, n_full) if args.cpu_elements > 0 else n_full
    lib = O.blas_open()
    O.blas_set_threads(1)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    st = O.make_state(n, 1, args.replicas, args.alpha, args.momentum, threads=threads)  # inputs only; timed on 1 thread
    O.bind_core(0)
    try:
        O.sma_step_blas(st)  # warm
        steps, t0 = 0, O.now()
        while True:
            O.sma_step_blas(st)
            steps += 1
            el = O.now() - t0
            if el >= args.cpu_seconds:
                break
    finally:
        O.unbind()
    b, _ = alg_bytes(n, args.replicas, args.momentum, 1)
    return {"value": round(b * steps / el / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{n} fp32 elements x {args.replicas} replicas, momentum {args.momentum}, {steps} steps "
                      f"in {el:.1f} s; reference BLAS call sequence (sma.c:13-231) on OpenBLAS "
                      f"({os.path.basename(lib)}), 1 thread pinned to core 0, same algorithmic-bytes formula"}


def bench_optimiser(gpu, torch, n, args, rounds=10):
    """the fused replica optimiser step (kernels/optimisers/
    sma.cu:3-100) of every replica, back to back on one torch stream.  Reads
    w, g, last and writes s, w, g, last: (12 + 16) n bytes per launch with
    momentum and weight decay (the reference issues 6 ops moving ~60n B)."""
    stream = torch.cuda.Stream()
    task = 0
    with torch.cuda.stream(stream):
        for i in range(args.replicas):  # warm
            gpu.replica_optimise(i, task, stream.cuda_stream)
            task += 1
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(rounds):
            for i in range(args.replicas):
                gpu.replica_optimise(i, task, stream.cuda_stream)
                task += 1
        e1.record(stream)
    e1.synchronize()
    gpu.wait()
    launches = rounds * args.replicas
    ms = e0.elapsed_time(e1) / launches
    m = 1 if args.momentum > 0 else 0
    b = (12 + 16) * n if m else 16 * n + 4 * n
    return {"kernel": "sma_optimise_kernel", "launch_ms_mean": round(ms, 4), "launches": launches,
            "alg_bytes_per_launch": b, "achieved_GBs": round(b / (ms * 1e-3) / 1e9, 1),
            "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "timed": "torch events around back-to-back launches on one stream (includes launch gaps)"}


def bench_seam(torch, n, args, steps=20):
    """The sma.c seam (cbx_sma_plan_step): the same step
    over buffers the caller owns -- here one torch allocation per buffer,
    exactly n floats each, as the reference's model manager allocates them --
    so one launch of the fused kernel runs the whole-trip bulk and, on extra
    workgroups of the same launch, the last elements.  Timed with torch
    events around back-to-back steps on the caller's stream (launch gaps
    included)."""
    from crossbow_amd.seam import SmaPlan
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(SEED)
    z = torch.randn(n, device=dev, generator=gen) * 0.05
    last = torch.randn(n, device=dev, generator=gen) * 0.001
    s = [z + 0.01 * torch.randn(n, device=dev, generator=gen) for _ in range(args.replicas)]
    w = [si + 0.001 * torch.randn(n, device=dev, generator=gen) for si in s]
    mom = args.momentum
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    with SmaPlan([0], n) as plan:
        reps = [(0, w[i].data_ptr(), s[i].data_ptr(), 1, 0) for i in range(args.replicas)]
        lp = [last.data_ptr()] if mom > 0 else None

        def one():
            plan.step([stream.cuda_stream], [z.data_ptr()], lp, reps, args.alpha, mom)
        for _ in range(3):
            one()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            one()
        e1.record(stream)
        e1.synchronize()
    ms = e0.elapsed_time(e1) / steps
    b, _ = alg_bytes(n, args.replicas, mom, 1)
    return {"entry": "cbx_sma_plan_step", "step_ms_mean": round(ms, 4), "steps": steps, "alg_bytes_per_step": b,
            "achieved_GBs": round(b / (ms * 1e-3) / 1e9, 1), "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "buffers": "caller-owned torch allocations of exactly n floats (no padding, no slot stagger)",
            "timed": "torch events around back-to-back steps on the caller's stream (one launch per step: bulk + tail workgroups; gaps included)"}


RCCL_TUNING_RE = re.compile(r"(\w+): (\d+) Bytes -> Algo (\S+) proto (\S+) channel\{Lo\.\.Hi\}=\{(\d+)\.\.(\d+)\}")


def rccl_tuning(path):
    """RCCL's per-collective tuning choices (NCCL_DEBUG=INFO,
    NCCL_DEBUG_SUBSYS=TUNING): one entry per (collective, bytes) with the
    algorithm, protocol and channel range RCCL picked and how often."""
    seen = {}
    try:
        with open(path, errors="replace") as f:
            for line in f:
                m = RCCL_TUNING_RE.search(line)
                if not m:
                    continue
                key = (m.group(1), int(m.group(2)), m.group(3), m.group(4), int(m.group(5)), int(m.group(6)))
                seen[key] = seen.get(key, 0) + 1
    except OSError:
        return None
    return [{"collective": k[0], "bytes": k[1], "algo": k[2], "proto": k[3], "channels": [k[4], k[5]], "calls": v}
            for k, v in sorted(seen.items(), key=lambda kv: (kv[0][0], kv[0][1]))]


def span_stats(gpu, _lib, locals_, steps):
    """Per-step summed busy spans of kernels A, collectives and kernels B over
    the last `steps` steps on every local device (cbx_timing_history: for a
    pipelined step each dispatch's stop minus the latest event that bounded
    its start; for a one-bucket step the exact START..A / A..AR / AR..B).
    Returns (A, coll, B) lists of per-step ms (device-major), None if any
    step kept no spans."""
    out = []
    for which in (_lib.T_KERNEL, _lib.T_ALLREDUCE, _lib.T_APPLY):
        vals = []
        for k in range(locals_):
            h = list(gpu.timing_history(which, local=k)[-steps:])
            if len(h) < steps or any(x <= 0 for x in h):
                return None
            vals += h
        out.append(vals)
    return tuple(out)


def base_identity(gpu, world):
    """After the timed region at G > 1: every GPU must hold a bitwise
    identical base model z and momentum `last`, because every GPU applies the
    same reduced difference D (sma.c:168-174; the tests' cross-rank check).
    A digest of each local device's z and last, gathered over the ranks
    (gloo) and compared, plus a finiteness check: a collective or peer read
    that ran out of order would show up here, so a fast but wrong
    configuration cannot pass as a measurement.  No oracle is involved."""
    import hashlib

    import numpy as np
    from crossbow_amd import BUF_DATA, BUF_LAST
    local = []
    finite = True
    top = 0.0
    for g in gpu.local_devices():
        h = hashlib.blake2b(digest_size=16)
        for kind in (BUF_DATA, BUF_LAST):
            a = gpu.base_read(g, kind)
            ok = bool(np.isfinite(a).all())
            finite = finite and ok
            top = max(top, (float(np.max(np.abs(a))) if a.size else 0.0) if ok else math.inf)
            h.update(a.view(np.uint8))
        local.append((int(g), h.hexdigest()))
    every = [local]
    if world > 1:
        import torch.distributed as dist
        every = [None] * world
        dist.all_gather_object(every, local)
    digests = {g: d for part in every for g, d in part}
    finite = all_ranks(finite, world)
    from crossbow_amd import dist as D
    top = D.max_over_ranks(top, world)
    return {"z_last_identical_on_every_gpu": len(set(digests.values())) == 1, "finite": finite,
            "max_abs_value": top if math.isfinite(top) else None,  # None: not finite (strict JSON has no inf)
            "gpus_checked": len(digests), "digest": sorted(set(digests.values()))[0] if digests else None,
            "checked": "blake2b of each GPU's base model z and momentum last after the timed region, compared "
                       "across every GPU (every GPU applies the same D, sma.c:168-174)"}


def state_max_abs(gpu, world):
    """max |value| of z and last over every GPU (the fresh state's yardstick
    for `dynamics`)."""
    import numpy as np
    from crossbow_amd import BUF_DATA, BUF_LAST
    top = 0.0
    for g in gpu.local_devices():
        for kind in (BUF_DATA, BUF_LAST):
            a = gpu.base_read(g, kind)
            top = max(top, float(np.max(np.abs(a))) if a.size else 0.0)
    from crossbow_amd import dist as D
    return D.max_over_ranks(top, world)


def sma_dynamics(alpha: float, momentum: float, replicas_total: int) -> dict:
    """How the bench's values evolve, whatever computes them.  The bench keeps
    every snapshot s_i fixed between steps (no optimiser runs), so the
    deviation e = z - mean(s) and the momentum `last` of the SMA step
    (sma.c:63-174: D = alpha * sum_i (s_i - z) = -alpha N e; last' = mu last +
    D; z' = z + last') follow the linear map [[1 - alpha N, mu], [-alpha N,
    mu]] (without momentum, e' = (1 - alpha N) e).  Its spectral radius is
    the growth per step; it exceeds 1 exactly when alpha N > 2 (1 + mu):
    3.8 at mu = 0.9.  C3 weak-scaled to 8 GPUs (8 x 8 replicas, alpha 0.1)
    has alpha N = 6.4 and radius 4.29, so the values grow ~4.3x per step from
    any start; the reference's own run (8 GPUs x 2, resnet-50.sh:74-102) and
    C5 (8 x 4) are inside the bound.  Re-snapshotting s_i <- w_i every step
    does not change the verdict (tests/test_bench_cpu.py).  The arithmetic per
    element, and so the timing, is the same whatever the values."""
    import numpy as np
    aN = alpha * replicas_total
    if momentum > 0:
        rho = float(max(abs(np.linalg.eigvals(np.array([[1.0 - aN, momentum], [-aN, momentum]])))))
    else:
        rho = abs(1.0 - aN)
    return {"alpha_times_replicas": round(aN, 4), "stability_bound": round(2 * (1 + max(momentum, 0.0)), 4),
            "spectral_radius_per_step": round(rho, 4), "bounded": rho <= 1.0 + 1e-9,
            "model": "fixed snapshots s_i: e = z - mean(s), [e, last]' = [[1 - aN, mu], [-aN, mu]] [e, last]"}


def form_agreement(gpu, world, step, chosen, one_bucket, algorithm_name):
    """After the timed region at G > 1, when the measured configuration is not
    the reference's own collective: one more step in that configuration, and
    the same step from the same state through one RCCL all-reduce of the
    whole buffer, in order (synch/common.c:3-57).  z and last must agree
    within the G > 1 tolerance (rtol 1e-5, atol 1e-6, BASELINE.md 2.5: the
    collectives sum in different orders; a peer-read sum and a 2-rank
    all-reduce are the same sum, so G = 2 is bit for bit).  The state is
    put back afterwards.  With `identity` this catches a configuration that
    is fast because it is wrong, on the hardware it ran on, without the
    oracle."""
    import numpy as np
    from crossbow_amd import BUF_DATA, BUF_LAST
    devs, reps = list(gpu.local_devices()), list(gpu.local_replicas())
    gpu.wait()
    base = {(g, k): gpu.base_read(g, k) for g in devs for k in (BUF_DATA, BUF_LAST)}
    ws = {i: gpu.replica_read(i, BUF_DATA) for i in reps}

    def restore():
        for (g, k), a in base.items():
            gpu.base_write(g, k, a)
        for i, a in ws.items():
            gpu.replica_write(i, BUF_DATA, a)

    def result():
        return {(g, k): gpu.base_read(g, k) for g in devs for k in (BUF_DATA, BUF_LAST)}

    step()
    gpu.wait()
    got = result()
    restore()
    gpu.set_allreduce_algorithm(0)
    gpu.set_bucket_elements(one_bucket)
    gpu.set_pipeline_mode(0)
    step()
    gpu.wait()
    ref = result()
    restore()
    gpu.set_allreduce_algorithm(chosen["algorithm"])
    gpu.set_bucket_elements(chosen["bucket_elements"])
    gpu.set_pipeline_mode(chosen["mode"])
    gpu.wait()
    diff = max(float(np.max(np.abs(got[key].astype(np.float64) - ref[key]))) for key in got)
    scale = max(float(np.max(np.abs(ref[key]))) for key in ref)  # the diff's yardstick
    close = all(np.allclose(got[key], ref[key], rtol=1e-5, atol=1e-6) for key in got)
    same = all(np.array_equal(got[key].view(np.uint32), ref[key].view(np.uint32)) for key in got)
    from crossbow_amd import dist as D
    scale = D.max_over_ranks(scale, world)
    # A tolerance relative to values far beyond the fresh state's (|z| ~ 0.3)
    # says nothing: at 1.7e13 rtol 1e-5 forgives 1.7e8 (VERDICT r04 Weak #3).
    vacuous = not scale <= AGREEMENT_MAX_ABS
    return {"configuration": f"{algorithm_name}, {chosen['buckets']} bucket(s), mode {chosen['mode']}",
            "against": "one RCCL all-reduce of the whole buffer, in order (synch/common.c:3-57)",
            "from": "fresh synthetic state (one step), so the tolerance is measured against values of order 1",
            "max_abs_diff": D.max_over_ranks(diff, world), "max_abs_value": scale,
            "within_tolerance": all_ranks(close, world) and not vacuous, "vacuous": vacuous,
            "bitwise_equal": all_ranks(same, world), "tolerance": "rtol 1e-5, atol 1e-6 (BASELINE.md 2.5)"}


# Above this the agreement check's relative tolerance is vacuous (form_agreement).
AGREEMENT_MAX_ABS = 1e3


def block_identity(gpu, world, step, chosen, one_bucket, peer_only, peer_algo, wd, blk=None, dynamics=None):
    """After a timed block at G > 1: z and last bitwise identical on every GPU
    (base_identity), and, unless the block ran the reference's own in-order
    all-reduce, one step of the block's configuration against one in-order
    all-reduce of the same step from a FRESH synthetic state
    (form_agreement).  `trusted`: both hold, finitely and not vacuously.
    `dynamics` (sma_dynamics) with the block's fresh-state max |value|: the
    observed growth per step since the fresh state, beside the predicted one."""
    idn = base_identity(gpu, world)
    if dynamics is not None and blk is not None and blk.get("fresh_max_abs"):
        k = blk["steps_since_fresh"]
        top = idn["max_abs_value"]
        ratio = top / blk["fresh_max_abs"] if top is not None else math.inf
        idn["dynamics"] = dict(dynamics, fresh_max_abs=blk["fresh_max_abs"], steps_since_fresh=k,
                               observed_growth_per_step=(round(ratio ** (1.0 / k), 4)
                                                         if ratio > 0 and k > 0 and math.isfinite(ratio) else None))
        # Beyond fp32's range by the predicted growth (from the fresh state's
        # largest |value|, an upper estimate of the diverging mode's start):
        # non-finite values are then the update's own, not a fault, and do
        # not cost the block its trust (identity and agreement still hold).
        predicted = math.log10(blk["fresh_max_abs"]) + k * math.log10(max(dynamics["spectral_radius_per_step"], 1e-30))
        idn["dynamics"]["predicted_log10_max_abs"] = round(predicted, 2)
        idn["dynamics"]["overflow_expected"] = predicted > math.log10(3.4e38)
    if not peer_only and (chosen["algorithm"] != 0 or chosen["buckets"] != 1):
        wd.enter("agreement with the all-reduce", 300)
        gpu.wait()
        gpu.fill_synthetic(SEED)
        idn["vs_all_reduce"] = form_agreement(gpu, world, step, chosen, one_bucket,
                                              "peer-read two-shot" if chosen["algorithm"] == peer_algo else
                                              "reduce-scatter+all-gather" if chosen["algorithm"] == 2 else "all-reduce")
    agree = idn.get("vs_all_reduce")
    overflow_expected = bool(idn.get("dynamics", {}).get("overflow_expected"))
    idn["trusted"] = bool(idn["z_last_identical_on_every_gpu"] and (idn["finite"] or overflow_expected) and
                          (agree is None or agree["within_tolerance"]))
    return idn


def all_ranks(flag: bool, world: int) -> bool:
    """Logical AND of a flag over the ranks."""
    if world <= 1:
        return flag
    from crossbow_amd import dist as D
    return D.max_over_ranks(0.0 if flag else 1.0, world) == 0.0


def rccl_tuning_run(args, G, single, cfg, wd):
    """RCCL's own algorithm / protocol / channel choices for the collectives
    of the chosen configuration, from a separate short run (3 steps) with
    RCCL's TUNING log on: the log writes a line per collective on the host's
    enqueue path, so the measured run keeps it off.  The same process form
    and device selection as this run; returns (entries or None, source)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(G), "--steps", "3", "--warmup", "1",
           "--calib-steps", "1", "--no-cpu-baseline", "--no-staged", "--no-copy-ceiling", "--no-optimiser",
           "--no-seam", "--rccl-tuning-log", "--no-rccl-tuning-run", "--watchdog-scale", str(args.watchdog_scale),
           "--model", args.model, "--replicas", str(args.replicas), "--alpha", str(args.alpha),
           "--momentum", str(args.momentum), "--bucket-elements", str(cfg["bucket_elements"]),
           "--pipeline-mode", str(cfg["mode"]), "--wait-stride", str(cfg["stride"]),
           "--allreduce-group", str(cfg["group"]), "--allreduce-algorithm", str(cfg["algorithm"])]
    if args.rehearse_one_gpu:
        cmd.append("--rehearse-one-gpu")
    if args.hw_queues is not None:
        cmd += ["--hw-queues", str(args.hw_queues)]
    env = {k: v for k, v in os.environ.items() if not k.startswith(("NCCL_DEBUG", "NCCL_HOSTID"))}
    if single:
        cmd += ["--single-process"]
        if cfg.get("enqueue_threads") is not None:
            cmd += ["--enqueue-threads", str(cfg["enqueue_threads"])]
    else:
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                  "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        env = {k: v for k, v in env.items() if not k.startswith("TORCHELASTIC")}
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(G),
               "--master-addr", "127.0.0.1", "--master-port", str(free_port())] + cmd[1:]
    wd.enter("rccl tuning run", 420)
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=360)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        return None, "the separate tuning-log run timed out (360 s)"
    if p.returncode != 0:
        return None, f"the separate tuning-log run failed (rc {p.returncode}): {err.strip()[-300:]}"
    try:
        line = [ln for ln in out.splitlines() if ln.strip()][-1]
        t = json.loads(line)["allreduce"]["rccl_tuning"]
    except (IndexError, KeyError, ValueError) as e:
        return None, f"the separate tuning-log run printed no tuning table ({e})"
    return t, ("RCCL's own log (NCCL_DEBUG=INFO, NCCL_DEBUG_SUBSYS=TUNING) of a separate 3-step run of the same "
               "configuration and process form: the timed steps above ran without the log")


def apply_config(gpu, chosen, single):
    """Put a measured configuration of the G > 1 pipeline back on the context."""
    gpu.set_allreduce_algorithm(chosen["algorithm"])
    gpu.set_bucket_elements(chosen["bucket_elements"])
    gpu.set_pipeline_mode(chosen["mode"])
    gpu.set_cross_wait_stride(chosen["stride"])
    gpu.set_allreduce_group(chosen["group"])
    if single and chosen.get("enqueue_threads") is not None:
        gpu.set_enqueue_threads(chosen["enqueue_threads"])


def timed_block(gpu, torch, D, args, world, step, wd, refill, label=""):
    """W warm-up steps, then EXACTLY K timed steps bracketed by a barrier and
    a device synchronisation on both sides; the wall time is the max over
    ranks.  `refill`: fresh synthetic state first, and its max |value| kept
    for `dynamics` (G > 1: with the snapshots s_i fixed, alpha N above
    2 (1 + mu) makes the values grow by sma_dynamics' radius per step, 4.3x
    at 8 GPUs x 8 replicas; the arithmetic per element is the same whatever
    the values)."""
    from crossbow_amd import _lib
    fresh = None
    if refill:
        gpu.wait()
        gpu.fill_synthetic(SEED)
        fresh = state_max_abs(gpu, world)
    wd.enter("warm-up" + label, 180)
    for _ in range(args.warmup):
        step()
    gpu.wait()
    torch.cuda.synchronize()
    D.barrier(world)
    wd.enter("timed region" + label, 120 + 0.2 * args.steps)
    host_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        h0 = time.perf_counter()
        step()
        host_ms.append((time.perf_counter() - h0) * 1e3)
    gpu.wait()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    D.barrier(world)
    el = D.max_over_ranks(el, world)
    wd.enter("timing read-back" + label, 120)
    return {"el": el, "host_ms": host_ms, "steps_ms": list(gpu.timing_history(_lib.T_STEP)[-args.steps:]),
            "fresh_max_abs": fresh, "steps_since_fresh": args.warmup + args.steps}


def block_fields(gpu, D, args, world, n, G, nlocal, split, blk, chosen, tuning, calib, rehearse):
    """The bench line's fields that come from one timed block: `value`,
    `ms_per_step`, the configuration that ran, `roofline` (the dominant
    kernel's mean launch from HIP events on its own dispatches in the timed
    region), the link rate of the collectives and the host's enqueue time."""
    from crossbow_amd import _lib
    ar_algo = chosen["algorithm"]
    step_bytes, kernel_bytes = alg_bytes(n, args.replicas, args.momentum, 2 if split else 1)
    form = ("peer-read two-shot" if ar_algo == _lib.ALLREDUCE_PEER else
            "reduce-scatter+all-gather" if ar_algo == 2 else "all-reduce")
    spans = span_stats(gpu, _lib, nlocal, args.steps) if split else None
    out = {
        "value": round(step_bytes * G * args.steps / blk["el"] / 1e9, 2),
        "ms_per_step": round(blk["el"] * 1e3 / args.steps, 4),
        "config": {
            # SURVEY 8(d)'s per-GPU bytes of the step, the unit `value` counts in
            # whichever collective form runs; the reduce-scatter form moves fewer
            # (kernel B without momentum plus the momentum pass on 1/G), shown apart
            "bytes_per_step_per_gpu": step_bytes,
            "hbm_bytes_moved_per_step_per_gpu": (
                step_bytes if not (split and ar_algo == 2) else
                (12 * args.replicas + 8) * n + 12 * n + (12 * n // G if args.momentum > 0 else 0)),
            "buckets": chosen["buckets"] if split else None,
            "pipeline_mode": chosen["mode"] if split else None,
            "cross_wait_stride": chosen["stride"] if split else None,
            "allreduce_group": chosen["group"] if split else None,
            "allreduce_algorithm": form if split else None,
            "enqueue_threads": chosen["enqueue_threads"] if G > 1 and nlocal > 1 else None,
            "bucket_tuning_ms_per_step": tuning.table if tuning else None,
            "tuning_errors": tuning.errors if tuning else None,
        },
    }
    kname = "sma_fused_kernel" if not split else "sma_accumulate_kernel"
    traffic, traffic_note = None, None
    try:
        from crossbow_amd.build import code_object_digest
        running = code_object_digest(_lib.LIB_PATH)
        with open(args.traffic_json) as f:
            tj = json.load(f)
        key = f"{kname}/{args.model}/R{args.replicas}/m{1 if args.momentum > 0 else 0}"
        entry = tj.get(key)
        if entry is None:
            traffic_note = f"no PMC measurement for {key} in {os.path.relpath(args.traffic_json, ROOT)}"
        elif entry.get("code_object_sha256") != running:
            # a measurement of another build of the kernels says nothing about this one
            traffic_note = (f"stale: measured on code object {str(entry.get('code_object_sha256'))[:12]}, "
                            f"running {running[:12]}; re-run scripts/gpu_pmc.sh")
        else:
            traffic = entry.get("hbm_bytes_per_launch")
            traffic_note = (f"PMC FETCH_SIZE x2 + WRITE_SIZE, separate passes, of this code object "
                            f"({running[:12]}); traffic / alg = {traffic / kernel_bytes:.4f}")
    except (OSError, ValueError) as e:
        traffic_note = f"unavailable: {e}"

    def roofline(kern, timed_in, kbytes=kernel_bytes, kernel=kname, mean_ms=None):
        kern_ms = statistics.mean(kern) if mean_ms is None else mean_ms
        achieved = kbytes / (kern_ms * 1e-3) / 1e9
        return {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": kbytes,
                "launch_ms_mean": round(kern_ms, 4), "launch_ms_median": round(statistics.median(kern), 4),
                "launches": len(kern), "timed_in": timed_in}

    coll_busy = None
    if not split:
        out["roofline"] = roofline(list(gpu.timing_history(_lib.T_KERNEL)[-args.steps:]), "timed region")
    else:
        # N > 1: the kernels as they ran in the timed region, beside the
        # collectives (per step: kernel A's dispatches' summed busy spans);
        # the calibration's one-bucket, in-order figure is kept apart.
        b_bytes = (12 + 8 * (1 if args.momentum > 0 else 0)) * n
        unpiped = roofline(calib["kernel"], "calibration steps (one bucket, in order)")
        # the slowest rank's mean times set the roofline and the link rate (max
        # over ranks; every rank takes part in both reductions)
        a_max = D.max_over_ranks(statistics.mean(spans[0]) if spans else -1.0, world)
        coll_max = D.max_over_ranks(statistics.mean(spans[1]) if spans else -1.0, world)
        if spans is not None:
            a_ms, coll_ms, b_ms = spans
            out["roofline"] = roofline(
                a_ms, "timed region: per step, the summed busy spans of kernel A's dispatches (each its stop minus "
                      "the latest event bounding its start: an upper bound incl. dispatch latency), beside the "
                      f"collectives; {'mean over the local devices, ' if nlocal > 1 else ''}slowest rank",
                mean_ms=a_max)
            out["roofline"]["apply_kernel"] = roofline(b_ms, "timed region (summed busy spans of kernel B)",
                                                       b_bytes, "sma_apply_kernel")
            ab = [x + y for x, y in zip(a_ms, b_ms)]
            out["roofline"]["a_plus_b"] = roofline(ab, "timed region (kernels A + B)", kernel_bytes + b_bytes,
                                                   "sma_accumulate_kernel+sma_apply_kernel")
            coll_busy = coll_max
            out["roofline"]["collective_busy_ms_mean"] = round(coll_busy, 4)
        else:
            out["roofline"] = dict(unpiped, timed_in=unpiped["timed_in"] + " (the timed steps kept no spans)")
        out["roofline_unpipelined"] = unpiped
    out["roofline"]["traffic"] = traffic
    out["roofline"]["traffic_note"] = traffic_note
    out["step_ms_device_median"] = round(statistics.median(blk["steps_ms"]), 4)
    if G > 1:
        out["host"] = {"enqueue_ms_per_step_timed": round(statistics.median(blk["host_ms"]), 4),
                       "devices_per_process": nlocal}
    if split:
        # The link: the collective's bytes per GPU over its busy time.  An
        # all-reduce (either form) moves 2(G-1)/G x 4n bytes per GPU (busbw);
        # the peer-read reduction reads (G-1)/G x 4n of its shard from the
        # peers (kernel B's remote reads of D sit inside kernel B's span).
        def link(ms, timed_in, algo=ar_algo):
            if not ms or ms <= 0 or G <= 1:
                return {"ms": round(ms, 4) if ms else ms, "timed_in": timed_in}
            algbw = 4 * n / (ms * 1e-3) / 1e9
            busbw = algbw * ((G - 1) / G if algo == _lib.ALLREDUCE_PEER else 2 * (G - 1) / G)
            r = {"ms": round(ms, 4), "algbw_GBs": round(algbw, 1), "busbw_GBs": round(busbw, 1),
                 "xgmi_frac": round(busbw / ((G - 1) * XGMI_LINK_GBS), 4), "timed_in": timed_in}
            if rehearse:
                # every rank on one GPU: the bytes never cross a link, so a
                # fraction of the xGMI bound would mean nothing
                r.update(xgmi_frac=None, note="rehearsal: every rank on one GPU, no xGMI link crossed")
            return r
        ar_ms = statistics.median(calib["allreduce"])
        # the calibration ran RCCL's all-reduce (one bucket, in order) whatever
        # form the block ran: its link rate is the all-reduce's
        unp = link(ar_ms, "calibration steps (one bucket, in order: one RCCL all-reduce alone)", 0)
        unp["form"] = "all-reduce"
        unp.update(apply_ms_median=round(statistics.median(calib["apply"]), 4),
                   step_ms_median=round(statistics.median(calib["step"]), 4))
        timed = (link(coll_busy, "timed region: per step, the union of the collectives' busy spans (each from the "
                                 "latest event bounding its start to its end), beside kernels A and B; slowest rank")
                 if coll_busy else None)
        out["allreduce"] = {"form": form, "xgmi_links": G - 1, "xgmi_peak_GBs": (G - 1) * XGMI_LINK_GBS,
                            "bytes_per_step": 4 * n,
                            "busbw_note": ("peer-read: (G-1)/G x 4n remote bytes per GPU in the reduction" if
                                           ar_algo == _lib.ALLREDUCE_PEER else "2(G-1)/G x 4n bytes per GPU"),
                            "timed": timed, "unpipelined": unp}
    return out


def merge_block(result, fields):
    """Put one timed block's fields into the line (its config keys into `config`)."""
    for k, v in fields.items():
        if k == "config":
            result["config"].update(v)
        elif k == "host":
            result.setdefault("host", {}).update(v)
        else:
            result[k] = v


def block_summary(fields, identity):
    """The timed block that did not set `value`, kept beside the line."""
    c = fields["config"]
    return {"value": fields["value"], "ms_per_step": fields["ms_per_step"],
            "config": {k: c[k] for k in ("allreduce_algorithm", "buckets", "pipeline_mode", "cross_wait_stride",
                                         "allreduce_group", "enqueue_threads", "bucket_tuning_ms_per_step",
                                         "tuning_errors")},
            "roofline": {k: fields["roofline"].get(k) for k in ("kernel", "achieved", "frac", "launch_ms_mean",
                                                                "timed_in")},
            "allreduce_timed": fields.get("allreduce", {}).get("timed"), "identity": identity}


def main():
    args = parse()
    if args.watchdog_selftest > 0:  # CPU test of the watchdog: a phase that stalls past its deadline
        wd = Watchdog(1.0, 0)
        wd.enter("selftest stall", args.watchdog_selftest)
        time.sleep(args.watchdog_selftest * 20 + 10)
        raise SystemExit("watchdog did not fire")
    # stdout carries the ONE JSON line and nothing else: native libraries
    # print banners there (RCCL's "RCCL version : ..." at communicator init),
    # so fd 1 is pointed at stderr for the run and the result goes to a
    # duplicate of the original stdout.
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.watchdog_selftest_result > 0 or args.selftest_raise:
        # CPU test: a line is assembled (as after the first timed region),
        # then a later phase stalls (or raises); that line must still come out
        wd = Watchdog(1.0, 0)
        wd.publish({"metric": METRIC, "value": 1.0, "unit": "GB/s", "config": {"peer_ipc": "mapping"}}, result_out)
        if args.selftest_raise:
            wd.enter("peer-read IPC mapping", 60)
            try:
                raise RuntimeError("selftest: a later phase raised")
            except Exception as e:  # noqa: BLE001
                wd.fail_now(e)
        wd.enter("selftest post-timed stall", args.watchdog_selftest_result)
        time.sleep(args.watchdog_selftest_result * 20 + 10)
        raise SystemExit("watchdog did not fire")
    if args.selftest_sigterm:
        # CPU test: the launcher's SIGTERM while the main thread waits (in a
        # handler-running wait, or -- "thread" -- one that never returns to
        # Python, as a HIP synchronize or a collective would not).  "launcher":
        # under torch.distributed.run, rank 1 is killed once rank 0 waits, and
        # the launcher's SIGTERM ends rank 0.
        rank = int(os.environ.get("RANK", "0"))
        mark = os.path.join(tempfile.gettempdir(), f"cbx_sigterm_selftest_{os.environ.get('MASTER_PORT', '0')}")
        if rank != 0:
            for _ in range(600):
                if os.path.exists(mark):
                    os.kill(os.getpid(), signal.SIGKILL)  # a crash: no handler, no line
                time.sleep(0.1)
            raise SystemExit("rank 0 never waited")
        wd = Watchdog(1.0, 0)
        wd.catch_sigterm()
        if args.selftest_sigterm != "unpublished":
            wd.publish({"metric": METRIC, "value": 1.0, "unit": "GB/s", "config": {}}, result_out)
        wd.enter("selftest wait for SIGTERM", 600)
        if args.selftest_sigterm in ("thread", "launcher"):
            signal.pthread_sigmask(signal.SIG_BLOCK, {signal.SIGTERM})
        log("[bench] selftest: waiting for SIGTERM")
        if args.selftest_sigterm == "launcher":
            open(mark, "w").close()
        threading.Event().wait(120)
        raise SystemExit("SIGTERM did not end the run")
    rank0 = int(os.environ.get("RANK", "0"))
    wd = Watchdog(args.watchdog_scale, rank0)
    wd.catch_sigterm()
    # the first `import torch` on a fresh box can take minutes (image paging)
    wd.enter("init (torch, HIP, communicators)", 900)
    from crossbow_amd import dist as D
    rank, world, local_rank = D.env_rank()
    G = args.gpus
    single = G > 1 and (args.single_process or "WORLD_SIZE" not in os.environ)
    if single:
        if world != 1:
            raise SystemExit("--single-process drives every GPU from one process: launch it without torch.distributed.run")
        devices = [0] * G if args.rehearse_one_gpu else list(range(G))
        local_rank = devices[0]
    else:
        if args.rehearse_one_gpu:
            D.rehearsal_env(rank)
            local_rank = 0
        if world != G:
            raise SystemExit(f"--gpus {G} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run "
                             "(one process per GPU) or without it (one process over N GPUs)")
    nlocal = G if single else 1
    peer_only = single and args.rehearse_one_gpu  # RCCL refuses a repeated device: the peer-read form only
    rccl_log = None
    if G > 1 and not peer_only and args.rccl_tuning_log:
        # RCCL reads these once, at its first call: every collective then logs
        # its algorithm / protocol / channels (one line each) to the file.
        rccl_log = os.path.join(tempfile.gettempdir(), f"cbx_rccl_tuning.r{rank}.{os.getpid()}.log")
        os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="TUNING", NCCL_DEBUG_FILE=rccl_log)

    import torch

    from crossbow_amd import SYNC_BSP, UPDATE_SMA, CbxError, TheGPU, _lib
    ALLREDUCE_PEER = _lib.ALLREDUCE_PEER
    from crossbow_amd.variables import MODELS, register

    torch.cuda.set_device(local_rank)
    gpu = TheGPU()
    if single:
        gpu.init(devices)
    else:
        D.init(world, rank)
        uid = D.share_unique_id(rank, world, TheGPU.unique_id)
        gpu.init_rank(local_rank, world, rank, uid)

    wd.enter("setup (model, synthetic replicas)", 300)
    shapes = MODELS[args.model]()
    n = register(gpu, shapes)
    gpu.setUpdateModelType(UPDATE_SMA)
    gpu.setEamsgdAlpha(args.alpha)
    gpu.setMomentum(args.momentum, 0)
    # scripts/benchmarks/resnet-50.sh:78-83: lr 0.1, multistep, gamma 0.1, decay 1e-4
    # (used by the replica optimiser step; the SMA step itself needs alpha only).
    gpu.setWeightDecay(1e-4)
    gpu.setLearningRateDecayPolicyMultiStep(0.1, 0.1, 0, [1 << 30])
    gpu.setModelManager(args.replicas, SYNC_BSP)
    gpu.set_kernel_config(args.block, args.blocks_per_cu, args.policy, args.unroll)
    gpu.set_kernel_occupancy(args.waves_per_cu)
    one_bucket = 1 << 62
    if args.bucket_elements > 0:
        bucket_elems = args.bucket_elements
    else:
        bucket_elems = int(args.bucket_mb * (1 << 20) / 4) if args.bucket_mb > 0 else (one_bucket if args.bucket_mb < 0 else 0)
    explicit = bucket_elems != 0
    if args.force_split:
        gpu.set_force_split(True)
    if peer_only:
        gpu.set_allreduce_algorithm(ALLREDUCE_PEER)
    gpu.fill_synthetic(SEED)
    gpu.set_timing(True)

    clock = 0

    def step():
        nonlocal clock
        clock += 1
        gpu.lockAny()
        try:
            gpu.synchronise(0, clock, 0, False)
        finally:
            gpu.unlockAny()

    split = G > 1 or args.force_split
    per_rank = G > 1 and not single
    # G > 1: every tuning candidate starts from the fresh synthetic state
    # (dist.tune_buckets), as every timed block does (timed_block's refill).
    dynamics = sma_dynamics(args.alpha, args.momentum, G * args.replicas) if G > 1 else None

    def refresh():
        gpu.wait()
        gpu.fill_synthetic(SEED)

    refresh = refresh if G > 1 else None
    # One process per GPU: the peer-read form needs every rank's acc and D
    # mapped through IPC handles first (cbx_peer_export / _import).  An
    # explicit peer-read configuration maps before anything else; otherwise
    # the mapping, the peer candidates and their timed block come AFTER the
    # RCCL forms' timed region, so nothing in them can cost the line (VERDICT
    # r04 Next #1): a phase there that misses its deadline makes the watchdog
    # print the line assembled so far.
    peer_ipc = None
    explicit_peer = per_rank and explicit and args.allreduce_algorithm == ALLREDUCE_PEER
    if explicit_peer:
        wd.enter("peer-read IPC mapping", args.peer_ipc_deadline)
        peer_ipc = D.setup_peer(gpu, world) or "mapped"
    elif per_rank:
        peer_ipc = ("not attempted: --no-peer-ipc" if args.no_peer_ipc else
                    "not attempted: explicit configuration" if explicit else "pending (after the timed region)")
    calib = None
    if rank == 0:
        log(f"[bench] {G} GPU(s) in {'one process' if single or G == 1 else f'{world} processes'}, n = {n}, "
            f"{args.replicas} replicas per GPU: {'calibration, tuning, ' if split else ''}warm-up, "
            f"{args.steps} timed steps")
    if split:
        # Calibration: one bucket, everything in order on the sync stream, so
        # HIP events separate kernel A, the collective and kernel B.
        wd.enter("calibration (one bucket, in order)", 180)
        gpu.set_bucket_elements(one_bucket)
        for _ in range(args.calib_steps):
            step()
        gpu.wait()
        k = max(1, args.calib_steps)
        calib = {"kernel": list(gpu.timing_history(_lib.T_KERNEL)[-k:]),
                 "allreduce": list(gpu.timing_history(_lib.T_ALLREDUCE)[-k:]),
                 "apply": list(gpu.timing_history(_lib.T_APPLY)[-k:]),
                 "step": list(gpu.timing_history(_lib.T_STEP)[-k:])}
    gpu.set_bucket_elements(bucket_elems)
    tuning = None
    chosen = {"bucket_elements": bucket_elems, "buckets": lib_buckets(n, bucket_elems, G), "mode": 0, "stride": 1,
              "group": 1, "algorithm": ALLREDUCE_PEER if peer_only else 0,
              "enqueue_threads": 0 if single else None}
    if split and not explicit:
        # warm-up autotune of the pipeline on the live communicator (same
        # choice on every rank); one process per GPU: RCCL's forms only here
        tuning = D.tune_buckets(gpu, n, world, step, progress=(lambda m: log(f"[bench] {m}")) if rank == 0 else None,
                                ndev=G, peer=single, peer_only=peer_only, threads=single,
                                steps=max(1, args.tune_steps), passes=max(1, args.tune_passes),
                                warmup=min(2, max(1, args.tune_steps)),
                                phase=lambda name: wd.enter(name, 90), refresh=refresh)
        chosen.update(bucket_elements=tuning.bucket_elements, buckets=tuning.buckets, mode=tuning.mode,
                      stride=tuning.stride, group=tuning.group, algorithm=tuning.algorithm,
                      enqueue_threads=tuning.enqueue_threads)
    elif split:
        for key, flag, setter in (("mode", args.pipeline_mode, gpu.set_pipeline_mode),
                                  ("stride", args.wait_stride, gpu.set_cross_wait_stride),
                                  ("group", args.allreduce_group, gpu.set_allreduce_group),
                                  ("algorithm", args.allreduce_algorithm, gpu.set_allreduce_algorithm)):
            if flag is not None:
                setter(flag)
                chosen[key] = flag
        if single and args.enqueue_threads is not None:
            gpu.set_enqueue_threads(args.enqueue_threads)
            chosen["enqueue_threads"] = args.enqueue_threads

    blk = timed_block(gpu, torch, D, args, world, step, wd, refill=split and G > 1)
    result = {
        "metric": METRIC,
        "value": None,
        "unit": "GB/s",
        "n_gpus": G,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (splitmix64 -> Box-Muller, BASELINE.md 2.3), generated on device",
        "config": {
            "workload": f"{args.model}-params SMA reduce+correct, {args.replicas} replicas/GPU x {G} GPU",
            "elements": n,
            "replicas_per_gpu": args.replicas,
            "alpha": args.alpha,
            "momentum": args.momentum,
            "parallelism": f"sma-dp{G}",
            "process_form": None if G == 1 else ("single" if single else "per-rank"),
            "pipeline": "fused" if not split else "accumulate+collective+apply, bucketed on two streams",
            # one process per GPU: whether the peer-read form's IPC mapping
            # (cbx_peer_export / _import) succeeded on every rank, else why not
            "peer_ipc": peer_ipc,
            # ROCclr's hardware queues per device (read once at HIP start)
            "hw_queues": {"GPU_MAX_HW_QUEUES": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                          "environment_had": HW_QUEUES_ENV,
                          "set_by": ("bench.py (--hw-queues)" if HW_QUEUES_SET else
                                     "the environment (HIP's default 4 when unset)")},
            "kernel_config": dict(block=args.block, blocks_per_cu=args.blocks_per_cu, policy=args.policy,
                                  unroll=args.unroll, waves_per_cu=args.waves_per_cu, bucket_mb=args.bucket_mb),
        },
    }
    fields = block_fields(gpu, D, args, world, n, G, nlocal, split, blk, chosen, tuning, calib,
                          args.rehearse_one_gpu)
    merge_block(result, fields)
    # From here on the line exists: a later phase that misses its deadline
    # makes the watchdog print it (with `incomplete_phase`) instead of nothing.
    wd.publish(result, result_out)
    try:
        if G > 1:
            wd.enter("cross-GPU identity of z and last", 180)
            result["identity"] = block_identity(gpu, world, step, chosen, one_bucket, peer_only, ALLREDUCE_PEER, wd,
                                                blk, dynamics)

        reported = chosen
        if per_rank and split and not explicit and not args.no_peer_ipc:
            # The per-rank peer-read form, as a second block after the RCCL forms'.
            result["config"]["peer_ipc"] = "mapping"
            wd.enter("peer-read IPC mapping", args.peer_ipc_deadline)
            why = D.setup_peer(gpu, world)
            result["config"]["peer_ipc"] = peer_ipc = why or "mapped"
            if why is None:
                ptuning = D.tune_buckets(gpu, n, world, step,
                                         progress=(lambda m: log(f"[bench] {m}")) if rank == 0 else None,
                                         ndev=G, peer=True, peer_only=True, threads=False,
                                         steps=max(1, args.tune_steps), passes=max(1, args.tune_passes),
                                         warmup=min(2, max(1, args.tune_steps)),
                                         phase=lambda name: wd.enter(name, 90), refresh=refresh)
                best_rccl, best_peer = min(tuning.table.values()), min(ptuning.table.values())
                pchosen = dict(chosen, bucket_elements=ptuning.bucket_elements, buckets=ptuning.buckets,
                               mode=ptuning.mode, stride=ptuning.stride, group=ptuning.group,
                               algorithm=ptuning.algorithm)
                if best_peer < best_rccl:
                    # the tuner's best peer-read candidate beat RCCL's best: time it
                    pblk = timed_block(gpu, torch, D, args, world, step, wd, refill=True, label=" (peer-read form)")
                    pfields = block_fields(gpu, D, args, world, n, G, nlocal, split, pblk, pchosen, ptuning, calib,
                                           args.rehearse_one_gpu)
                    wd.enter("cross-GPU identity of z and last (peer-read form)", 180)
                    pident = block_identity(gpu, world, step, pchosen, one_bucket, False, ALLREDUCE_PEER, wd,
                                            pblk, dynamics)
                    if pfields["value"] > result["value"] and pident.get("trusted", False):
                        other = block_summary({k: result[k] for k in pfields}, result["identity"])
                        merge_block(result, pfields)
                        result["identity"] = pident
                        result["other_form"] = other
                        reported = pchosen
                    else:
                        result["other_form"] = block_summary(pfields, pident)
                else:
                    result["other_form"] = {
                        "config": {"allreduce_algorithm": "peer-read two-shot",
                                   "bucket_tuning_ms_per_step": ptuning.table, "tuning_errors": ptuning.errors},
                        "timed": (f"not timed: the tuner's best peer-read candidate ({best_peer:.4f} ms per step) was "
                                  f"slower than RCCL's best ({best_rccl:.4f} ms)")}
            apply_config(gpu, reported, single)
        ar_algo = reported["algorithm"]

        if G > 1:
            # Host side of the step (lockAny + synchronise + unlockAny, every local
            # device's enqueue) against the device's step: the single-process form
            # enqueues all G devices' kernels and collectives from one thread.
            wd.enter("host enqueue (idle GPU)", 120)
            idle = []
            for _ in range(5):
                gpu.wait()
                h0 = time.perf_counter()
                step()
                idle.append((time.perf_counter() - h0) * 1e3)
            gpu.wait()
            result["host"].update(
                enqueue_ms_per_step_idle_gpu=round(statistics.median(idle), 4),
                note="perf_counter around lockAny+synchronise+unlockAny; 'idle_gpu' after a wait, so no queue "
                     "back-pressure; host-bound when it exceeds ms_per_step")
        if args.rehearse_one_gpu:
            result["rehearsal"] = (f"{G} ranks on ONE GPU over RCCL's socket transport (NCCL_HOSTID per rank): "
                                   "a check of the N > 1 code path, not an N-GPU measurement" if not single else
                                   f"{G} devices of one process that are all device 0, peer-read all-reduce (RCCL "
                                   "refuses a repeated device): the single-process form's host side and code path, "
                                   "not an N-GPU measurement")
        if split and rccl_log:
            gpu.wait()
            result["allreduce"]["rccl_tuning"] = rccl_tuning(rccl_log)
            try:
                os.remove(rccl_log)
            except OSError:
                pass
            result["allreduce"]["rccl_tuning_source"] = (
                "RCCL's own log (NCCL_DEBUG=INFO, NCCL_DEBUG_SUBSYS=TUNING) of THIS run (--rccl-tuning-log): every "
                "collective of calibration, tuning and the timed region")

        step_bytes, _ = alg_bytes(n, args.replicas, args.momentum, 2 if split else 1)
        if G > 1 and not args.no_staged and peer_only:
            result["host_staged"] = {"skipped": "the host-staged step's collective is RCCL's, which refuses a repeated device"}
        elif G > 1 and not args.no_staged:
            # Host-staged rate at N > 1 (north_star: the path starts and ends in
            # host memory): each GPU's replicas live in its own pinned mirror and
            # cross its own PCIe link; zero-copy staging kernels, kernel A /
            # all-reduce / kernel B per bucket.  Max over ranks of the median of 3.
            # The pinned mirror is allocated first (no collective); every rank
            # must have one before any rank enters the staged step's collectives.
            wd.enter("host-staged step", 300)
            why = None
            try:
                gpu.stage_in()
                gpu.wait()
            except CbxError as e:
                why = str(e)
            if D.max_over_ranks(0.0 if why is None else 1.0, world) > 0.0:
                result["host_staged"] = {"skipped": f"pinned host mirror unavailable on some rank ({why or 'another rank'})"}
            else:
                gpu.set_staging_mode(_lib.STAGING_ZEROCOPY)
                runs = []
                for _ in range(3):
                    clock += 1
                    gpu.lockAny()
                    gpu.synchronise_staged(0, clock, 0, args.staged_buckets)
                    gpu.unlockAny()
                    gpu.wait()
                    runs.append(max(gpu.last_timing(k)[_lib.T_STEP] for k in range(nlocal)))
                ms = D.max_over_ranks(sorted(runs)[1], world)
                result["host_staged"] = {"zerocopy": {
                    "buckets": args.staged_buckets, "step_ms": round(ms, 3),
                    "end_to_end_GBs": round(step_bytes * G / (ms * 1e-3) / 1e9, 2),
                    "per_gpu_GBs": round(step_bytes / (ms * 1e-3) / 1e9, 2),
                    "timed": "HIP events per device (staged step: host in, host and device out), max over devices"}}

        if rank == 0 and G == 1 and not args.no_optimiser:
            wd.enter("replica optimiser step", 120)
            result["replica_optimiser"] = bench_optimiser(gpu, torch, n, args)
        if rank == 0 and G == 1 and not args.no_seam:
            wd.enter("sma.c seam", 180)
            result["seam"] = bench_seam(torch, n, args)

        if rank == 0 and G == 1:
            if not args.no_copy_ceiling:
                wd.enter("copy ceiling", 120)
                result["copy_ceiling_GBs"] = round(gpu.bench_copy(1 << 30, 20), 1)
            if not args.no_staged:
                # Host-staged rate (north_star): pinned H2D of z, last, s_i, w_i,
                # the step, pinned D2H of z, last, w_i.  Reported, never `value`.
                wd.enter("host-staged step", 300)
                samples = []
                for _ in range(3):
                    gpu.stage_in()
                    step()
                    gpu.stage_out()
                    gpu.wait()
                    samples.append(gpu.last_timing(0))
                t = sorted(samples, key=lambda x: x[_lib.T_H2D] + x[_lib.T_KERNEL] + x[_lib.T_D2H])[1]
                m = 1 if args.momentum > 0 else 0
                h2d = (2 * args.replicas + 1 + m) * 4 * n
                d2h = (args.replicas + 1 + m) * 4 * n
                tot = (t[_lib.T_H2D] + t[_lib.T_KERNEL] + t[_lib.T_D2H]) * 1e-3
                result["host_staged"] = {
                    "h2d_ms": round(t[_lib.T_H2D], 3), "kernel_ms": round(t[_lib.T_KERNEL], 4),
                    "d2h_ms": round(t[_lib.T_D2H], 3),
                    "h2d_GBs": round(h2d / (t[_lib.T_H2D] * 1e-3) / 1e9, 2),
                    "d2h_GBs": round(d2h / (t[_lib.T_D2H] * 1e-3) / 1e9, 2),
                    "end_to_end_GBs": round(step_bytes / tot / 1e9, 2),
                }
                # The same step through cbx_synchronise_staged, both staging modes:
                # DMA (uploads, kernels and downloads pipelined over buckets on
                # three streams) and zero-copy (the kernels read and write the
                # pinned mirror over PCIe themselves; the library default).
                def staged(mode):
                    nonlocal clock
                    gpu.set_staging_mode(mode)
                    runs = []
                    for _ in range(3):
                        clock += 1
                        gpu.lockAny()
                        gpu.synchronise_staged(0, clock, 0, args.staged_buckets)
                        gpu.unlockAny()
                        gpu.wait()
                        runs.append(gpu.last_timing(0))
                    return sorted(runs, key=lambda x: x[_lib.T_STEP])[1]
                p = staged(_lib.STAGING_DMA)
                result["host_staged"]["pipelined"] = {
                    "buckets": args.staged_buckets, "step_ms": round(p[_lib.T_STEP], 3),
                    "h2d_ms": round(p[_lib.T_H2D], 3), "d2h_ms": round(p[_lib.T_D2H], 3),
                    "end_to_end_GBs": round(step_bytes / (p[_lib.T_STEP] * 1e-3) / 1e9, 2),
                    "timed": "HIP events: sync stream at entry to sync stream after the last download"}
                z = staged(_lib.STAGING_ZEROCOPY)
                result["host_staged"]["zerocopy"] = {
                    "step_ms": round(z[_lib.T_STEP], 3),
                    "end_to_end_GBs": round(step_bytes / (z[_lib.T_STEP] * 1e-3) / 1e9, 2),
                    "pcie_GBs_both_ways": round((h2d + d2h) / (z[_lib.T_STEP] * 1e-3) / 1e9, 2),
                    "timed": "HIP events on the fused staged kernel's own dispatch (one launch: host in, host + device out)"}
            if not args.no_cpu_baseline:
                # multithreaded first: OpenBLAS's pool must not start out bound to core 0
                wd.enter("CPU baseline", 4 * args.cpu_seconds + 240)
                threads = max(1, min(16, len(os.sched_getaffinity(0))))
                mt = cpu_baseline_threads(args, n, threads)
                result["cpu_baseline"] = cpu_baseline(args, n)
                result["cpu_baseline"]["cpu_model"] = mt["cpu_model"] = cpu_model()
                result["cpu_baseline_multithread"] = mt
                result["cpu_c1_lenet"] = cpu_c1()
            else:
                result["cpu_baseline"] = None

        wd.enter("free", 120)
        gpu.free()
        if split and G > 1 and not rccl_log:
            # RCCL's algorithm / protocol / channel choices, from a separate short
            # run of the chosen configuration with RCCL's tuning log on (rank 0
            # launches it once this run's buffers are freed; the others wait).
            if peer_only or ar_algo == ALLREDUCE_PEER:
                entries, source = None, "no RCCL collective in the chosen form"
            elif args.no_rccl_tuning_run:
                entries, source = None, "--no-rccl-tuning-run"
            elif args.rehearse_one_gpu and not single and 2 * G + 2 > 16:
                # the separate run's ranks would join this run's on the one GPU
                entries, source = None, f"not run: a {G}-rank rehearsal plus {G} more ranks exceeds 16 processes on one GPU"
            elif rank == 0:
                entries, source = rccl_tuning_run(args, G, single, reported, wd)
            else:
                wd.enter("rccl tuning run (rank 0's)", 420)
                entries, source = None, None
            if world > 1:
                D.barrier(world)
            result["allreduce"]["rccl_tuning"] = entries
            result["allreduce"]["rccl_tuning_source"] = source
    except Exception as e:  # noqa: BLE001 -- a later phase must not cost the measured line
        import traceback
        traceback.print_exc()
        wd.fail_now(e)
    if not wd.finish():  # a SIGTERM ending is printing the line: let it end the process
        time.sleep(60)
        os._exit(0)
    if rank == 0:
        print(json.dumps(result), file=result_out, flush=True)
    # the line is out: a teardown that never returns must not keep the rank alive
    ender = threading.Timer(120, lambda: os._exit(0))
    ender.daemon = True
    ender.start()
    D.finalize(world)


if __name__ == "__main__":
    main()
