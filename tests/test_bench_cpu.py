"""bench.py's host-side machinery on the CPU (no GPU needed)."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_watchdog_fires_on_a_stalled_phase():
    # A phase that stalls past its deadline ends the run with exit code 3 and
    # every thread's Python stack on stderr (no restart, no exec): the
    # driver's multi-GPU run cannot hang silently.
    p = subprocess.run([sys.executable, "bench.py", "--watchdog-selftest", "1"], cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "WATCHDOG" in p.stderr and "'selftest stall' missed its 1 s deadline" in p.stderr, p.stderr[-2000:]
    assert 'File "' in p.stderr and "in main" in p.stderr and "in _watch" in p.stderr, p.stderr[-2000:]
    assert p.stdout == ""


def test_lib_buckets_matches_the_library_rule():
    # bench.py's config.buckets: the library's bucket geometry (whole
    # 1,024-float4 units, SplitStep::prepare_common)
    sys.path.insert(0, ROOT)
    import bench
    n = 25_557_032
    assert bench.lib_buckets(n, 0, 1) == 1
    assert bench.lib_buckets(n, 0, 8) == 8
    assert bench.lib_buckets(n, 1 << 62, 8) == 1
    assert bench.lib_buckets(n, -(-n // 4), 2) == 4
    assert bench.lib_buckets(300_001, 65_536, 1) == 5
    assert bench.lib_buckets(300_000, 16_384, 1) == 19
    assert bench.lib_buckets(300_000, 4096, 1) == 74


def test_rccl_tuning_run_repeats_the_chosen_configuration(monkeypatch):
    # The separate short run that fills allreduce.rccl_tuning (RCCL's tuning
    # log stays off in the measured run) must time the configuration the
    # tuner chose, in the same process form, and parse RCCL's table from the
    # child's one JSON line.
    import json
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    class FakePopen:
        def __init__(self, cmd, cwd, env, stdout, stderr, text, start_new_session):
            seen["cmd"], seen["env"] = cmd, env
            self.pid, self.returncode = 12345, 0

        def communicate(self, timeout=None):
            line = json.dumps({"allreduce": {"rccl_tuning": [{"collective": "AllReduce", "bytes": 4, "algo": "RING",
                                                                "proto": "SIMPLE", "channels": [0, 3], "calls": 1}]}})
            return "RCCL version banner\n" + line + "\n", ""

    class FakeWd:
        def enter(self, name, secs):
            seen["phase"] = name

    monkeypatch.setattr(bench.subprocess, "Popen", FakePopen)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--rehearse-one-gpu"])
    args = bench.parse()
    for k, v in {"RANK": "3", "WORLD_SIZE": "8", "MASTER_PORT": "29500", "NCCL_DEBUG": "WARN",
                 "TORCHELASTIC_RUN_ID": "x"}.items():
        monkeypatch.setenv(k, v)
    cfg = {"bucket_elements": 3194629, "mode": 1, "stride": 2, "group": 4, "algorithm": 2, "enqueue_threads": None}
    t, source = bench.rccl_tuning_run(args, 8, False, cfg, FakeWd())
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node" in cmd
    i = cmd.index("bench.py") if "bench.py" in cmd else [j for j, c in enumerate(cmd) if c.endswith("bench.py")][0]
    child = cmd[i:]
    for flag, value in (("--bucket-elements", "3194629"), ("--pipeline-mode", "1"), ("--wait-stride", "2"),
                        ("--allreduce-group", "4"), ("--allreduce-algorithm", "2"), ("--gpus", "8")):
        assert child[child.index(flag) + 1] == value, (flag, child)
    assert "--rccl-tuning-log" in child and "--no-rccl-tuning-run" in child and "--rehearse-one-gpu" in child
    assert not any(k in seen["env"] for k in ("RANK", "WORLD_SIZE", "MASTER_PORT", "NCCL_DEBUG", "TORCHELASTIC_RUN_ID"))
    assert t and t[0]["algo"] == "RING" and "separate" in source and seen["phase"] == "rccl tuning run"
    # one process over every device: the same bench.py, no launcher, the enqueue threading passed on
    cfg["enqueue_threads"] = 1
    bench.rccl_tuning_run(args, 8, True, cfg, FakeWd())
    cmd = seen["cmd"]
    assert cmd[1].endswith("bench.py") and "--single-process" in cmd
    assert cmd[cmd.index("--enqueue-threads") + 1] == "1"


def test_watchdog_prints_the_line_when_a_later_phase_stalls():
    # Once the first timed region has produced the line, a later phase that
    # misses its deadline (e.g. the per-rank peer-read form's IPC mapping)
    # must not cost it: the watchdog prints exactly that one line, naming the
    # phase that did not finish, with every thread's kernel-side state on
    # stderr, and the run exits 0 (VERDICT r04 Next #1).
    import json
    p = subprocess.run([sys.executable, "bench.py", "--watchdog-selftest-result", "1"], cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.returncode, p.stderr[-2000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and d["incomplete_phase"]["phase"] == "selftest post-timed stall"
    assert "WATCHDOG" in p.stderr and " wchan=" in p.stderr and " syscall=" in p.stderr, p.stderr[-2000:]


def test_watchdog_names_a_stalled_ipc_mapping_in_the_line():
    # The line the watchdog prints for a stalled IPC mapping says so in
    # config.peer_ipc (the field the driver's N > 1 line carries).
    sys.path.insert(0, ROOT)
    import json

    import bench
    wd = bench.Watchdog(0, 0)
    wd.publish({"metric": bench.METRIC, "value": 5.0, "config": {"peer_ipc": "mapping"}}, None)
    d = json.loads(wd._line("peer-read IPC mapping", 300.0, "agreement with the all-reduce"))
    assert d["config"]["peer_ipc"].startswith("failed: 'peer-read IPC mapping' missed its 300 s deadline")
    assert d["incomplete_phase"]["last_completed"] == "agreement with the all-reduce" and d["value"] == 5.0


def test_thread_states_lists_every_thread():
    sys.path.insert(0, ROOT)
    import threading

    import bench
    ev = threading.Event()
    t = threading.Thread(target=ev.wait, name="waiter", daemon=True)
    t.start()
    try:
        out = bench.thread_states()
    finally:
        ev.set()
    rows = [ln for ln in out.splitlines() if ln.strip().startswith("tid ")]
    assert len(rows) >= 2 and all(" wchan=" in r and " syscall=" in r for r in rows), out


class _FakeGpu:
    """Just enough of TheGPU for bench.form_agreement on the CPU: z and last of
    one device, replicas' w, and a 'step' that moves z by a fixed amount
    (the measured form) or by that amount plus `skew` (the reference form)."""

    def __init__(self, z, skew=0.0):
        import numpy as np
        self.np = np
        self.z = np.asarray(z, dtype=np.float32)
        self.last = np.zeros_like(self.z)
        self.w = {0: np.ones_like(self.z)}
        self.algo, self.skew = 1, skew

    def local_devices(self):
        return [0]

    def local_replicas(self):
        return [0]

    def wait(self):
        pass

    def base_read(self, g, kind):
        return (self.z if kind == 0 else self.last).copy()

    def base_write(self, g, kind, a):
        if kind == 0:
            self.z = a.copy()
        else:
            self.last = a.copy()

    def replica_read(self, i, kind):
        return self.w[i].copy()

    def replica_write(self, i, kind, a):
        self.w[i] = a.copy()

    def set_allreduce_algorithm(self, a):
        self.algo = a

    def set_bucket_elements(self, b):
        pass

    def set_pipeline_mode(self, m):
        pass

    def step(self):
        self.z = (self.z + self.np.float32(0.5) + (self.np.float32(self.skew) if self.algo == 0 else 0)).astype(
            self.np.float32)


def test_agreement_check_is_vacuous_at_blown_up_values():
    # The G > 1 agreement check compares the measured form's step with one
    # in-order all-reduce of the same step within rtol 1e-5: at |z| ~ 1.7e13
    # that forgives 1.7e8, so a large diff would pass.  Above 1e3 the check
    # reports itself vacuous and not within tolerance (VERDICT r04 Weak #3).
    sys.path.insert(0, ROOT)
    import bench
    from crossbow_amd import BUF_DATA, BUF_LAST
    assert (BUF_DATA, BUF_LAST) == (0, 1) or True
    chosen = {"algorithm": 1, "bucket_elements": 1 << 20, "mode": 1, "buckets": 4}
    big = _FakeGpu([1.6e13, -3.0, 2.0], skew=1.0e6)
    r = bench.form_agreement(big, 1, big.step, chosen, 1 << 62, "peer-read two-shot")
    assert r["vacuous"] is True and r["within_tolerance"] is False and r["max_abs_value"] > 1e13
    small = _FakeGpu([0.25, -0.1, 0.05])
    r = bench.form_agreement(small, 1, small.step, chosen, 1 << 62, "peer-read two-shot")
    assert r["vacuous"] is False and r["within_tolerance"] is True and r["bitwise_equal"] is True
    skewed = _FakeGpu([0.25, -0.1, 0.05], skew=1e-3)
    r = bench.form_agreement(skewed, 1, skewed.step, chosen, 1 << 62, "peer-read two-shot")
    assert r["vacuous"] is False and r["within_tolerance"] is False


def test_a_later_phase_that_raises_still_prints_the_line():
    # An exception in a phase after the first timed region (the peer-read
    # form's mapping, its tuner, the host-staged leg, ...) ends the run with
    # the measured line, naming the phase and the error, exit 0.
    import json
    p = subprocess.run([sys.executable, "bench.py", "--selftest-raise"], cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, (p.returncode, p.stderr[-2000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    inc = d["incomplete_phase"]
    assert inc["phase"] == "peer-read IPC mapping" and "selftest: a later phase raised" in inc["error"], inc
    assert d["config"]["peer_ipc"].startswith("failed: 'peer-read IPC mapping' raised RuntimeError"), d["config"]


def test_block_fields_shape_at_two_gpus():
    # The fields one timed block contributes to the N > 1 line (value, the
    # kernels' roofline beside the collective, the link rate, the host's
    # enqueue time), how a block merges into the line and how the other
    # block is summarised in `other_form`: a fake context's timing records
    # stand in for the GPU.
    sys.path.insert(0, ROOT)
    import argparse

    import bench
    from crossbow_amd import _lib
    from crossbow_amd import dist as D
    n, K = 25_557_032, 4

    class FakeGpu:
        hist = {_lib.T_KERNEL: [0.30] * K, _lib.T_ALLREDUCE: [0.12] * K, _lib.T_APPLY: [0.07] * K,
                _lib.T_STEP: [0.45] * K}

        def timing_history(self, which, local=0):
            return list(self.hist[which])

    args = argparse.Namespace(replicas=8, momentum=0.9, steps=K, model="resnet50",
                              traffic_json=os.path.join(ROOT, "profiles", "traffic.json"))
    blk = {"el": K * 0.5e-3, "host_ms": [0.05] * K, "steps_ms": [0.45] * K}
    calib = {"kernel": [0.43, 0.43], "allreduce": [0.2, 0.2], "apply": [0.08, 0.08], "step": [0.72, 0.72]}
    chosen = {"algorithm": _lib.ALLREDUCE_RCCL, "buckets": 4, "mode": 1, "stride": 2, "group": 1,
              "enqueue_threads": None, "bucket_elements": -(-n // 4)}

    class Tune:
        table = {"4/1/s2": 0.5}
        errors = {}

    f = bench.block_fields(FakeGpu(), D, args, 1, n, 2, 1, True, blk, chosen, Tune(), calib, False)
    step_bytes = (12 * 8 + 8) * n + (12 + 8) * n
    assert f["value"] == round(step_bytes * 2 * K / blk["el"] / 1e9, 2) and f["ms_per_step"] == 0.5
    r = f["roofline"]
    assert r["kernel"] == "sma_accumulate_kernel" and r["launch_ms_mean"] == 0.3
    assert r["apply_kernel"]["kernel"] == "sma_apply_kernel" and r["a_plus_b"]["launch_ms_mean"] == 0.37
    assert r["collective_busy_ms_mean"] == 0.12 and f["roofline_unpipelined"]["launch_ms_mean"] == 0.43
    ar = f["allreduce"]
    assert ar["form"] == "all-reduce" and ar["timed"]["busbw_GBs"] > 0 and ar["timed"]["xgmi_frac"] > 0
    assert f["config"]["buckets"] == 4 and f["config"]["allreduce_algorithm"] == "all-reduce"
    assert f["host"] == {"enqueue_ms_per_step_timed": 0.05, "devices_per_process": 1}
    line = {"metric": bench.METRIC, "config": {"workload": "w", "peer_ipc": "mapped"}}
    bench.merge_block(line, f)
    assert line["value"] == f["value"] and line["config"]["peer_ipc"] == "mapped" and line["config"]["buckets"] == 4
    s = bench.block_summary(f, {"trusted": True})
    assert s["value"] == f["value"] and s["config"]["allreduce_algorithm"] == "all-reduce"
    assert s["roofline"]["frac"] == r["frac"] and s["identity"] == {"trusted": True}


def _sigterm_run(variant: str):
    import signal
    p = subprocess.Popen([sys.executable, "bench.py", "--selftest-sigterm", variant], cwd=ROOT,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    err = []
    try:
        for line in p.stderr:  # the selftest says when it is waiting
            err.append(line)
            if "waiting for SIGTERM" in line:
                break
        p.send_signal(signal.SIGTERM)
        out, rest = p.communicate(timeout=60)
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    return p.returncode, out, "".join(err) + rest


@pytest.mark.parametrize("variant", ["main", "thread"])
def test_launcher_sigterm_still_prints_the_line(variant):
    # torch.distributed.run sends SIGTERM to every rank once one rank fails:
    # rank 0 prints the line it already holds, naming the phase that was
    # ended, and exits 0 -- also when its main thread is in a wait that never
    # returns to Python ("thread": SIGTERM blocked there, as inside a HIP
    # synchronize the watchdog thread handles it through the wakeup fd).
    import json
    rc, out, err = _sigterm_run(variant)
    assert rc == 0, (rc, err[-2000:])
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out
    inc = json.loads(lines[0])["incomplete_phase"]
    assert inc["phase"] == "selftest wait for SIGTERM" and inc["error"] == "SIGTERM", inc
    assert "was ended by SIGTERM" in inc["note"]
    assert "SIGTERM in phase 'selftest wait for SIGTERM'" in err, err[-2000:]


def test_launcher_sigterm_before_the_line_ends_the_rank_as_sigterm_would():
    rc, out, err = _sigterm_run("unpublished")
    assert rc == 143 and not out.strip(), (rc, out, err[-2000:])


def test_launcher_ending_a_failed_run_keeps_rank_0s_line():
    # The real launcher: rank 1 dies (SIGKILL, as a crash would) while rank 0
    # holds a line and waits in a wait that never returns to Python;
    # torch.distributed.run then SIGTERMs rank 0, which prints that line.
    import json
    import socket
    import tempfile
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mark = os.path.join(tempfile.gettempdir(), f"cbx_sigterm_selftest_{port}")
    if os.path.exists(mark):
        os.unlink(mark)
    try:
        # the launcher imports torch: through tests/torch_loader_check.py (a no-op on a healthy install)
        boot = ("import runpy, sys; from tests.torch_loader_check import ensure_torch_loadable; "
                "ensure_torch_loadable(); sys.argv = ['torch.distributed.run'] + sys.argv[1:]; "
                "runpy.run_module('torch.distributed.run', run_name='__main__')")
        p = subprocess.run([sys.executable, "-c", boot, "--nnodes=1", "--nproc-per-node", "2",
                            "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py",
                            "--selftest-sigterm", "launcher"], cwd=ROOT, capture_output=True, text=True, timeout=180)
    finally:
        if os.path.exists(mark):
            os.unlink(mark)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, (p.returncode, p.stdout, p.stderr[-3000:])
    inc = json.loads(lines[0])["incomplete_phase"]
    assert inc["error"] == "SIGTERM" and inc["phase"] == "selftest wait for SIGTERM", inc
    assert p.returncode != 0  # the launcher still reports rank 1's failure


def test_fixed_snapshot_dynamics_match_the_oracle():
    # VERDICT r05 Weak #5: the G > 1 bench's values grow after the timed
    # region at 8 GPUs.  That is the SMA update itself with the snapshots held
    # fixed (no optimiser between steps), not the kernels: the oracle grows at
    # the radius bench.sma_dynamics predicts where alpha N > 2 (1 + mu), and
    # stays bounded at the reference's own 8 x 2 run and at C5's 8 x 4.
    # Re-snapshotting s_i <- w_i every step does not bound it either.
    import numpy as np

    import bench
    from oracle import oracle as O

    def run(G, R, steps, resnap=False):
        st = O.make_state(4096, G, R, 0.1, 0.9)
        top0 = max(float(np.max(np.abs(z))) for z in st.z + st.last)
        for _ in range(steps):
            O.sma_step(st)
            if resnap:
                for i in range(st.size):
                    st.s[i][:] = st.w[i]
        return max(float(np.max(np.abs(z))) for z in st.z + st.last) / top0

    d88 = bench.sma_dynamics(0.1, 0.9, 64)
    assert not d88["bounded"] and abs(d88["spectral_radius_per_step"] - 4.2902) < 1e-3, d88
    growth = (run(8, 8, 30) / run(8, 8, 20)) ** (1 / 10)  # past the first steps' transient
    assert abs(growth - d88["spectral_radius_per_step"]) < 0.1 * d88["spectral_radius_per_step"], growth
    assert run(8, 8, 20, resnap=True) > 1e6
    for G, R in ((8, 2), (8, 4), (4, 8)):
        d = bench.sma_dynamics(0.1, 0.9, G * R)
        assert d["bounded"] and d["spectral_radius_per_step"] < 1.0, (G, R, d)
        assert run(G, R, 40) < 2.0, (G, R)
    assert bench.sma_dynamics(0.1, 0.0, 16)["bounded"] and not bench.sma_dynamics(0.1, 0.0, 32)["bounded"]


def test_identity_trusts_overflow_only_where_the_dynamics_predicts_it(monkeypatch):
    # At 8 GPUs x 8 replicas the values grow ~4x per step (sma_dynamics); a
    # long enough timed region takes them past fp32's range.  Non-finite z /
    # last then do not cost the block its trust, and the line stays strict
    # JSON (max_abs_value None); at a step count where no overflow is
    # predicted, non-finite values still mark the block untrusted.
    import json

    import bench
    monkeypatch.setattr(bench, "base_identity", lambda gpu, world: {
        "z_last_identical_on_every_gpu": True, "finite": False, "max_abs_value": None})
    chosen = {"algorithm": 0, "buckets": 1}
    dyn = bench.sma_dynamics(0.1, 0.9, 64)
    for steps, trusted in ((100, True), (23, False)):
        idn = bench.block_identity(None, 1, None, chosen, 1, True, 1, None,
                                   {"fresh_max_abs": 0.26, "steps_since_fresh": steps}, dyn)
        assert idn["dynamics"]["overflow_expected"] is trusted and idn["trusted"] is trusted, (steps, idn)
        assert idn["dynamics"]["observed_growth_per_step"] is None
        json.loads(json.dumps(idn, allow_nan=False))
    bounded = bench.sma_dynamics(0.1, 0.9, 32)
    idn = bench.block_identity(None, 1, None, chosen, 1, True, 1, None,
                               {"fresh_max_abs": 0.26, "steps_since_fresh": 1000}, bounded)
    assert not idn["dynamics"]["overflow_expected"] and not idn["trusted"]
