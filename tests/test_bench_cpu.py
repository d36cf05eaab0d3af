"""bench.py's host-side machinery on the CPU (no GPU needed)."""
from __future__ import annotations

import os
import subprocess
import sys

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
