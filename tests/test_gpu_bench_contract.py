"""bench.py's output contract, on the GPU: exactly ONE JSON line on stdout
(native libraries' banners go to stderr), with the fields the driver reads,
at N = 1 and through the driver's own N > 1 launcher (torch.distributed.run,
two ranks on the one GPU over RCCL's socket transport: --rehearse-one-gpu).
Short runs: the numbers are not checked here, only the shape of the line."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUICK = ["--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-staged", "--no-copy-ceiling", "--no-optimiser", "--no-seam"]


def _one_line(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, f"stdout must carry exactly one line, got {len(lines)}: {lines[:3]}"
    return json.loads(lines[0])


def _check(d: dict, n: int):
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert key in d, key
    assert d["n_gpus"] == n and d["steps"] == 3 and d["warmup"] == 1
    assert d["unit"] == "GB/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] < 1 and r["achieved"] > 0
    assert "workload" in d["config"]


@pytest.mark.timeout(240)
def test_bench_one_gpu_prints_one_json_line():
    p = subprocess.run([sys.executable, "bench.py"] + QUICK, cwd=ROOT, capture_output=True, text=True, timeout=220)
    assert p.returncode == 0, p.stderr[-2000:]
    _check(_one_line(p.stdout), 1)


@pytest.mark.timeout(300)
def test_bench_two_ranks_through_the_launcher_prints_one_json_line():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29671", "bench.py", "--gpus", "2",
           "--rehearse-one-gpu", "--bucket-mb", "16"] + QUICK
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _one_line(p.stdout)
    _check(d, 2)
    assert d["config"]["parallelism"] == "sma-dp2" and "allreduce" in d and "rehearsal" in d


@pytest.mark.timeout(300)
def test_bench_two_ranks_host_staged_field():
    # the N > 1 host-staged leg (zero-copy staging over two rehearsal ranks)
    quick = [a for a in QUICK if a != "--no-staged"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29673", "bench.py", "--gpus", "2",
           "--rehearse-one-gpu", "--bucket-mb", "16"] + quick
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _one_line(p.stdout)
    _check(d, 2)
    z = d["host_staged"]["zerocopy"]
    assert z["step_ms"] > 0 and z["end_to_end_GBs"] > 0 and z["per_gpu_GBs"] > 0
