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
