"""A/B of the fused C3 kernel's load and store order (round 6 experiment, not
part of the library).  membench v11 (profiles/r01/membench11.jsonl) measured,
in a stand-alone copy of the kernel, +1-1.5 % for storing each w_r right after
its fma ("SO 1") and +1 % for loading every s before every w ("LO 1").  This
rebuilds the library itself with each change, in scratch directories:

  base   the shipped crossbow_amd/csrc
  so1    each w_r stored right after its fma
  lo1    every s_r loaded before every w_r

--build  (here, on the CPU) writes scripts/ab_build/<variant>/libcrossbow_sma.so
--run    (on the GPU box) times the C3 fused step of every variant, interleaved
         over --rounds fresh contexts, through the torch-free C-ABI bindings:
         the median of --steps HIP-event kernel times per round, one JSON line
         per (round, variant), then a summary line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import shutil
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "crossbow_amd", "csrc")
OUT = os.path.join(ROOT, "scripts", "ab_build")
N, R = 25_557_032, 8

FMA_THEN_STORE = '''          acc[u] = vfma(al, d, acc[u]);
        }
      }
      if constexpr (!COPY) {
#pragma unroll
        for (int r = 0; r < RR; ++r) {
          if (R < 0 && c + r >= nrep) break;
#pragma unroll
          for (int u = 0; u < U; ++u) sto<P>(a.w[c + r], (base + u * 64u) * 16u, wv[u][r]);
        }
      }
      if constexpr (R >= 0) break;'''
STORE_EACH = '''          acc[u] = vfma(al, d, acc[u]);
          if constexpr (!COPY) sto<P>(a.w[c + r], (base + u * 64u) * 16u, wv[u][r]);
        }
      }
      if constexpr (R >= 0) break;'''
LOAD_PAIRS = '''        for (int u = 0; u < U; ++u) {
          const uint32_t i = (base + u * 64u) * 16u;
          sv[u][r] = ldo<P>(a.s[c + r], i);
          if constexpr (!COPY) wv[u][r] = ldo<P>(a.w[c + r], i);
        }
      }
      // Keep every load'''
LOAD_S_THEN_W = '''        for (int u = 0; u < U; ++u) sv[u][r] = ldo<P>(a.s[c + r], (base + u * 64u) * 16u);
      }
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (R < 0 && c + r >= nrep) break;
#pragma unroll
        for (int u = 0; u < U; ++u)
          if constexpr (!COPY) wv[u][r] = ldo<P>(a.w[c + r], (base + u * 64u) * 16u);
      }
      // Keep every load'''
VARIANTS = {"base": [], "so1": [(FMA_THEN_STORE, STORE_EACH)], "lo1": [(LOAD_PAIRS, LOAD_S_THEN_W)]}


def build():
    for name, patches in VARIANTS.items():
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        for f in os.listdir(CSRC):
            if f.endswith((".hip", ".h")):
                shutil.copy(os.path.join(CSRC, f), d)
        h = os.path.join(d, "context_internal.h")  # its relative include of the ABI header, from here
        text = open(h).read().replace('"../../include/crossbow_sma.h"', '"crossbow_sma.h"')
        open(h, "w").write(text)
        k = os.path.join(d, "sma_kernels.hip")
        src = open(k).read()
        for old, new in patches:
            # the fused kernel's occurrence comes first in the file
            assert old in src, (name, old[:60])
            src = src.replace(old, new, 1)
        open(k, "w").write(src)
        objs = []
        for f in ("context.hip", "sync_steps.hip", "sma_kernels.hip", "sma_seam.hip"):
            o = os.path.join(d, f.replace(".hip", ".o"))
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
                            f"-cuid=crossbow_{f[:-4]}", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                            "-c", "-o", o, os.path.join(d, f)], check=True)
            objs.append(o)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o",
                        os.path.join(d, "libcrossbow_sma.so")] + objs +
                       ["-lrccl", "-lrocprofiler-sdk-roctx", "-lpthread"], check=True)
        print("built", name, flush=True)


def run(rounds: int, steps: int):
    import importlib.util
    spec = importlib.util.spec_from_file_location("cbx_abi", os.path.join(ROOT, "crossbow_amd", "_abi.py"))
    A = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(A)
    libs = {name: A.bind(ctypes.CDLL(os.path.join(OUT, name, "libcrossbow_sma.so"))) for name in VARIANTS}
    res = {name: [] for name in VARIANTS}
    for rnd in range(rounds):
        order = list(VARIANTS) if rnd % 2 == 0 else list(reversed(VARIANTS))
        for name in order:
            L = libs[name]
            c = ctypes.c_void_p()
            devs = (ctypes.c_int * 1)(0)
            assert L.cbx_init(ctypes.byref(c), devs, 1) == 0, L.cbx_last_error()
            try:
                shape = (ctypes.c_int * 1)(N)
                for fn, args in (("cbx_set_model", (1, 4 * N)), ("cbx_set_model_variable", (0, 1, 1, shape, 4 * N)),
                                 ("cbx_set_update_model_type", (7,)), ("cbx_set_eamsgd_alpha", (ctypes.c_float(0.1),)),
                                 ("cbx_set_momentum", (ctypes.c_float(0.9), 0)), ("cbx_set_model_manager", (R, 0)),
                                 ("cbx_fill_synthetic", (20190701,)), ("cbx_set_timing", (1,))):
                    assert getattr(L, fn)(c, *args) >= 0, (fn, L.cbx_last_error())
                for k in range(5 + steps):
                    assert L.cbx_lock_any(c) >= 0
                    assert L.cbx_synchronise(c, 0, k + 1, 0, 0) == 0, L.cbx_last_error()
                    assert L.cbx_unlock_any(c) >= 0
                assert L.cbx_wait(c) == 0
                buf = (ctypes.c_float * steps)()
                got = L.cbx_timing_history(c, 0, 0, buf, steps)
                ms = statistics.median(list(buf)[:got])
            finally:
                L.cbx_free(c)
            res[name].append(ms)
            print(json.dumps({"round": rnd, "variant": name, "kernel_ms_median": round(ms, 5),
                              "GBs": round(112 * N / (ms * 1e-3) / 1e9, 1)}), flush=True)
    summary = {name: {"best_ms": round(min(v), 5), "median_ms": round(statistics.median(v), 5),
                      "GBs_median": round(112 * N / (statistics.median(v) * 1e-3) / 1e9, 1)} for name, v in res.items()}
    print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--build", action="store_true")
    p.add_argument("--run", action="store_true")
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--steps", type=int, default=50)
    a = p.parse_args()
    if a.build:
        build()
    if a.run:
        run(a.rounds, a.steps)
    if not (a.build or a.run):
        sys.exit("--build and / or --run")
