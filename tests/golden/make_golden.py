"""Generate the golden SMA fixtures in tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

The reference holds no golden vectors for this path and cannot be built here
(SURVEY.md 8c), so these fixtures come from the CPU restatement
(oracle/sma_oracle.c) and are pinned two ways before being written:
  1. the fmaf restatement and an OpenBLAS replay of the reference's exact
     saxpy call sequence (clib-multigpu/synch/sma.c) must agree bit for bit;
  2. inputs are regenerated from seeds (splitmix64 -> Box-Muller), and their
     sha256 is stored so a changed generator is detected.
Each fixture stores the configuration, the input sha256 and the full outputs.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402

CASES = [
    # name, n, G, R, alpha, momentum, first, unlocked ids, copy ids
    ("g1_r1_mu0", 1031, 1, 1, 0.1, 0.0, 0, (), ()),
    ("g1_r4_mu9", 1031, 1, 4, 0.1, 0.9, 0, (), ()),
    ("g1_r8_mu9_ragged", 4099, 1, 8, 0.1, 0.9, 0, (), ()),
    ("g1_r4_alpha_half", 1031, 1, 4, 0.5, 0.0, 0, (), ()),
    ("g1_r4_copy", 1031, 1, 4, 0.1, 0.9, 0, (), (3,)),
    ("g1_r6_first2_unlocked4", 1031, 1, 6, 0.1, 0.9, 2, (4,), ()),
    ("g2_r2_mu9", 1031, 2, 2, 0.1, 0.9, 0, (), ()),
    ("g4_r2_mu0_copy", 1031, 4, 2, 0.1, 0.0, 0, (), (5,)),
    ("g8_r4_mu9", 1031, 8, 4, 0.1, 0.9, 0, (), ()),
]


def sha(arrs) -> str:
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a, dtype=np.float32).tobytes())
    return h.hexdigest()


def build_state(n, G, R, alpha, momentum, first, unlocked, copy_ids) -> O.SmaState:
    st = O.make_state(n, G, R, alpha, momentum)
    st.first = first
    for i in unlocked:
        st.locked[i] = 0
    for i in copy_ids:
        st.copy[i] = 1
    return st


def input_arrays(st: O.SmaState):
    return [st.z[0]] + ([st.last[0]] if st.last is not None else []) + st.s + st.w


def main() -> None:
    O.blas_open()
    manifest = {}
    for name, n, G, R, alpha, mom, first, unlocked, copy_ids in CASES:
        st = build_state(n, G, R, alpha, mom, first, unlocked, copy_ids)
        in_sha = sha(input_arrays(st))
        a, b = st.clone(), st.clone()
        ca = O.sma_step(a)
        cb = O.sma_step_blas(b)
        assert ca == cb
        outs_a = a.z + a.w + (a.last or [])
        outs_b = b.z + b.w + (b.last or [])
        for x, y in zip(outs_a, outs_b):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), f"{name}: fma vs OpenBLAS mismatch"
        cfg = dict(name=name, n=n, G=G, R=R, alpha=alpha, momentum=mom, first=first,
                   unlocked=list(unlocked), copy=list(copy_ids), copies=ca, input_sha256=in_sha,
                   z_head=[float(v) for v in st.z[0][:4]])
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, config=np.array(json.dumps(cfg)),
                            z_out=np.stack(a.z), w_out=np.stack(a.w),
                            last_out=np.stack(a.last) if a.last is not None else np.zeros((0, n), np.float32))
        with open(path, "rb") as f:
            manifest[os.path.basename(path)] = hashlib.sha256(f.read()).hexdigest()
        print(f"{name}: copies={ca} input_sha={in_sha[:12]}")
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
