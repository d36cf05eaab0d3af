"""CPU tests of the oracle (oracle/sma_oracle.c), pinned before it is trusted.

* splitmix64 against the published known-answer vector of its author;
* the fmaf restatement against an OpenBLAS replay of the reference's saxpy
  call sequence (the BLAS the reference links, clib-multigpu/BLAS.c:32,328),
  bit for bit, over a grid of configurations;
* the committed golden fixtures (tests/golden/, from make_golden.py);
* the reference semantics that are easy to get wrong: hard-coded base momentum
  0.9 (sma.c:152), unlocked replicas untouched, Phase D copies, `first`.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden_cases():
    from tests.golden.make_golden import build_state, input_arrays, sha
    cases = []
    for path in sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))):
        with np.load(path, allow_pickle=False) as f:
            cfg = json.loads(str(f["config"]))
            st = build_state(cfg["n"], cfg["G"], cfg["R"], cfg["alpha"], cfg["momentum"], cfg["first"],
                             cfg["unlocked"], cfg["copy"])
            assert sha(input_arrays(st)) == cfg["input_sha256"], f"{path}: input generator changed"
            cases.append(dict(name=cfg["name"], G=cfg["G"], cfg=cfg, state=st, z_out=list(f["z_out"]),
                              w_out=list(f["w_out"]),
                              last_out=list(f["last_out"]) if f["last_out"].size else None))
    return cases


def _eq(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


def test_splitmix64_known_answer():
    # Vigna's splitmix64.c seeded with 1234567: the first five outputs.
    want = [6457827717110365317, 3203168211198807973, 9817491932198370423, 4593380528125082431,
            16408922859458223821]
    golden = 0x9E3779B97F4A7C15
    got = [O.splitmix64((1234567 + k * golden) & 0xFFFFFFFFFFFFFFFF) for k in range(5)]
    assert got == want


def test_normal_generator_moments():
    x = O.fill_normal(200_000, 3, 1.0).astype(np.float64)
    assert abs(x.mean()) < 0.01 and abs(x.std() - 1.0) < 0.01
    y = O.fill_normal(1000, 3, 1.0)
    assert _eq(y, x[:1000].astype(np.float32)), "counter-based: prefix independent of length"


@pytest.mark.parametrize("G,R", [(1, 1), (1, 2), (1, 4), (1, 8), (2, 2), (4, 2), (2, 4), (8, 1)])
@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_fma_restatement_equals_openblas_sequence(G, R, momentum):
    st = O.make_state(2053, G, R, 0.1, momentum)
    st.copy[G * R - 1] = 1 if R > 1 else 0
    a, b = st.clone(), st.clone()
    assert O.sma_step(a) == O.sma_step_blas(b)
    for x, y in zip(a.z + a.w + (a.last or []), b.z + b.w + (b.last or [])):
        assert _eq(x, y)


def test_golden_manifest():
    with open(os.path.join(GOLDEN_DIR, "MANIFEST.json")) as f:
        manifest = json.load(f)
    assert len(manifest) >= 9
    for name, digest in manifest.items():
        with open(os.path.join(GOLDEN_DIR, name), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == digest, name


def test_golden_fixtures():
    cases = load_golden_cases()
    assert len(cases) >= 9
    for case in cases:
        st = case["state"].clone()
        copies = O.sma_step(st)
        assert copies == case["cfg"]["copies"]
        for k in range(st.G):
            assert _eq(st.z[k], case["z_out"][k]), case["name"]
        for k in range(st.size):
            assert _eq(st.w[k], case["w_out"][k]), case["name"]
        if case["last_out"] is not None:
            for k in range(st.G):
                assert _eq(st.last[k], case["last_out"][k]), case["name"]


def test_base_momentum_is_hard_coded():
    # sma.c:150-152: any positive momentum becomes 0.9 for the base model.
    a = O.make_state(1031, 1, 2, 0.1, 0.9)
    b = a.clone()
    b.momentum = 0.3
    O.sma_step(a)
    O.sma_step(b)
    assert _eq(a.z[0], b.z[0]) and _eq(a.last[0], b.last[0])


def test_unlocked_and_first_are_skipped():
    st = O.make_state(1031, 1, 5, 0.1, 0.0)
    st.locked[3] = 0
    st.first = 1
    ref = st.clone()
    O.sma_step(st)
    assert _eq(st.w[0], ref.w[0]), "replica below `first` untouched"
    assert _eq(st.w[3], ref.w[3]), "unlocked replica untouched"
    assert not _eq(st.w[1], ref.w[1])
    # the step only used replicas 1, 2, 4
    z = ref.z[0]
    acc = np.zeros_like(z)
    for i in (1, 2, 4):
        acc = acc + np.float32(0.1) * (ref.s[i] - z)
    np.testing.assert_allclose(st.z[0], z + acc, rtol=0, atol=2e-7)


def test_phase_d_copy_resets_flags():
    st = O.make_state(1031, 2, 2, 0.1, 0.9)
    st.copy[1] = 1
    assert O.sma_step(st) == 1
    assert st.copy.sum() == 0
    for i in range(st.size):
        assert _eq(st.w[i], st.z[i % 2])


def test_multi_gpu_bases_stay_identical():
    st = O.make_state(1031, 4, 2, 0.1, 0.9)
    O.sma_step(st)
    for k in range(1, 4):
        assert _eq(st.z[k], st.z[0]) and _eq(st.last[k], st.last[0])


def test_bytes_per_step_formula():
    n = 25_557_032
    assert O.bytes_per_step(n, 8, 0.9) == 112 * n  # C3: 2.862 GB
    assert O.bytes_per_step(1_111_946, 4, 0.0) == 56 * 1_111_946  # C2
    assert O.bytes_per_step(n, 4, 0.9, G=8) == 76 * n  # C5 per GPU


@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("wd", [0.0, 5e-4])
def test_optimiser_restatement_equals_openblas_sequence(momentum, wd):
    # kernels/optimisers/sma.cu:3-100: the fmaf restatement and the literal
    # saxpy / sscal / memcpy sequence agree bit for bit.
    n = 4099
    w = O.fill_normal(n, 100, 0.05)
    g = O.fill_normal(n, 101, 0.01)
    last = O.fill_normal(n, 102, 0.001) if momentum > 0 else None
    s = np.zeros(n, np.float32)
    a = [x.copy() if x is not None else None for x in (w, g, last, s)]
    b = [x.copy() if x is not None else None for x in (w, g, last, s)]
    O.sma_optimise(-0.1, momentum, wd, *a)
    O.sma_optimise(-0.1, momentum, wd, *b, blas=True)
    for x, y in zip(a, b):
        if x is not None:
            assert _eq(x, y)
    assert _eq(a[3], w), "s is the snapshot of w before the update (sma.cu:71,87)"
    assert not _eq(a[0], w)


@pytest.mark.parametrize("momentum", [0.0, 0.9])
@pytest.mark.parametrize("wd", [0.0, 5e-4])
def test_default_task_restatement_equals_openblas_sequence(momentum, wd):
    # kernels/optimisers/default.cu:3-131: replica and base model take the same
    # step; fmaf restatement == literal saxpy / sscal / memcpy sequence.
    n = 4099
    w = O.fill_normal(n, 110, 0.05)
    g = O.fill_normal(n, 111, 0.01)
    last = O.fill_normal(n, 112, 0.001) if momentum > 0 else None
    z = O.fill_normal(n, 113, 0.05)
    a = [x.copy() if x is not None else None for x in (w, g, last, z)]
    b = [x.copy() if x is not None else None for x in (w, g, last, z)]
    O.default_task(-0.1, momentum, wd, *a)
    O.default_task(-0.1, momentum, wd, *b, blas=True)
    for x, y in zip(a, b):
        if x is not None:
            assert _eq(x, y)
    # both models moved by the same (scaled) gradient
    np.testing.assert_allclose(a[0] - w, a[3] - z, rtol=0, atol=1e-6)


def test_default_sync_copies_base_to_locked_replicas():
    # synch/default.c:5-43: w_i = z for locked i >= first; others untouched.
    st = O.make_state(1031, 1, 4, 0.1, 0.0)
    st.locked[2] = 0
    st.first = 1
    w0 = [x.copy() for x in st.w]
    O.default_sync(st)
    assert _eq(st.w[0], w0[0]) and _eq(st.w[2], w0[2])
    assert _eq(st.w[1], st.z[0]) and _eq(st.w[3], st.z[0])
    with pytest.raises(ValueError):
        O.default_sync(O.make_state(64, 2, 1, 0.1, 0.0))


def test_optimiser_then_sma_moves_replicas_toward_base():
    # One clock of the whole loop on the oracle: local steps, then averaging.
    st = O.make_state(2053, 1, 4, 0.5, 0.9)
    grads = [O.fill_normal(st.n, 200 + i, 0.01) for i in range(st.size)]
    lasts = [np.zeros(st.n, np.float32) for _ in range(st.size)]
    spread0 = max(float(np.abs(st.w[i] - st.z[0]).max()) for i in range(st.size))
    for i in range(st.size):
        O.sma_optimise(-0.01, 0.9, 0.0, st.w[i], grads[i], lasts[i], st.s[i])
    O.sma_step(st)
    spread1 = max(float(np.abs(st.w[i] - st.z[0]).max()) for i in range(st.size))
    assert spread1 < spread0


@pytest.mark.parametrize("G", [1, 2, 4])
@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_ssgd_restatement_equals_openblas_sequence(G, momentum):
    # Synchronous SGD (WORKER): task steps (synchronoussgd.cu:3-56) then the
    # barrier (synchronoussgd.c:13-106) -- fmaf restatement == BLAS replay.
    n, R = 2053, 2
    st = O.make_state(n, G, R, 0.1, momentum)
    st.locked[0] = 0
    grads = [O.fill_normal(n, 600 + i, 0.01) for i in range(st.size)]
    outs = []
    for blas in (False, True):
        s2 = st.clone()
        acc = [np.zeros(n, np.float32) for _ in range(G)]
        gs = [x.copy() for x in grads]
        for i in range(s2.size):
            O.ssgd_worker(np.float32(-0.05), 1e-4, s2.w[i], gs[i], acc[i % G], blas=blas)
        O.ssgd_sync(s2, acc, 8, blas=blas)
        outs.append((s2, acc, gs))
    (a, acc_a, g_a), (b, acc_b, g_b) = outs
    for x, y in zip(a.z + a.w + (a.last or []) + acc_a + g_a, b.z + b.w + (b.last or []) + acc_b + g_b):
        assert _eq(x, y)
    assert all(not x.any() for x in acc_a), "barrier resets base->gradient (synchronoussgd.c:103)"
    assert _eq(a.w[0], st.w[0]), "unlocked replica keeps its data"
    for i in range(1, a.size):
        assert _eq(a.w[i], a.z[i % G])


def test_bn_average_matches_formula():
    # cudnnbatchnormparams.c:157-222 over 3 layers and 4 devices.
    G, elements = 4, [64, 256, 3]
    mean = [[O.fill_normal(e, 700 + 10 * g + l, 0.5) for l, e in enumerate(elements)] for g in range(G)]
    var = [[np.abs(O.fill_normal(e, 800 + 10 * g + l, 1.0)) for l, e in enumerate(elements)] for g in range(G)]
    updated = [[1, 1, 1], [1, 0, 1], [0, 0, 1], [1, 0, 0]]
    want_m, want_v = [], []
    for l in range(len(elements)):
        cnt = [0] + [g for g in range(1, G) if updated[g][l]]
        m = sum(mean[g][l].astype(np.float64) for g in cnt) / len(cnt)
        v = sum(var[g][l].astype(np.float64) for g in cnt) / len(cnt)
        want_m.append(m)
        want_v.append(v)
    O.bn_average(mean, var, updated)
    for g in range(G):
        for l in range(len(elements)):
            np.testing.assert_allclose(mean[g][l], want_m[l], rtol=2e-6, atol=1e-7)
            np.testing.assert_allclose(var[g][l], want_v[l], rtol=2e-6, atol=1e-7)
            assert _eq(mean[g][l], mean[0][l]) and _eq(var[g][l], var[0][l])


def test_bn_average_single_device_is_noop():
    m = [[O.fill_normal(32, 900, 0.5)]]
    v = [[O.fill_normal(32, 901, 0.5)]]
    m0, v0 = m[0][0].copy(), v[0][0].copy()
    O.bn_average(m, v, [[0]])
    assert _eq(m[0][0], m0) and _eq(v[0][0], v0)
