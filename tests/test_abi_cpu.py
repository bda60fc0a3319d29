"""CPU: the C-ABI library loads and exports every symbol include/syzsig.h
declares; host-side pieces (synthetic generator, error paths) without a GPU."""
import os
import re
import subprocess

import numpy as np
import pytest

from syzkaller_amd import _lib, synth
from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "syzsig.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|double|uint64_t|const char\*|void\*)\s+\**(syzsig_\w+)\s*\(", txt, re.M)))


def test_header_symbols_exported_and_bound():
    names = declared()
    assert len(names) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (syzsig_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)
    L = _lib.lib()
    for n in names:
        assert getattr(L, n) is not None


def test_abi_version_matches_header():
    m = re.search(r"#define SYZSIG_ABI_VERSION (\d+)", open(HEADER).read())
    assert _lib.lib().syzsig_abi_version() == int(m.group(1))


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", _lib.LIB_PATH], capture_output=True,
                         text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_ctx_create_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import ctypes

    h = ctypes.c_void_p()
    rc = _lib.lib().syzsig_ctx_create(0, ctypes.byref(h))
    assert rc == _lib.SYZSIG_EIO and not h.value
    assert b"device" in _lib.lib().syzsig_last_error()


def test_synth_deterministic_and_in_range():
    cfg = synth.synth_default()
    cl = synth.call_lengths(4, 8, 0, ragged=(0, 3000), seed=2)
    a = synth.traces(cfg, 10, 4, 8, cl)
    b = synth.traces(cfg, 10, 4, 8, cl)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    pcs, cs, prio = a
    assert ((pcs >= 0xFFFFFFFF80000000) & (pcs < 0xFFFFFFFFFF000000)).all()  # cover_check passes
    assert ((pcs - 0xFFFFFFFF81000000) % 5 == 0).all()
    c = synth.traces(cfg, 11, 4, 8, cl)
    assert not np.array_equal(a[0], c[0])


def test_synth_prio_distribution():
    cfg = synth.synth_default()
    n = 20000
    cl = np.zeros(n, np.uint32)
    _, _, prio = synth.traces(cfg, 0, n, 1, cl)
    failed = ((prio >> 1) & 1) == 0
    anyp = (prio & 1) == 0
    assert abs(failed.mean() - 0.3) < 0.02 and abs(anyp.mean() - 0.1) < 0.02
    assert set(np.unique(prio).tolist()) <= {0, 1, 2, 3}


def test_synth_zipf_entries_global_walk():
    """skew=2 on the global walk (SURVEY 8(d)'s C5 input): a call's walk
    starts at the entry block of a Zipf(1.1)-chosen syscall (csrc/common.h
    synth_zipf4096), and then walks b <- (4b + 1 + r%4) mod 2^20."""
    cfg = synth.synth_default(global_walk=1, skew=2)
    n = 40000
    pcs, cs, _ = synth.traces(cfg, 0, n, 1, np.full(n, 2, np.uint32))
    first = ((pcs[cs.astype(np.int64)] - 0xFFFFFFFF81000000) // 5).astype(np.int64)
    second = ((pcs[cs.astype(np.int64) + 1] - 0xFFFFFFFF81000000) // 5).astype(np.int64)
    assert (((second - (4 * first + 1)) % (1 << 20)) < 4).all()  # the global walk's step
    # the start blocks' frequencies follow the ranks' k^-1.1
    k = np.arange(1, 4097, dtype=np.float64)
    w = k ** -1.1
    w /= w.sum()
    vals, counts = np.unique(first, return_counts=True)
    top = counts[np.argsort(-counts)][:5] / n
    assert abs(top[0] - w[0]) < 0.03 and abs(top[1] - w[1]) < 0.015 and abs(top[4] - w[4]) < 0.01
    assert vals.size > 1500  # a long tail of distinct entries


def test_synth_m0_known_edges_cover_the_syscalls_signals():
    """Every signal the executor derives for a call to a syscall < known_sys is
    an element of M0's known part (M0 enumerates the region's edges)."""
    from oracle import oracle as O

    cfg = synth.synth_default()
    known = 64
    e, p = synth.m0(cfg, known, known * (5 * 256 + 1))
    kset = set(e.tolist())
    assert set(np.unique(p).tolist()) <= {0, 1, 2, 3}
    lib = _lib.lib()
    import ctypes

    hits = 0
    for prog in range(200):
        pcs, cs, prio = synth.traces(cfg, prog, 1, 1, np.array([3000], np.uint32))
        # recover the syscall: its entry block starts the trace
        sigs, cnt, _ = O.exec_program(pcs, cs, np.array([3000], np.uint32))
        entry_sig = int(sigs[0])
        if entry_sig in kset:
            hits += 1
            assert set(sigs[: cnt[0]].tolist()) <= kset
    assert hits > 0
    del lib, ctypes


def test_owner_hash_torch_matches_reference_formula():
    import torch

    from syzkaller_amd.dist import owner_of_torch
    from tests.test_gpu_minimize_shard import _owner

    x = np.random.default_rng(0).integers(0, 2**32, size=2000, dtype=np.uint64)
    for n in (1, 2, 3, 8):
        got = owner_of_torch(torch.from_numpy(x.astype(np.int64)), n).numpy()
        exp = np.array([_owner(int(v), n) for v in x])
        np.testing.assert_array_equal(got, exp)
