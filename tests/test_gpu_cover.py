"""GPU: pkg/cover Cover (cover.go:7-30) on device -- Merge/Serialize/Len against
the restatement (oracle.OCover), including the nil-receiver rule and the
manager's corpusCover accumulation (syz-manager/manager.go:998)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_cover_nil_and_empty(gpu):
    from syzkaller_amd.signal import Cover

    c, o = Cover(gpu.eng), O.OCover()
    assert c.is_nil() and len(c) == 0 and c.Serialize().size == 0
    c.Merge(np.empty(0, np.uint32))  # a nil receiver is allocated even for an empty raw
    o.Merge([])
    assert not c.is_nil() and o.c is not None and len(c) == 0


def test_cover_merge_matches_restatement(gpu):
    from syzkaller_amd.signal import Cover

    rng = np.random.default_rng(7)
    c, o = Cover(gpu.eng), O.OCover()
    for i in range(40):
        n = int(rng.integers(0, 50000))
        raw = (0x81000000 + rng.integers(0, 400000, n)).astype(np.uint32)  # many repeats across merges
        if i % 7 == 0:
            raw = np.concatenate([raw, np.array([0, 0xFFFFFFFF], np.uint32)])
        c.Merge(raw)
        o.Merge(raw)
        assert len(c) == len(o.c)
    np.testing.assert_array_equal(np.sort(c.Serialize()), np.array(o.Serialize(), np.uint32))


def test_cover_large_merge(gpu):
    from syzkaller_amd.signal import Cover

    rng = np.random.default_rng(8)
    raw = rng.integers(0, 1 << 32, 3_000_000, dtype=np.uint64).astype(np.uint32)
    c = Cover(gpu.eng)
    c.Merge(raw)
    c.Merge(raw[::3])
    u = np.unique(raw)
    assert len(c) == u.size
    np.testing.assert_array_equal(np.sort(c.Serialize()), u)
