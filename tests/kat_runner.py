"""Runs tests/kat_cases.py against an implementation adapter, so the oracle
(CPU) and the engine (GPU) are held to the same known answers."""
import numpy as np

from tests import kat_cases as K


class Impl:
    """Adapter: nil() / empty() / from_dict(d) / from_raw / minimize / check_new."""

    def nil(self):
        raise NotImplementedError

    def empty(self):
        raise NotImplementedError

    def from_dict(self, d):
        raise NotImplementedError

    def make(self, d):
        if d is None:
            return self.nil()
        if not d:
            return self.empty()
        return self.from_dict(d)


def as_result(sig):
    """nil -> None, non-nil empty -> "EMPTY", else dict"""
    if sig.is_nil():
        return None
    d = sig.to_dict()
    return d if d else "EMPTY"


def norm(exp):
    return exp


def run_from_raw(impl):
    for desc, raw, prio, exp in K.FROM_RAW:
        got = as_result(impl.from_raw(np.array(raw, np.uint32), prio))
        assert got == exp, desc


def run_diff(impl):
    for desc, s, s1, exp in K.DIFF:
        got = as_result(impl.make(s).Diff(impl.make(s1)))
        assert got == exp, desc


def run_diff_raw(impl):
    for desc, s, raw, prio, exp in K.DIFF_RAW:
        got = as_result(impl.make(s).DiffRaw(np.array(raw, np.uint32), prio))
        assert got == exp, desc


def run_intersection(impl):
    for desc, s, s1, exp in K.INTERSECTION:
        got = as_result(impl.make(s).Intersection(impl.make(s1)))
        assert got == exp, desc


def run_merge(impl):
    for desc, s, s1, exp in K.MERGE:
        a = impl.make(s)
        a.Merge(impl.make(s1))
        got = as_result(a)
        if exp == {} or (isinstance(exp, dict) and not exp):
            exp = "EMPTY"
        assert got == exp, desc


def run_deserialize(impl):
    for desc, e, p, exp in K.DESERIALIZE:
        if exp == "CORRUPT":
            try:
                impl.deserialize(np.array(e, np.uint32), np.array(p, np.int8))
            except impl.corrupt_exc:
                continue
            raise AssertionError(desc + ": no panic")
        got = as_result(impl.deserialize(np.array(e, np.uint32), np.array(p, np.int8)))
        assert got == exp, desc


def run_minimize(impl):
    for desc, ctxs, exp in K.MINIMIZE:
        got = impl.minimize(ctxs)
        assert sorted(got) == sorted(exp), desc


def run_check_new(impl):
    for desc, m0, calls, exp_calls, exp_max, exp_new, exp_recs in K.CHECK_NEW:
        calls_got, max_d, new_d, rec_sets = impl.check_new(m0, calls)
        assert calls_got == exp_calls, desc
        assert max_d == exp_max, desc
        assert new_d == exp_new, desc
        assert rec_sets == exp_recs, desc


ALL = [run_from_raw, run_diff, run_diff_raw, run_intersection, run_merge, run_deserialize, run_minimize,
       run_check_new]


def flatten_calls(calls):
    sigs = np.array([e for raw, _ in calls for e in raw], np.uint32)
    lens = np.array([len(raw) for raw, _ in calls], np.uint32)
    starts = np.zeros(len(calls), np.uint64)
    if len(calls) > 1:
        starts[1:] = np.cumsum(lens[:-1])
    prios = np.array([p & 0xFF for _, p in calls], np.uint8)
    return sigs, starts, lens, prios


def rec_sets_from_bits(bits, starts, lens):
    out = []
    for s, n in zip(starts, lens):
        out.append({j for j in range(int(n)) if (int(bits[(int(s) + j) >> 5]) >> ((int(s) + j) & 31)) & 1})
    return out
