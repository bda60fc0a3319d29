"""Known-answer cases for pkg/signal and checkNewSignal, derived by hand from
the reference source (pkg/signal/signal.go, syz-fuzzer/fuzzer.go:494-521).
The Go reference cannot be run here (no Go toolchain), so these pin the
restatement: every expected value below follows one line of the Go code,
cited per case.  A Signal is written as a dict {elem: prio}; None is nil.
"""

# (signal.go line, s, raw, prio, expected)   FromRaw(raw, prio)
FROM_RAW = [
    ("31-34 empty raw -> nil", [], 3, None),
    ("35-38 dups collapse", [1, 2, 2, 3], 2, {1: 2, 2: 2, 3: 2}),
    ("38 prioType(uint8 255) == -1", [5], 255, {5: -1}),
    ("elem 0 is a valid element", [0, 0xFFFFFFFF], 1, {0: 1, 0xFFFFFFFF: 1}),
]

# (desc, s, s1, expected)   s.Diff(s1)
DIFF = [
    ("74-76 nil.Diff(nil) -> nil", None, None, None),
    ("74-76 s.Diff(empty) -> nil", {1: 1}, {}, None),
    ("79-80 nil receiver: everything new", None, {1: 0, 2: -3}, {1: 0, 2: -3}),
    ("79 p >= p1 skips; lower or absent is new", {1: 1, 2: 2, 3: -1}, {1: 1, 2: 3, 3: 0, 4: -5},
     {2: 3, 3: 0, 4: -5}),
    ("87 nothing new -> nil", {1: 3, 2: 0}, {1: 2, 2: 0}, None),
]

# (desc, s, raw, prio, expected)   s.DiffRaw(raw, prio)
DIFF_RAW = [
    ("92-94 equal prio is not new", {1: 2}, [1, 1, 2, 3, 3], 2, {2: 2, 3: 2}),
    ("92 higher prio is new", {1: 2}, [1, 2], 3, {1: 3, 2: 3}),
    ("93 int8 compare: uint8 200 == -56", {1: -100, 2: -56}, [1, 2], 200, {1: -56}),
    ("91 empty raw -> nil", {1: 1}, [], 1, None),
    ("nil receiver", None, [4, 4, 5], 0, {4: 0, 5: 0}),
    ("101 none new -> nil", {7: 3}, [7, 7], 1, None),
]

# (desc, s, s1, expected)   s.Intersection(s1); "EMPTY" = non-nil empty
INTERSECTION = [
    ("105-107 s1 nil -> nil", {1: 1}, None, None),
    ("105-107 s1 empty -> nil", {1: 1}, {}, None),
    ("108 nil receiver, s1 non-empty -> non-nil empty", None, {1: 1}, "EMPTY"),
    ("110 keep e if s1[e] >= s[e], with s's prio", {1: 1, 2: 2, 3: 3}, {1: 1, 2: 1, 4: 5}, {1: 1}),
    ("111 keeps the receiver's prio", {1: 0}, {1: 3}, {1: 0}),
    ("no overlap -> non-nil empty", {1: 0}, {2: 0}, "EMPTY"),
]

# (desc, s, s1, expected)   s.Merge(s1)
MERGE = [
    ("118-120 nil.Merge(nil) stays nil", None, None, None),
    ("118-120 merge of empty is a no-op", {1: 1}, {}, {1: 1}),
    ("121-125 nil receiver is allocated", None, {1: 1}, {1: 1}),
    ("127 max prio", {1: 1, 2: 3}, {1: 2, 2: 1, 3: -1}, {1: 2, 2: 3, 3: -1}),
]

# (desc, elems, prios, expected or "CORRUPT")   Serial{elems, prios}.Deserialize()
DESERIALIZE = [
    ("60-62 length mismatch panics", [1, 2], [1], "CORRUPT"),
    ("63-65 empty -> nil", [], [], None),
    ("67-69 later duplicate overwrites (even lower)", [1, 2, 1], [3, 1, 0], {1: 0, 2: 1}),
]

# Minimize (signal.go:138-166): contexts as dicts, expected surviving indices
MINIMIZE = [
    ("A covers 1,2; B raises 1; C unique; D only ties -> dropped",
     [{1: 1, 2: 1}, {1: 2}, {3: 0}, {2: 1}], [0, 1, 2]),
    ("equal Len and prio: the earlier context wins", [{5: 1}, {5: 1}], [0]),
    ("longer context sorts first and wins ties", [{5: 1}, {5: 1, 6: 0}], [1]),
    ("empty signal never wins", [{}, {1: 1}], [1]),
    ("empty corpus", [], []),
    ("strictly greater prio replaces the winner", [{1: 0, 2: 0}, {1: 1}], [0, 1]),
]

# checkNewSignal (fuzzer.go:494-511): (desc, M0, calls [(raw, prio)], exp_calls,
#   exp_max, exp_new, exp_new_records: per call the set of record indices in its DiffRaw result)
CHECK_NEW = [
    ("sequential merges across calls", {}, [([1, 2], 2), ([2, 3], 3), ([1, 4], 1)], [0, 1, 2],
     {1: 2, 2: 3, 3: 3, 4: 1}, {1: 2, 2: 3, 3: 3, 4: 1}, [{0, 1}, {0, 1}, {1}]),
    ("duplicates within a call are all in its diff", {}, [([7, 7], 1)], [0], {7: 1}, {7: 1}, [{0, 1}]),
    ("equal prio later is not new", {}, [([9], 1), ([9], 1)], [0], {9: 1}, {9: 1}, [{0}, set()]),
    ("lower then higher: both new", {}, [([9], 0), ([9], 2)], [0, 1], {9: 2}, {9: 2}, [{0}, {0}]),
    ("higher then lower: only first", {}, [([9], 3), ([9], 1)], [0], {9: 3}, {9: 3}, [{0}, set()]),
    ("M0 prio equal: not new; greater: new", {9: 2}, [([9], 2), ([9], 3)], [1], {9: 3}, {9: 3}, [set(), {0}]),
    ("empty calls are never new", {1: 0}, [([], 3), ([1], 1)], [1], {1: 1}, {1: 1}, [set(), {0}]),
    ("more than 4 distinct prios", {}, [([1], 0), ([1], 1), ([1], 2), ([1], 3), ([1], 4), ([1], 3), ([2], 200)],
     [0, 1, 2, 3, 4, 6], {1: 4, 2: -56}, {1: 4, 2: -56}, [{0}, {0}, {0}, {0}, {0}, set(), {0}]),
]
