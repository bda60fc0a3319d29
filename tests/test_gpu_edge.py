"""GPU: K1+K2 (edge.hip) bit-exact against the reference executor's own output
(golden vectors) and against the oracle on larger synthetic batches."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu

# K2's two marking modes (edge.hip), forced; None = the library's own choice
MODES = [None, "markall", "passes"]


@pytest.fixture
def mode(gpu, request):
    from syzkaller_amd._lib import SYZSIG_DEBUG_EDGE_MARKALL, SYZSIG_DEBUG_EDGE_PASSES

    m = request.param
    gpu.eng.set_debug({None: 0, "markall": SYZSIG_DEBUG_EDGE_MARKALL, "passes": SYZSIG_DEBUG_EDGE_PASSES}[m])
    yield m
    gpu.eng.set_debug(0)


def _run(gpu, pcs, call_start, call_len, prog_call):
    d = gpu.dev
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(d)  # noqa: E731
    sigs, cnt, comp = gpu.edge_derive(t(pcs, np.int64), t(call_start, np.int64), t(call_len, np.int32),
                                      t(prog_call, np.int32))
    torch.cuda.synchronize()
    return (sigs.cpu().numpy().view(np.uint32), cnt.cpu().numpy().view(np.uint32),
            comp.cpu().numpy().view(np.uint32))


def _check(fx_sigs, fx_cnt, fx_comp, call_start, sigs, cnt, comp):
    np.testing.assert_array_equal(comp, fx_comp)
    np.testing.assert_array_equal(cnt, fx_cnt)
    for c in range(len(call_start)):
        s, n = int(call_start[c]), int(fx_cnt[c])
        np.testing.assert_array_equal(sigs[s: s + n], fx_sigs[s: s + n], err_msg=f"call {c}")


@pytest.mark.parametrize("mode", MODES, indirect=True)
@pytest.mark.parametrize("name", golden_names())
def test_edge_matches_reference_executor_goldens(gpu, name, mode):
    fx = load_golden(name)
    out = _run(gpu, fx["pcs"], fx["call_start"], fx["call_len"], fx["prog_call"])
    _check(fx["exp_sigs"], fx["exp_cnt"], fx["exp_completed"], fx["call_start"], *out)


@pytest.mark.parametrize("over,ragged", [({}, None), ({"region_log2": 12}, (0, 3000)),
                                          ({"bad_pc_ppm": 20}, (0, 4000)), ({"skew": 1}, None),
                                          ({"global_walk": 1}, None)])
@pytest.mark.parametrize("mode", MODES[1:], indirect=True)
def test_edge_c1_batch_vs_oracle(gpu, over, ragged, mode):
    """Config 1 shape: 64 programs x 32 calls x 2k PCs (ragged variants)."""
    from syzkaller_amd import synth

    cfg = synth.synth_default(**over)
    nprog, cpp = 64, 32
    cl = synth.call_lengths(nprog, cpp, 2048, ragged=ragged, seed=1)
    pcs, cs, prio = synth.traces(cfg, 0, nprog, cpp, cl)
    pidx = synth.prog_call_index(nprog, cpp)
    exp = O.exec_batch(pcs, cs, cl, pidx)
    out = _run(gpu, pcs, cs, cl, pidx)
    _check(*exp, cs, *out)


@pytest.mark.parametrize("over", [{"skew": 1}, {"skew": 2, "global_walk": 1}])
def test_device_synth_matches_host(gpu, over):
    from syzkaller_amd import synth

    cfg = synth.synth_default(**over)
    cl = synth.call_lengths(16, 8, 0, ragged=(0, 3000), seed=4)
    pcs, cs, prio = synth.traces(cfg, 5, 16, 8, cl)
    dpcs, dcs, dcl, dprio = gpu.synth_traces(cfg, 5, 16, 8, torch.from_numpy(cl.view(np.int32)))
    np.testing.assert_array_equal(dpcs.cpu().numpy().view(np.uint64), pcs)
    np.testing.assert_array_equal(dprio.cpu().numpy(), prio)
    e, p = synth.m0(cfg, 10, 20000)
    de, dp = gpu.synth_m0(cfg, 10, 20000)
    np.testing.assert_array_equal(de.cpu().numpy().view(np.uint32), e)
    np.testing.assert_array_equal(dp.cpu().numpy(), p)


def test_edge_rejects_oversized_call(gpu):
    from syzkaller_amd._lib import SyzsigError

    n = 262144  # kCoverSize: executor_linux.cc:186-187 fail("too much cover")
    pcs = np.full(n, 0xFFFFFFFF81000000, np.uint64)
    with pytest.raises(SyzsigError):
        _run(gpu, pcs, np.array([0], np.uint64), np.array([n], np.uint32), np.array([0, 1], np.uint32))


@pytest.mark.parametrize("mode", ["markall"], indirect=True)
def test_edge_markall_clear_after_one_round_chunks(gpu, mode):
    """in the mark-all mode a chunk that leaves no lane
    pending after its first round clears its slot marks and returns with no
    barrier behind the clear, while the next chunk of the same prefetch group
    marks with no K1 barrier in front of it.  The trace alternates such chunks
    with chunks of colliding pairs (whose lost marks would let a blocked lane
    write), over 1024 programs so many waves interleave; bit-exact against the
    oracle (which the CPU test pins to the round restatement's shape)."""
    from tests.test_edge_rounds_cpu import clear_race_trace

    pcs, cs, cl, pidx = clear_race_trace(1024, nchunks=16, seed=11)
    exp = O.exec_batch(pcs, cs, cl, pidx)
    for _ in range(3):
        out = _run(gpu, pcs, cs, cl, pidx)
        _check(*exp, cs, *out)
