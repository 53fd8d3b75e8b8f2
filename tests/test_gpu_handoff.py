"""GPU: the cross-workgroup and host hand-offs under forced interleavings.

The engine's in-kernel hand-offs between workgroups are the fused 2-means
pass (kpass_kernel): every workgroup of a record publishes its tile partial
and per-wave counts, and the record's last arriver reads them all
(DESIGN.md 3b); and kpersist_kernel, which does the same once per iteration
and then publishes the record's next decision to the record's other
workgroups.  The host hand-offs are the round results and status words in
host-coherent memory, reused by round parity.  Each test forces the state the
protocol must tolerate (dq_hip_set_debug flags, dq_kernels.h kDebug*) and
checks every output against the reference build's fixtures:

* prewarm -- every workgroup loads its record's partial / count lines into its
  own L1 and its XCD's L2 before storing its own, so a last arriver that read
  them without an agent-scope acquire would see stale values;
* uneven -- 1 in 8 workgroups of the 2-means passes, partitions and epilogues
  stall ~10 us before publishing (late last arrivers, uneven XCD load);
* host delay -- the host sleeps 200 us between a round's status word and its
  results (the GPU runs ahead into the other parity slot);
* plan stall -- the plan kernel publishes its counts ~20 us late.

Each configuration runs once (three calls); a failure names the frame and the
check (colortable or output hash).
"""
import numpy as np
import pytest

import dq_fixtures as fx

pytestmark = pytest.mark.gpu

W4, H4 = 3840, 2160
ALL = 1 | 2 | 4 | 8


def _c4_share(gpu, flags, lanes, calls=3):
    import torch
    fix = fx.load_json("c4.json")
    t_in = [torch.from_numpy(fx.xorshift(W4 * H4, seed=fx.SEED + f).view(np.int32)).to("cuda:0")
            for f in range(8)]
    t_out = [torch.empty_like(t) for t in t_in]
    gpu.set_lanes(lanes)
    gpu.set_debug(flags)
    try:
        for c in range(calls):
            for t in t_out:
                t.fill_(-1)
            cts, _ = gpu.quant_batch_device(t_in, t_out, 256)
            torch.cuda.synchronize()
            for f in range(8):
                ref = fix["f%02d" % f]
                assert [int(v) for v in cts[f]] == ref["ct"], ("call", c, "frame", f, "colortable")
                assert "%016x" % fx.fnv(t_out[f].cpu().numpy().view(np.uint32)) == ref["out_fnv"], \
                    ("call", c, "frame", f, "output")
    finally:
        gpu.set_debug(0)
        gpu.set_lanes(0)


@pytest.mark.parametrize("flags", [1, 1 | 2, ALL])
def test_kpass_handoff_forced_interleavings_one_lane(gpu, flags):
    _c4_share(gpu, flags, lanes=1)


def test_handoffs_forced_interleavings_three_lanes(gpu):
    _c4_share(gpu, ALL, lanes=3)


@pytest.mark.parametrize("persist", [True, False])
def test_c3_forced_interleavings(gpu, persist):
    """C3 (one 4K frame per call): its last round's 2-means iterations start
    before the split status (speculation) -- the chain the host delay and the
    plan stall shift the most.  persist: they run as one kpersist_kernel
    launch, whose records' workgroups meet per iteration on device counters
    (prewarm: every workgroup loads its record's lines before it waits, so a
    wait without the agent-scope acquire would re-read a stale decision;
    uneven: 1 in 8 workgroups arrive ~10 us late per iteration)."""
    import torch
    fix = fx.load_json("c4.json")["f00"]
    t_in = torch.from_numpy(fx.xorshift(W4 * H4).view(np.int32)).to("cuda:0")
    t_out = torch.empty_like(t_in)
    gpu.set_persist(persist)
    gpu.set_debug(ALL)
    try:
        for c in range(3):
            ct, _ = gpu.quant_device(t_in, t_out, 256)
            torch.cuda.synchronize()
            assert (gpu.last_persist_rounds() > 0) == persist
            assert [int(v) for v in ct] == fix["ct"], c
            assert "%016x" % fx.fnv(t_out.cpu().numpy().view(np.uint32)) == fix["out_fnv"], c
    finally:
        gpu.set_debug(0)
        gpu.set_persist(True)
