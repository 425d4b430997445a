"""Counter slots of the dynamically scheduled kernels (include/kvecc.h
kvecc_reserve_counter_slots): launches that can overlap never share counters.

The fused shim reads (Golay and interpolating Hamming(8,4)), the per-head Golay
rows decode and the packed Golay decode take tiles from work counters
(TileSchedule); MHA paged attention's fused combine counts finished splits.
Each of these kernels needs its counters zero and to itself while it runs.
The library gives every stream its own slot and every captured (graph, stream)
one more.  Here more than 65 such launches alternate between two streams with
nothing ordering them, and a captured graph replays beside eager launches on
another stream.  Every output and statistic must equal a single-stream
baseline, which equals the host twin (the reads) bit for bit, and afterwards
every counter of every slot must be back to zero.  The reference has no
counterpart: it launches one Triton program per row (ecc_shim.py:626-737,
990-1071) and schedules nothing.
"""

import math

import pytest
import torch

from tests.test_shim_read_batch import make_cache

pytestmark = pytest.mark.gpu

# big enough for the dynamic tail: more tiles than the persistent grid's waves
B, L, H, D, BS = 4, 4096, 8, 128, 16


def _workloads(dev):
    """name -> (run(out_bufs, stats), make_out(), host reference or None)."""
    from kvecc import cpu_ops, ops
    work = {}
    kc, vc, ks, vs, table = make_cache("golay", B, L, H, D, BS, layers=1, seed=3, ber=1e-2)
    g = {n: t.to(dev) for n, t in dict(kc=kc, vc=vc, ks=ks, vs=vs, table=table).items()}
    ref = cpu_ops.shim_read_batch(kc, vc, ks, vs, table, L, D, 0, "golay", torch.float16,
                                  stats=cpu_ops.new_stats())
    work["golay_read"] = (
        lambda o, st: ops.shim_read_batch(g["kc"], g["vc"], g["ks"], g["vs"], g["table"], L, D, 0, "golay",
                                          torch.float16, stats=st, out=o),
        lambda: tuple(torch.empty(B, H, L, D, dtype=torch.float16, device=dev) for _ in range(2)), ref)

    hk, hv, hks, hvs, htab = make_cache("hamming84", B, L, H, D, BS, layers=1, seed=4, ber=1e-3)
    h = {n: t.to(dev) for n, t in dict(kc=hk, vc=hv, ks=hks, vs=hvs, table=htab).items()}
    href = cpu_ops.shim_read_batch(hk, hv, hks, hvs, htab, L, D, 0, "hamming84", torch.float16,
                                   stats=cpu_ops.new_stats(), interp=True)
    work["h84_interp_read"] = (
        lambda o, st: ops.shim_read_batch(h["kc"], h["vc"], h["ks"], h["vs"], h["table"], L, D, 0, "hamming84",
                                          torch.float16, stats=st, interp=True, out=o),
        lambda: tuple(torch.empty(B, H, L, D, dtype=torch.float16, device=dev) for _ in range(2)), href)

    rows = g["kc"].view(-1, (D + 2) // 3)
    work["golay_rows"] = (
        lambda o, st: ops.golay_decode_rows_into(rows, o[0], stats=st),
        lambda: (torch.empty(rows.shape[0], D, dtype=torch.uint8, device=dev),), None)

    m = rows.numel()
    pk = rows.reshape(-1).view(torch.uint8).view(-1, 4)[:, :3].contiguous().view(-1)  # 3 bytes per codeword
    work["golay_packed"] = (
        lambda o, st: ops.golay_decode_packed_into(pk, o[0], m=m, stats=st),
        lambda: (torch.empty((3 * m + 1) // 2, dtype=torch.uint8, device=dev),), None)

    gen = torch.Generator().manual_seed(5)
    q = torch.randn(B, H, D, generator=gen).to(dev)
    lens = torch.full((B,), L, dtype=torch.int32, device=dev)
    work["attn_mha"] = (
        lambda o, st: ops.paged_attention_into(q, h["kc"], h["vc"], h["table"], lens, h["ks"], h["vs"], o[0], 0, BS,
                                               1 / math.sqrt(D), "hamming84", L),
        lambda: (torch.empty(B, H, D, dtype=torch.float32, device=dev),), None)
    return work


def _same(a, b):
    return all(torch.equal(x, y) for x, y in zip(a, b))


def test_two_streams_and_graph_replay_keep_counters_private(gpu):
    from kvecc import ops
    dev = gpu
    work = _workloads(dev)
    names = list(work)
    # single-stream baseline (and the host twin where there is one)
    base, base_st = {}, {}
    for n, (run, mk, ref) in work.items():
        o, st = mk(), ops.new_stats(dev)
        run(o, st)
        torch.cuda.synchronize()
        base[n] = tuple(t.clone() for t in o)
        base_st[n] = ops.read_stats(st)
        if ref is not None:
            assert all(torch.equal(x.cpu(), y) for x, y in zip(o, ref)), n
    s = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    outs = {(k, n): work[n][1]() for k in range(2) for n in names}
    stats = {(k, n): ops.new_stats(dev) for k in range(2) for n in names}
    count = {key: 0 for key in outs}
    torch.cuda.synchronize()
    launches = 0
    for i in range(80):  # > 64 dynamically scheduled launches, alternating streams
        k, n = i % 2, names[(i // 2) % len(names)]
        with torch.cuda.stream(s[k]):
            work[n][0](outs[(k, n)], stats[(k, n)])
        count[(k, n)] += 1
        launches += 1
    assert launches > 64
    # a graph of every workload, captured on a third stream, replayed beside
    # eager launches on the first
    s3 = torch.cuda.Stream(dev)
    gout = {n: work[n][1]() for n in names}
    gst = {n: ops.new_stats(dev) for n in names}
    torch.cuda.synchronize()
    ops.reserve_counter_slots(8, dev)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s3):
        for n in names:
            work[n][0](gout[n], gst[n])
    torch.cuda.synchronize()
    for st in gst.values():
        st.zero_()
    s3.wait_stream(torch.cuda.current_stream())  # the zeroing lands before the replays
    replays = 0
    for i in range(12):
        with torch.cuda.stream(s3):
            graph.replay()
        replays += 1
        n = names[i % len(names)]
        with torch.cuda.stream(s[0]):
            work[n][0](outs[(0, n)], stats[(0, n)])
        count[(0, n)] += 1
    torch.cuda.synchronize()
    for (k, n), o in outs.items():
        if count[(k, n)]:
            assert _same(o, base[n]), (k, n)
            got = ops.read_stats(stats[(k, n)])
            assert got == [v * count[(k, n)] for v in base_st[n]], (k, n, got, base_st[n])
    for n in names:
        assert _same(gout[n], base[n]), ("graph", n)
        assert ops.read_stats(gst[n]) == [v * replays for v in base_st[n]], ("graph", n)
    used, nonzero = ops.counter_slots_check(dev)
    assert nonzero == 0, f"{nonzero} counter words left non-zero in {used} slots"
    assert used >= 3  # default stream, two side streams, the graph's (plus any torch used)


def test_counter_slots_check_api(gpu):
    from kvecc import ops
    used, nonzero = ops.counter_slots_check(gpu)
    assert used >= 0 and nonzero == 0
    ops.reserve_counter_slots(4, gpu)


def test_many_captures_on_one_stream_and_slot_release(gpu):
    """A serving loop's pattern: warm up eagerly, capture, repeat -- 80 graphs on
    one stream, all alive at once, with no kvecc_reserve_counter_slots call (the
    eager launches keep the capture reserve topped up).  Every graph's slot is
    its own while the graph lives, every replay is exact, and the slots return
    to the pool when the graphs are destroyed (HIP user objects)."""
    import gc
    import time

    from kvecc import ops
    dev = gpu
    work = _workloads(dev)
    run, mk, _ = work["golay_rows"]
    base, st = mk(), ops.new_stats(dev)
    run(base, st)
    torch.cuda.synchronize()
    base_st = ops.read_stats(st)
    s = torch.cuda.Stream(dev)
    out = mk()
    used0, _ = ops.counter_slots_check(dev)
    graphs, gstats = [], []
    for i in range(80):
        with torch.cuda.stream(s):
            run(out, ops.new_stats(dev))  # eager warm-up on the capture stream
        g, gs = torch.cuda.CUDAGraph(), ops.new_stats(dev)
        with torch.cuda.graph(g, stream=s):
            run(out, gs)
        graphs.append(g)
        gstats.append(gs)
    torch.cuda.synchronize()
    used1, nz = ops.counter_slots_check(dev)
    assert nz == 0 and used1 >= used0 + 80, (used0, used1)
    for g, gs in zip(graphs, gstats):
        gs.zero_()
        for t in out:
            t.zero_()
        s.wait_stream(torch.cuda.current_stream())  # the zeroing lands before the replay
        with torch.cuda.stream(s):
            g.replay()
        torch.cuda.synchronize()
        assert _same(out, base) and ops.read_stats(gs) == base_st
    del graphs, g
    gc.collect()
    torch.cuda.synchronize()
    t0 = time.time()
    used2 = used1
    while time.time() - t0 < 5:
        used2, nz = ops.counter_slots_check(dev)
        if used2 <= used0 + 1:
            break
        time.sleep(0.1)
    assert nz == 0
    assert used2 <= used0 + 1, f"captured slots not returned: {used0} before, {used1} alive, {used2} after"


def _hip_streams(n):
    """n new HIP streams of the runtime torch loaded (torch.cuda.Stream() hands
    out 32 pooled streams per priority round-robin: the 33rd is the 1st again,
    possibly the capture stream itself)."""
    import ctypes
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    hip = ctypes.CDLL(path)
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    raw = []
    for _ in range(n):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        raw.append(h.value)
    return [torch.cuda.ExternalStream(h) for h in raw], lambda: [hip.hipStreamDestroy(h) for h in raw]


def test_eager_launches_beside_a_global_capture_grow_the_pool(gpu):
    """torch.cuda.graph captures in global mode by default, which forbids hipMalloc
    and stream syncs from every thread.  While stream A captures, eager launches
    on 70 new streams each take a slot of their own, so the pool grows past its
    reserve in the middle of the capture (the library allocates in relaxed
    mode); neither the eager results nor the capture may break."""
    from kvecc import ops
    dev = gpu
    run, mk, _ = _workloads(dev)["golay_rows"]
    base, st = mk(), ops.new_stats(dev)
    run(base, st)
    torch.cuda.synchronize()
    base_st = ops.read_stats(st)
    used0, _ = ops.counter_slots_check(dev)
    side, destroy = _hip_streams(70)
    outs = [mk() for _ in side]
    for o in outs:
        o[0].fill_(0xEE)
    sts = [ops.new_stats(dev) for _ in side]
    a = torch.cuda.Stream(dev)
    gout, gst = mk(), ops.new_stats(dev)
    with torch.cuda.stream(a):
        run(gout, ops.new_stats(dev))  # eager warm-up on the capture stream
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=a):
        run(gout, gst)
        for s, o, t in zip(side, outs, sts):
            with torch.cuda.stream(s):
                run(o, t)
    torch.cuda.synchronize()
    bad = [i for i, (o, t) in enumerate(zip(outs, sts)) if not (_same(o, base) and ops.read_stats(t) == base_st)]
    assert not bad, bad
    used1, nz = ops.counter_slots_check(dev)
    assert nz == 0 and used1 >= used0 + 70, (used0, used1)
    gst.zero_()
    for t in gout:
        t.zero_()
    a.wait_stream(torch.cuda.current_stream())  # the zeroing lands before the replay
    with torch.cuda.stream(a):
        g.replay()
    torch.cuda.synchronize()
    assert _same(gout, base) and ops.read_stats(gst) == base_st
    del g
    destroy()


def test_failed_graph_retain_keeps_the_slot_with_its_capture(gpu):
    """when the slot cannot be tied to its graph (the retain step
    fails; forced here through kvecc_debug_fail_graph_retain), the slot must
    stay with the capture for the process's life -- never go back to the pool
    while the graph can still replay.  So: the graph still replays exactly
    after 40 eager launches on new streams (each taking a slot of its own), and
    destroying the graph does not return its slot."""
    import gc
    import time

    from kvecc import _lib, ops
    dev = gpu
    run, mk, _ = _workloads(dev)["golay_rows"]
    base, st = mk(), ops.new_stats(dev)
    run(base, st)
    torch.cuda.synchronize()
    base_st = ops.read_stats(st)
    s = torch.cuda.Stream(dev)
    out, gs = mk(), ops.new_stats(dev)
    with torch.cuda.stream(s):
        run(out, ops.new_stats(dev))
    torch.cuda.synchronize()
    used0, _ = ops.counter_slots_check(dev)
    _lib.call("kvecc_debug_fail_graph_retain", 1)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            run(out, gs)
    finally:
        _lib.call("kvecc_debug_fail_graph_retain", 0)
    torch.cuda.synchronize()
    used1, _ = ops.counter_slots_check(dev)
    assert used1 == used0 + 1, (used0, used1)
    side, destroy = _hip_streams(40)
    outs = [mk() for _ in side]
    for sd, o in zip(side, outs):
        with torch.cuda.stream(sd):
            run(o, ops.new_stats(dev))
    gs.zero_()
    for t in out:
        t.zero_()
    # the zeroing (default stream, behind the blocking side streams' launches)
    # must land before the replay on the non-blocking capture stream
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.replay()
    torch.cuda.synchronize()
    assert _same(out, base) and ops.read_stats(gs) == base_st
    assert all(_same(o, base) for o in outs)
    used2, _ = ops.counter_slots_check(dev)
    del g
    gc.collect()
    torch.cuda.synchronize()
    time.sleep(0.5)
    used3, nz = ops.counter_slots_check(dev)
    assert nz == 0
    assert used3 == used2, f"the unretained slot went back to the pool: {used2} -> {used3}"
    destroy()
