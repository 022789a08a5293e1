"""Parity of the HIP path (through the C ABI) against the CPU oracle and the golden vectors.

Bit-exact is the only bar: the filter is integer byte work (inverter.py:41).  Sizes: the
golden KATs and seeded frames at 480x480 / 480p / 1080p / 4K, configs[1]'s 32 x 1080p batch,
mixed-resolution gathers (configs[3]), and configs[4]'s smallest HBM-resident sweep point
(256 x 1080p = 1.59 GB) checked by size-independent properties (double inversion is the
identity; every frame's digest matches the expected one).
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import vfilter
from oracle import oracle

pytestmark = pytest.mark.gpu

FB_1080 = 1080 * 1920 * 3


def _kats(golden_dir):
    with open(os.path.join(golden_dir, "kat.json")) as f:
        return json.load(f)["kats"]


def test_kats_through_bitwise_not(vf_ctx, golden_dir):
    for k in _kats(golden_dir):
        raw = bytes.fromhex(k["input_hex"])
        x = np.frombuffer(raw, dtype=np.uint8).reshape(k["shape"])  # read-only view, as inverter.py:34
        y = vfilter.bitwise_not(x, ctx=vf_ctx)
        assert y.shape == x.shape and y.dtype == np.uint8
        assert y.tobytes() == bytes.fromhex(k["expected_hex"]), k["name"]
        assert x.tobytes() == raw  # input untouched


def test_seeded_frames_all_sizes(vf_ctx, golden_dir):
    with open(os.path.join(golden_dir, "seeded_digests.json")) as f:
        recs = json.load(f)["frames"]
    for r in recs:
        h, w, _ = r["shape"]
        x = oracle.synthetic_frame(r["seed"], h, w)
        assert hashlib.sha256(x.tobytes()).hexdigest() == r["input_sha256"]
        y = vfilter.bitwise_not(x, ctx=vf_ctx)
        assert hashlib.sha256(y.tobytes()).hexdigest() == r["expected_sha256"], (r["size"], r["seed"])


def test_dst_argument_and_in_place(vf_ctx):
    x = oracle.synthetic_frame(3, 480, 640)
    want = oracle.invert(x)
    out = np.empty_like(x)
    assert vfilter.bitwise_not(x, out, ctx=vf_ctx) is out
    assert np.array_equal(out, want)
    vfilter.bitwise_not(out, out, ctx=vf_ctx)  # in place
    assert np.array_equal(out, x)


def test_batch_configs1_1080p_x32(vf_ctx):
    frames = np.stack([oracle.synthetic_frame(s, 1080, 1920) for s in range(32)])
    out = vfilter.invert_batch(frames, ctx=vf_ctx)
    assert np.array_equal(out, oracle.c_invert(frames))
    assert vf_ctx.elapsed_ms() > 0.0


def test_mixed_resolution_frames(vf_ctx):
    shapes = [(480, 640), (1080, 1920), (2160, 3840), (17, 13), (1, 1), (0, 0), (480, 480)] * 2
    frames = [oracle.synthetic_frame(i, h, w) for i, (h, w) in enumerate(shapes)]
    outs = vfilter.invert_frames(frames, ctx=vf_ctx)
    for f, o in zip(frames, outs):
        assert o.shape == f.shape and np.array_equal(o, oracle.invert(f))
    # bytes objects (the worker's wire payloads) work as sources too
    outs = vfilter.invert_frames([f.tobytes() for f in frames], ctx=vf_ctx)
    for f, o in zip(frames, outs):
        assert o.tobytes() == oracle.invert_bytes(f.tobytes())


@pytest.mark.parametrize("soff,doff", [(0, 0), (1, 1), (3, 7), (15, 0), (8, 9)])
def test_unaligned_host_buffers(vf_ctx, soff, doff):
    n = 1_000_003
    base_s = np.zeros(n + 32, np.uint8)
    base_d = np.zeros(n + 32, np.uint8)
    base_s[soff:soff + n] = np.random.default_rng(soff * 31 + doff).integers(0, 256, n, dtype=np.uint8)
    vf_ctx.invert_host(base_s[soff:soff + n], base_d[doff:doff + n], n)
    assert np.array_equal(base_d[doff:doff + n], oracle.c_invert(base_s[soff:soff + n]))
    assert not base_d[:doff].any() and not base_d[doff + n:].any()  # no stray writes


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 4095, 4096 * 4 + 5, 8 << 20, (8 << 20) + 1, 3 * (8 << 20) + 77])
def test_sizes_around_tile_and_slot_boundaries(vf_ctx, n):
    x = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    y = np.empty_like(x)
    vf_ctx.invert_host(x, y, n)
    assert np.array_equal(y, oracle.invert(x))


@pytest.mark.parametrize("soff,doff", [(0, 0), (5, 5), (2, 11), (0, 1)])
def test_device_entry_alignment(vf_ctx, soff, doff):
    n = 3_000_001
    x = np.random.default_rng(11).integers(0, 256, n, dtype=np.uint8)
    ds = vf_ctx.alloc_device(n + 64)
    dd = vf_ctx.alloc_device(n + 64)
    try:
        vf_ctx.memset_device(dd, 0, n + 64)
        vf_ctx.upload(ds + soff, x, n)
        vf_ctx.invert_device(ds + soff, dd + doff, n)
        vf_ctx.sync()
        y = np.empty(n + 64, np.uint8)
        vf_ctx.download(y, dd, n + 64)
        vf_ctx.sync()
        assert np.array_equal(y[doff:doff + n], oracle.invert(x))
        assert not y[:doff].any() and not y[doff + n:].any()
    finally:
        vf_ctx.free_device(ds)
        vf_ctx.free_device(dd)


def test_device_all_relative_offsets(vf_ctx):
    """Every (src mod 16, dst mod 16) pair: equal offsets take the streaming kernel, unequal
    ones the shifting kernel (aligned stores, v_alignbyte funnel shifts).  Sizes below, at and
    across one 16-KiB tile; no byte outside [dst, dst + n) is touched."""
    x = np.random.default_rng(5).integers(0, 256, 70_000, dtype=np.uint8)
    ds = vf_ctx.alloc_device(x.nbytes + 64)
    dd = vf_ctx.alloc_device(x.nbytes + 64)
    try:
        vf_ctx.upload(ds, np.zeros(x.nbytes + 64, np.uint8), x.nbytes + 64)
        for soff in range(16):
            vf_ctx.upload(ds + soff, x, x.nbytes)
            for doff in range(16):
                for n in (1, 15, 17, 4095, 16 * 1024 + 5, 70_000 - 16):
                    vf_ctx.memset_device(dd, 0x5A, x.nbytes + 64)
                    vf_ctx.invert_device(ds + soff, dd + doff, n)
                    y = np.empty(x.nbytes + 64, np.uint8)
                    vf_ctx.download(y, dd, y.nbytes)
                    vf_ctx.sync()
                    assert np.array_equal(y[doff:doff + n], oracle.invert(x[:n])), (soff, doff, n)
                    assert (y[:doff] == 0x5A).all() and (y[doff + n:] == 0x5A).all(), (soff, doff, n)
    finally:
        vf_ctx.free_device(ds)
        vf_ctx.free_device(dd)


def test_device_frames_every_offset(vf_ctx):
    """The descriptor kernel with 32 frames at every src/dst offset mod 16 (aligned and
    shifted paths in one launch), sizes from 1 B to a 1080p frame."""
    rng = np.random.default_rng(9)
    sizes = [int(v) for v in rng.integers(1, 200_000, 31)] + [1920 * 1080 * 3]
    frames = [rng.integers(0, 256, n, dtype=np.uint8) for n in sizes]
    srcs = [vf_ctx.alloc_device(n + 32) for n in sizes]
    dsts = [vf_ctx.alloc_device(n + 32) for n in sizes]
    soffs = [i % 16 for i in range(32)]
    doffs = [(7 * i + 3) % 16 for i in range(32)]
    tables = [vf_ctx.alloc_device(8 * 32) for _ in range(3)]
    try:
        for f, s, o in zip(frames, srcs, soffs):
            vf_ctx.upload(s + o, f, f.nbytes)
        for d, n in zip(dsts, sizes):
            vf_ctx.memset_device(d, 0x5A, n + 32)
        sp = np.array([s + o for s, o in zip(srcs, soffs)], np.uint64)
        dp = np.array([d + o for d, o in zip(dsts, doffs)], np.uint64)
        nb = np.array(sizes, np.uint64)
        for t, a in zip(tables, (sp, dp, nb)):
            vf_ctx.upload(t, a, a.nbytes)
        vf_ctx.invert_device_frames(tables[0], tables[1], tables[2], 32, sum(sizes))
        vf_ctx.sync()
        for f, d, o, n in zip(frames, dsts, doffs, sizes):
            y = np.empty(n + 32, np.uint8)
            vf_ctx.download(y, d, n + 32)
            vf_ctx.sync()
            assert np.array_equal(y[o:o + n], np.bitwise_not(f)), (o, n)
            assert (y[:o] == 0x5A).all() and (y[o + n:] == 0x5A).all()
    finally:
        for p in srcs + dsts + tables:
            vf_ctx.free_device(p)


@pytest.mark.parametrize("soff,n", [(3, (600 << 20) + 77), (0, (512 << 20) + 16), (7, 1_300_000_009)])
def test_device_split_launch_ragged(vf_ctx, soff, n):
    """Bodies above 512 MiB are cut into <= 256 MiB sub-launches (vf_kernels.hip
    launch_stream): the head goes with the first, the tail with the last; no byte outside
    [dst, dst+n) is touched.  Checked against the oracle on the whole range."""
    x = np.random.default_rng(n & 0xFFFF).integers(0, 256, n, dtype=np.uint8)
    ds = vf_ctx.alloc_device(n + 64)
    dd = vf_ctx.alloc_device(n + 64)
    try:
        vf_ctx.memset_device(dd, 0x5A, n + 64)
        vf_ctx.upload(ds + soff, x, n)
        vf_ctx.invert_device(ds + soff, dd + soff, n)
        vf_ctx.sync()
        y = np.empty(n + 64, np.uint8)
        vf_ctx.download(y, dd, n + 64)
        vf_ctx.sync()
        assert np.array_equal(y[soff:soff + n], oracle.invert(x))
        assert (y[:soff] == 0x5A).all() and (y[soff + n:] == 0x5A).all()
    finally:
        vf_ctx.free_device(ds)
        vf_ctx.free_device(dd)


def test_device_frames_descriptor_kernel(vf_ctx):
    shapes = [(480, 640), (1080, 1920), (2160, 3840), (17, 13), (480, 480)]
    frames = [oracle.synthetic_frame(40 + i, h, w) for i, (h, w) in enumerate(shapes)]
    sizes = [f.nbytes for f in frames]
    srcs = [vf_ctx.alloc_device(s + 16) for s in sizes]
    dsts = [vf_ctx.alloc_device(s + 16) for s in sizes]
    offs = [0, 3, 0, 1, 0]  # one misaligned frame exercises the per-frame byte path
    tables = [vf_ctx.alloc_device(8 * len(frames)) for _ in range(3)]
    try:
        for f, s, o in zip(frames, srcs, offs):
            vf_ctx.upload(s + o, f, f.nbytes)
        sp = np.array([s + o for s, o in zip(srcs, offs)], np.uint64)
        dp = np.array([d + o for d, o in zip(dsts, offs)], np.uint64)
        nb = np.array(sizes, np.uint64)
        for t, a in zip(tables, (sp, dp, nb)):
            vf_ctx.upload(t, a, a.nbytes)
        vf_ctx.invert_device_frames(tables[0], tables[1], tables[2], len(frames), sum(sizes))
        vf_ctx.sync()
        for f, d, o in zip(frames, dsts, offs):
            y = np.empty(f.nbytes, np.uint8)
            vf_ctx.download(y, d + o, f.nbytes)
            vf_ctx.sync()
            assert y.tobytes() == oracle.invert_bytes(f.tobytes())
    finally:
        for p in srcs + dsts + tables:
            vf_ctx.free_device(p)


def test_pinned_and_registered_host_memory(vf_ctx):
    n = 32 * FB_1080 // 8
    x = np.random.default_rng(5).integers(0, 256, n, dtype=np.uint8)
    # pinned allocations from the library: direct DMA, no staging copy
    ps, pd = vf_ctx.alloc_host(n), vf_ctx.alloc_host(n)
    try:
        hs = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ps))
        hd = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(pd))
        hs[:] = x
        vf_ctx.invert_host(ps, pd, n)
        assert np.array_equal(hd, oracle.invert(x))
    finally:
        vf_ctx.free_host(ps)
        vf_ctx.free_host(pd)
    # an existing buffer page-locked in place (what a shared-memory frame ring does)
    src = np.ascontiguousarray(x)
    dst = np.zeros_like(src)
    a = vf_ctx.host_register(src)
    b = vf_ctx.host_register(dst)
    try:
        vf_ctx.invert_host(src, dst, n)
        assert np.array_equal(dst, oracle.invert(x))
    finally:
        vf_ctx.host_unregister(a)
        vf_ctx.host_unregister(b)


def test_errors_are_raised_not_swallowed(vf_ctx):
    x = np.zeros(100, np.uint8)
    with pytest.raises(vfilter.VFilterError, match="partially overlap"):
        vf_ctx.invert_host(x[:90], x[5:95], 90)
    with pytest.raises(vfilter.VFilterError):
        vf_ctx.invert_frames_host([x], [x[1:]], [99])  # partial overlap inside a frame
    with pytest.raises(NotImplementedError):
        vfilter.bitwise_not(x, mask=x, ctx=vf_ctx)


def test_hbm_resident_sweep_point_batch256(vf_ctx):
    """configs[4] smallest point: 256 x 1080p (1.59 GB) resident in HBM, one call (7 sub-launches)."""
    n_frames = 256
    total = n_frames * FB_1080
    seeds = [0, 1, 2, 3]
    base = [oracle.synthetic_frame(s, 1080, 1920).reshape(-1) for s in seeds]
    inv = [oracle.invert(b) for b in base]
    ds, d1, d2 = (vf_ctx.alloc_device(total) for _ in range(3))
    try:
        for f in range(n_frames):
            vf_ctx.upload(ds + f * FB_1080, base[f % 4], FB_1080)
        vf_ctx.invert_device(ds, d1, total)
        vf_ctx.invert_device(d1, d2, total)  # ~~x == x
        vf_ctx.sync()
        y = np.empty(FB_1080, np.uint8)
        for f in list(range(0, n_frames, 17)) + [n_frames - 1]:
            vf_ctx.download(y, d1 + f * FB_1080, FB_1080)
            vf_ctx.sync()
            assert np.array_equal(y, inv[f % 4]), f
            vf_ctx.download(y, d2 + f * FB_1080, FB_1080)
            vf_ctx.sync()
            assert np.array_equal(y, base[f % 4]), f
        # whole-buffer check: every frame of d2 equals the source frame
        big = np.empty(total, np.uint8)
        vf_ctx.download(big, d1, total)
        vf_ctx.sync()
        big = big.reshape(n_frames, FB_1080)
        for k in range(4):
            assert np.array_equal(big[k::4], np.broadcast_to(inv[k], big[k::4].shape))
    finally:
        for p in (ds, d1, d2):
            vf_ctx.free_device(p)


def _digests_1080p(golden_dir):
    with open(os.path.join(golden_dir, "seeded_digests.json")) as f:
        recs = {r["seed"]: r for r in json.load(f)["frames"] if r["size"] == "1080p"}
    return ([recs[s]["input_sha256"] for s in range(4)], [recs[s]["expected_sha256"] for s in range(4)])


def test_hbm_resident_sweep_top_batch4096(vf_ctx, golden_dir):
    """configs[4] top point: 4096 x 1080p = 25.48 GB resident in, the same out, ONE
    vf_invert_device call (the bench's configs4_sweep shape), then ~~x over the whole buffer.

    Every frame of both outputs is checked by sha256 against the golden seeded digests
    (frame f holds seed f % 4).  Byte offsets cross 2^32, 2^33 and 2^34: the frames that
    straddle them are named and checked first, so a 32-bit offset bug in launch_stream's
    sub-launch arithmetic (vf_stream.h) shows up as a named frame, not a count."""
    import concurrent.futures as cf
    n_frames = 4096
    total = n_frames * FB_1080
    in_sha, out_sha = _digests_1080p(golden_dir)
    base = [oracle.synthetic_frame(s, 1080, 1920).reshape(-1) for s in range(4)]
    for s in range(4):
        assert hashlib.sha256(base[s]).hexdigest() == in_sha[s]
    straddle = {k: (1 << k) // FB_1080 for k in (32, 33, 34)}
    for k, f in straddle.items():
        assert f * FB_1080 < (1 << k) < (f + 1) * FB_1080
    piece = 160  # frames per host piece (995 MB); a multiple of 4 keeps the seed pattern
    chunk = np.concatenate([base[f % 4] for f in range(piece)])
    ds, d1, d2 = (vf_ctx.alloc_device(total) for _ in range(3))
    pool = cf.ThreadPoolExecutor(16)  # hashlib releases the GIL on large buffers
    try:
        for f0 in range(0, n_frames, piece):
            nf = min(piece, n_frames - f0)
            vf_ctx.upload(ds + f0 * FB_1080, chunk, nf * FB_1080)
        vf_ctx.sync()
        vf_ctx.invert_device(ds, d1, total)  # one call: 25.48 GB, ~100 sub-launches
        vf_ctx.invert_device(d1, d2, total)
        vf_ctx.sync()
        y = np.empty(FB_1080, np.uint8)
        for k, f in straddle.items():
            vf_ctx.download(y, d1 + f * FB_1080, FB_1080)
            vf_ctx.sync()
            assert hashlib.sha256(y).hexdigest() == out_sha[f % 4], f"frame {f} straddling 2^{k}"
            vf_ctx.download(y, d2 + f * FB_1080, FB_1080)
            vf_ctx.sync()
            assert hashlib.sha256(y).hexdigest() == in_sha[f % 4], f"frame {f} straddling 2^{k} (~~x)"
        host = np.empty(piece * FB_1080, np.uint8)
        for dev, want in ((d1, out_sha), (d2, in_sha)):
            bad = []
            for f0 in range(0, n_frames, piece):
                nf = min(piece, n_frames - f0)
                vf_ctx.download(host, dev + f0 * FB_1080, nf * FB_1080)
                vf_ctx.sync()
                views = [host[i * FB_1080:(i + 1) * FB_1080] for i in range(nf)]
                got = list(pool.map(lambda v: hashlib.sha256(v).hexdigest(), views))
                bad += [f0 + i for i in range(nf) if got[i] != want[(f0 + i) % 4]]
            assert not bad, f"{len(bad)} frames differ, first {bad[:8]}"
    finally:
        pool.shutdown()
        for p in (ds, d1, d2):
            vf_ctx.free_device(p)


def test_timeline_chunks_cover_the_call(vf_ctx):
    """vf_last_timeline: one record per chunk, bytes sum to the call, H2D <= kernel <= D2H."""
    x = np.random.default_rng(1).integers(0, 256, 3 * (16 << 20) + 123, dtype=np.uint8)
    y = np.empty_like(x)
    vf_ctx.invert_host(x, y, x.nbytes)
    tl = vf_ctx.last_timeline()
    assert len(tl) >= 3 and sum(t[0] for t in tl) == x.nbytes
    for nb, h0, k0, k1, d1 in tl:
        assert 0.0 <= h0 <= k0 <= k1 <= d1
    assert np.array_equal(y, oracle.invert(x))


def test_async_frames_on_pinned_memory(vf_ctx):
    """vf_invert_frames_async: several batches queued back to back on page-locked memory,
    completed out of host order (wait on the last first), every byte exact; pageable
    buffers are refused, and a synchronous call after async ones sees consistent slots."""
    sizes = [1080 * 1920 * 3, 480 * 640 * 3, 17 * 13 * 3, 2160 * 3840 * 3]
    total = sum(sizes)
    nb = 6
    ps = [vf_ctx.alloc_host(total) for _ in range(nb)]
    pd = [vf_ctx.alloc_host(total) for _ in range(nb)]
    try:
        hs = [np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(p)) for p in ps]
        hd = [np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(p)) for p in pd]
        for b in range(nb):
            hs[b][:] = np.random.default_rng(b).integers(0, 256, total, dtype=np.uint8)
        tickets = []
        for b in range(nb):
            offs = np.cumsum([0] + sizes[:-1])
            srcs = [ps[b] + int(o) for o in offs]
            dsts = [pd[b] + int(o) for o in offs]
            tickets.append(vf_ctx.invert_frames_async(srcs, dsts, sizes))
        assert tickets == sorted(tickets) and len(set(tickets)) == nb
        assert vf_ctx.wait(tickets[-1]) >= 0.0
        for t in tickets:
            assert vf_ctx.query(t)
            vf_ctx.wait(t)
        for b in range(nb):
            assert np.array_equal(hd[b], oracle.invert(hs[b])), b
        # pageable buffers go through the engine's staging copies, queued behind pinned jobs
        xs = [oracle.synthetic_frame(60 + i, 480, 640) for i in range(3)]
        ys = [np.empty_like(x) for x in xs]
        t_pin = vf_ctx.invert_frames_async([ps[0]], [pd[0]], [sizes[0]])
        t_pg = vf_ctx.invert_frames_async(xs, ys, [x.nbytes for x in xs])
        vf_ctx.wait(t_pg)  # the pinned job runs zero-copy beside the ring: any completion order
        vf_ctx.wait(t_pin)
        assert np.array_equal(hd[0], oracle.invert(hs[0]))
        for x, y_ in zip(xs, ys):
            assert np.array_equal(y_, oracle.invert(x))
        with pytest.raises(vfilter.VFilterError, match="unknown ticket"):
            vf_ctx.wait(10 ** 9)
        y = oracle.synthetic_frame(77, 480, 640)  # sync path after async work
        assert np.array_equal(vfilter.bitwise_not(y, ctx=vf_ctx), oracle.invert(y))
    finally:
        for p in ps + pd:
            vf_ctx.free_host(p)


def test_sync_zero_copy_while_async_in_flight(vf_ctx):
    """A synchronous zero-copy call (Engine::run_now, on the caller's thread) while async jobs
    are in flight on the engine thread: both take and give events from the same free list
    (vfilter.h allows async submits followed by a sync call on one thread).
    200 rounds of three async jobs + one sync call; every byte exact."""
    n = 1 << 20
    ps = [vf_ctx.alloc_host(n) for _ in range(5)]
    pd = [vf_ctx.alloc_host(n) for _ in range(5)]
    try:
        hs = [np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p)) for p in ps]
        hd = [np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p)) for p in pd]
        for i, h in enumerate(hs):
            h[:] = np.random.default_rng(100 + i).integers(0, 256, n, dtype=np.uint8)
        for r in range(200):
            ts = [vf_ctx.invert_frames_async([ps[k]], [pd[k]], [n]) for k in range(3)]
            hd[4][:16] = 0
            vf_ctx.invert_host(ps[4], pd[4], n)
            assert _zero_copy(vf_ctx.last_timeline())
            assert np.array_equal(hd[4], ~hs[4]), r
            for t in ts:
                vf_ctx.wait(t)
        for k in (0, 1, 2, 4):
            assert np.array_equal(hd[k], ~hs[k]), k
    finally:
        for p in ps + pd:
            vf_ctx.free_host(p)


@pytest.mark.parametrize("n", [1, 17, 300_001, FB_1080, 3 * FB_1080 + 5])
def test_staged_small_jobs_every_side(vf_ctx, n):
    """Synchronous jobs up to 32 MiB with an unmapped side run on the caller's thread
    (Engine::run_staged): pageable source -> pinned arena destination (the drop-in's
    bitwise_not(frame)), pinned source -> pageable destination, pageable -> pageable, and in
    place; every byte exact, nothing outside the destination touched, one launch record."""
    rng = np.random.default_rng(n)
    x = rng.integers(0, 256, n + 32, dtype=np.uint8)
    want = ~x[7:7 + n]
    d = vf_ctx.pinned_empty((n + 32,))
    d[:] = 0x5A
    vf_ctx.invert_host(x[7:7 + n], d[3:3 + n], n)          # pageable -> mapped
    assert _zero_copy(vf_ctx.last_timeline())
    assert np.array_equal(d[3:3 + n], want) and (d[:3] == 0x5A).all() and (d[3 + n:] == 0x5A).all()
    p = vf_ctx.pinned_empty((n,))
    p[:] = x[7:7 + n]
    y = np.full(n + 32, 0x5A, np.uint8)
    vf_ctx.invert_host(p, y[5:5 + n], n)                    # mapped -> pageable
    assert _zero_copy(vf_ctx.last_timeline())
    assert np.array_equal(y[5:5 + n], want) and (y[:5] == 0x5A).all() and (y[5 + n:] == 0x5A).all()
    z = np.full(n + 32, 0x5A, np.uint8)
    vf_ctx.invert_host(x[7:7 + n], z[1:1 + n], n)          # pageable -> pageable
    assert np.array_equal(z[1:1 + n], want) and z[0] == 0x5A and (z[1 + n:] == 0x5A).all()
    w = x.copy()
    vf_ctx.invert_host(w, w, w.nbytes)                      # in place, pageable
    assert np.array_equal(w, ~x)
    r = vfilter.bitwise_not(x[7:7 + n], ctx=vf_ctx)         # the drop-in: result in the arena
    assert np.array_equal(r, want)


@pytest.mark.parametrize("threads", ["0", "1"])
def test_staged_jobs_without_copy_threads(monkeypatch, threads):
    """VF_HOST_THREADS=0 (or 1) leaves the staging copy pool with no or one worker thread: the
    staged job's copy-in must still land before its launch (with 0 threads the
    launch read uninitialised staging memory and returned success)."""
    monkeypatch.setenv("VF_HOST_THREADS", threads)
    with vfilter.Context(0, max_frame_bytes=FB_1080, max_batch=4) as ctx:
        for n in (17, FB_1080, 3 * FB_1080 + 5):
            x = np.random.default_rng(n + 1).integers(0, 256, n + 16, dtype=np.uint8)
            want = ~x[3:3 + n]
            d = ctx.pinned_empty((n,))
            d[:] = 0
            ctx.invert_host(x[3:3 + n], d, n)                   # pageable -> mapped (staged in)
            assert _zero_copy(ctx.last_timeline())
            assert np.array_equal(d, want), n
            z = np.zeros(n, np.uint8)
            ctx.invert_host(x[3:3 + n], z, n)                   # pageable -> pageable (both staged)
            assert np.array_equal(z, want), n
            assert np.array_equal(vfilter.bitwise_not(x[3:3 + n], ctx=ctx), want)


@pytest.mark.parametrize("budget", [None, "0"])
def test_gated_dropin_frames(vf_ctx, monkeypatch, capfd, budget):
    """The drop-in's pageable frame with an aligned destination takes the gated launch
    (Engine::run_gated; by default above 8 MiB, here at every size): the kernel is queued
    before the staging copy and each tile waits for its piece (32 KiB and up).  Ragged sizes
    around the piece and tile edges up to a 4K frame and the 32-MiB staging cap, into the pinned
    arena and into a pageable array, and in place; with a give-up budget of 0 the waves leave at
    their first missing piece and the frame is inverted again, ungated -- bit-exact either way,
    nothing outside the destination touched."""
    monkeypatch.setenv("VF_STAGE_TRACE", "1")
    monkeypatch.setenv("VF_STAGE_GATE_MIN", "0")  # every size (the default gates frames above 8 MiB)
    if budget is not None:
        monkeypatch.setenv("VF_STAGE_GATE_BUDGET_US", budget)
    sizes = [1, 15, 16, 4097, 262143, 262144, 262145, FB_1080, 2160 * 3840 * 3 + 3, 32 << 20]
    rng = np.random.default_rng(7)
    x = rng.integers(0, 256, (32 << 20) + 64, dtype=np.uint8)
    for n in sizes:
        src = x[5:5 + n]
        want = ~src
        r = vfilter.bitwise_not(src, ctx=vf_ctx)                 # pageable -> pinned arena
        assert np.array_equal(r, want), n
        d = np.full(n + 32, 0x5A, np.uint8)
        dv = d[16:16 + n]
        if dv.ctypes.data % 16:
            dv = d[16 - dv.ctypes.data % 16:][:n]
        off = dv.ctypes.data - d.ctypes.data
        vf_ctx.invert_host(src, dv, n)                            # pageable -> pageable
        assert np.array_equal(dv, want), n
        assert (d[:off] == 0x5A).all() and (d[off + n:] == 0x5A).all(), n
    w = x[:FB_1080 + 16].copy()
    vf_ctx.invert_host(w, w, w.nbytes)                            # in place
    assert np.array_equal(w, ~x[:FB_1080 + 16])
    err = capfd.readouterr().err
    assert err.count("vf_stage: gated") >= 2 * len(sizes), err[-2000:]
    if budget == "0":
        assert "re-run ungated" in err


def _zero_copy(tl):
    """A zero-copy call reports one record whose H2D start = kernel start = 0 and kernel end =
    D2H end (one launch read the source and wrote the destination over PCIe)."""
    return len(tl) == 1 and tl[0][1] == 0.0 and tl[0][2] == 0.0 and tl[0][3] == tl[0][4]


def test_zero_copy_ranges_every_offset_and_split(vf_ctx):
    """Page-locked ranges from vf_alloc_host are inverted in place over PCIe (one launch per 64
    ranges, descriptors in the kernel arguments): every relative src/dst offset mod 16 with
    ragged lengths, 0-length ranges, 150 ranges (3 launches), and interior pointers of a
    registered numpy buffer -- bit-exact, and the timeline says the zero-copy path ran."""
    cap = 8 << 20
    ps, pd = vf_ctx.alloc_host(cap), vf_ctx.alloc_host(cap)
    try:
        hs = np.ctypeslib.as_array((ctypes.c_uint8 * cap).from_address(ps))
        hd = np.ctypeslib.as_array((ctypes.c_uint8 * cap).from_address(pd))
        hs[:] = np.random.default_rng(11).integers(0, 256, cap, dtype=np.uint8)
        rng = np.random.default_rng(12)
        # one range per (src offset, dst offset) pair, each in its own 32 KiB cell
        srcs, dsts, sizes = [], [], []
        for so in range(16):
            for do in range(16):
                cell = (so * 16 + do) * 32768
                srcs.append(ps + cell + so)
                dsts.append(pd + cell + do)
                sizes.append(int(rng.integers(1, 32768 - 16)))
        for lo in range(0, len(srcs), 150):  # 150 ranges per call: launches of 64, 64, 22
            hd[:] = 0
            sel = slice(lo, lo + 150)
            vf_ctx.invert_frames_host(srcs[sel], dsts[sel], sizes[sel])
            assert _zero_copy(vf_ctx.last_timeline())
            for s_, d_, n in zip(srcs[sel], dsts[sel], sizes[sel]):
                so, do = s_ - ps, d_ - pd
                assert np.array_equal(hd[do:do + n], ~hs[so:so + n]), (so % 16, do % 16, n)
                assert hd[do + n] == 0  # nothing past the range
        # 0-length ranges mixed in, and one large range (1080p x 1, 7 MiB)
        hd[:] = 0
        vf_ctx.invert_frames_host([ps, ps + 100, ps + 4096], [pd, pd + 100, pd + 4096],
                                  [0, 3, FB_1080])
        assert np.array_equal(hd[100:103], ~hs[100:103]) and hd[99] == 0 and hd[103] == 0
        assert np.array_equal(hd[4096:4096 + FB_1080], ~hs[4096:4096 + FB_1080])
        # very different sizes in one launch (a 480p / 1080p / 4K-like mix): the tiles are
        # numbered across the ranges, so each range is covered whatever its share
        hd[:] = 0
        offs = [(7, 3, 17), (100, 5000, 921600 + 5), (2 << 20, (2 << 20) + 9, 3 << 20), (64, (6 << 20) + 64, 31)]
        vf_ctx.invert_frames_host([ps + a for a, _, _ in offs], [pd + b for _, b, _ in offs], [n for _, _, n in offs])
        assert _zero_copy(vf_ctx.last_timeline())
        for a, b, n in offs:
            assert np.array_equal(hd[b:b + n], ~hs[a:a + n]), (a, b, n)
        # async, several jobs in flight on the zero-copy stream
        ts = [vf_ctx.invert_frames_async([ps + k * (1 << 20)], [pd + k * (1 << 20)], [1 << 20])
              for k in range(8)]
        for t in ts:
            vf_ctx.wait(t)
        assert np.array_equal(hd, ~hs)
    finally:
        vf_ctx.free_host(ps)
        vf_ctx.free_host(pd)
    # interior pointers of a registered numpy buffer (a shared-memory frame ring's case)
    buf = np.random.default_rng(13).integers(0, 256, 3 << 20, dtype=np.uint8)
    out = np.zeros_like(buf)
    a, b = vf_ctx.host_register(buf), vf_ctx.host_register(out)
    try:
        vf_ctx.invert_frames_host([buf[5:], buf[1 << 20:]], [out[9:], out[(1 << 20) + 3:]],
                                  [(1 << 20) - 100, (2 << 20) - 7])
        assert _zero_copy(vf_ctx.last_timeline())
        assert np.array_equal(out[9:9 + (1 << 20) - 100], ~buf[5:5 + (1 << 20) - 100])
        n2 = (2 << 20) - 7
        assert np.array_equal(out[(1 << 20) + 3:(1 << 20) + 3 + n2], ~buf[1 << 20:(1 << 20) + n2])
    finally:
        vf_ctx.host_unregister(a)
        vf_ctx.host_unregister(b)


def test_zero_copy_falls_back_and_can_be_disabled(vf_ctx, monkeypatch):
    """A job with any byte outside the noted page-locked ranges takes the slot ring (staged),
    and VF_ZEROCOPY=0 at context creation sends page-locked jobs to the ring's direct DMA:
    both bit-exact, with the ring's per-chunk timeline."""
    n = 3 * (16 << 20) + 77
    p = vf_ctx.alloc_host(n)
    try:
        h = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p))
        h[:] = np.random.default_rng(14).integers(0, 256, n, dtype=np.uint8)
        y = np.empty(n, np.uint8)  # pageable destination
        vf_ctx.invert_host(p, y, n)
        assert not _zero_copy(vf_ctx.last_timeline())
        assert np.array_equal(y, ~h)
    finally:
        vf_ctx.free_host(p)
    monkeypatch.setenv("VF_ZEROCOPY", "0")
    with vfilter.Context(0, max_frame_bytes=FB_1080, max_batch=4) as ctx:
        ps, pd = ctx.alloc_host(n), ctx.alloc_host(n)
        try:
            hs = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ps))
            hd = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(pd))
            hs[:] = np.random.default_rng(15).integers(0, 256, n, dtype=np.uint8)
            ctx.invert_host(ps, pd, n)
            tl = ctx.last_timeline()
            assert len(tl) >= 3 and sum(t[0] for t in tl) == n
            assert np.array_equal(hd, ~hs)
        finally:
            ctx.free_host(ps)
            ctx.free_host(pd)
