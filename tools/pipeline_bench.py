#!/usr/bin/env python3
"""Distributor-level throughput: BASELINE.json configs[2] (4K, batch 16, frame-index sharded
over N workers, in-order reassembly) and configs[3] (mixed 480p/1080p/4K stream, ordering
overhead), host->host through the whole fan-out.

One Distributor (lossless ``shard`` or ``pull`` policy, ``ordered`` reassembly, shared-memory
ring with one slice per worker on its GPU's NUMA node, zero-copy in and out) feeds N
``python -m vfilter.inverter`` worker processes, worker i on GPU i % G.  Each worker page-locks
its own slice, so frames go slice -> GPU -> slice by DMA.
Reported: delivered frames/s in index order, GB/s each way, per-frame latency (commit ->
in-order release), reorder wait and buffer depth.

  python tools/pipeline_bench.py --workers 2 --size 4k --batch 16 --frames 512
  python tools/pipeline_bench.py --workers 2 --size mixed --policy pull
  python tools/pipeline_bench.py --workers 1 --size 1080p --jpeg --batch 32   # the reference default mode

``--jpeg``: frames are JPEGs (the app's encode, webcam_app.py:110, here the product's GPU
encoder on camera-like scenes) and the workers run in the reference's default JPEG mode
(decode -> bitwise_not -> encode, inverter.py:32-44); results are JPEGs of their own sizes,
compared with the product's own invert of the same input — length always, every
``--verify-every``-th in full, the others on their first and last 4 KiB (the GPU codec's
parity with libjpeg-turbo is tests/test_gpu_jpeg.py's job).

Producer modes: ``copy`` (default) — each frame is copied into its slot from a pre-generated
frame (what a producer that cannot decode straight into the ring pays); ``resident`` — ring
slots are filled once with random bytes and frames are committed without a host copy,
isolating distribution + PCIe + kernel + reassembly.  Every ``--verify-every``-th frame is
checked in full against its input; the others on their first and last 4 KiB.
"""
import argparse
import json
import os
import signal
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-video-filter_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

from vfilter.distributor import Distributor  # noqa: E402
from vfilter.shm import copy_into, shm_free_bytes  # noqa: E402
from vfilter.synthetic import SIZES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=0, help="devices to spread workers over (0 = all visible)")
    ap.add_argument("--size", default="1080p", choices=list(SIZES) + ["mixed"])
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--policy", default="shard", choices=("shard", "pull"))
    ap.add_argument("--producer", default="copy", choices=("resident", "copy"))
    ap.add_argument("--ring-slots", type=int, default=0,
                    help="slots per worker slice (0 = batches in flight + 1 (raw) or + 2 (JPEG), capped by /dev/shm)")
    ap.add_argument("--verify-every", type=int, default=8)
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in progress per worker (0: the worker's default, 2 raw / 3 JPEG)")
    ap.add_argument("--jpeg", action="store_true", help="JPEG frames, workers in JPEG mode")
    ap.add_argument("--profile", default="",
                    help="sample the distributor's threads and each worker's (tools/sampler.py); "
                         "reports go to PROFILE.distributor and PROFILE.<worker pid>")
    ap.add_argument("--producers", type=int, default=0,
                    help="producer threads (0: one per worker, at most 8); each reserves, fills and "
                         "commits its own frames, so copies into the slices run in parallel")
    ap.add_argument("--content", default="scene", choices=("scene", "hard"),
                    help="--jpeg frames: camera-like scenes at q85 (8 distinct per shape), or 'hard': noisy "
                         "scenes at q95 (32 distinct per shape, vfilter.synthetic.synthetic_noisy_scene)")
    ap.add_argument("--numa-local", type=int, default=1,
                    help="1: frame copies and full checks run on threads pinned to the NUMA node of the "
                         "slot's ring slice (per-node pools; each node gets its own copy of the source "
                         "frames); 0: on the producer / one verification pool")
    ap.add_argument("--consume", type=int, default=64, help="results taken per get_next_batch call")
    ap.add_argument("--worker-batch", type=int, default=None,
                    help="the workers' --batch (default: --batch; 0: the worker's own choice, "
                         "vfilter.inverter.auto_credit); --batch still sizes the ring slices")
    ap.add_argument("--verify-pool", type=int, default=-1,
                    help="JPEG results verified and released on the verification pool (1) or inline (0); "
                         "-1: the pool from 2 workers on")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    shapes = [SIZES["480p"], SIZES["1080p"], SIZES["4k"]] if args.size == "mixed" else [SIZES[args.size]]
    fbytes = [h * w * 3 for h, w in shapes]
    jpgs = want = None
    if args.jpeg:  # 8 distinct JPEGs per shape and their inverted JPEGs, from the product
        from vfilter import Context
        from vfilter.jpeg import TurboJPEG
        from vfilter.synthetic import synthetic_noisy_scene, synthetic_scene
        hard = args.content == "hard"
        gen, nd, q = (synthetic_noisy_scene, 32, 95) if hard else (synthetic_scene, 8, 85)
        with Context(int(os.environ.get("VF_DEVICE", "0"))) as cctx:
            tj = TurboJPEG(ctx=cctx)
            jpgs = [bytes(j) for h, w in shapes for j in tj.encode_batch([gen(s, h, w) for s in range(nd)], quality=q)]
            want = [bytes(o) for o in tj.invert_batch(jpgs)]
        want_np = [np.frombuffer(w_, np.uint8) for w_ in want]
        fbytes = [len(j) for j in jpgs]
        shapes = [None] * len(jpgs)
    slot_bytes = max(fbytes) * 2 if args.jpeg else max(fbytes)  # room for a result larger than its input
    inflight = args.inflight or (3 if args.jpeg else 2)  # the worker's own default when not given
    # every batch in flight holds its slots until its results are consumed: room for those
    # plus one (raw) or two (JPEG, small frames, fast batches) batches being filled
    slots = args.ring_slots or (inflight + (2 if args.jpeg else 1)) * args.batch
    free = shm_free_bytes()
    if free is not None:
        slots = max(2 * args.batch, min(slots, int(free * 0.6) // (2 * slot_bytes * args.workers)))
    ngpu = args.gpus
    if ngpu <= 0:
        from vfilter import device_count
        ngpu = max(1, device_count())

    d = Distributor(0, 0, policy=args.policy, reassembly="ordered", transport="tcp", host="127.0.0.1",
                    queue_size=3 * args.batch * args.workers, ring_slots=slots, ring_slot_bytes=slot_bytes,
                    shard_workers=args.workers, shard_chunk=args.batch, zero_copy=True, verbose=False)
    d.start()
    env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + os.environ.get("PYTHONPATH", ""))
    procs = []
    for i in range(args.workers):
        e = dict(env, VF_DEVICE=str(i % ngpu))
        if args.profile:
            e["VF_SAMPLER_OUT"] = args.profile
        launcher = ([os.path.join(ROOT, "tools", "profiled_inverter.py")] if args.profile else
                    ["-m", "vfilter.inverter"])
        cmd = [sys.executable] + launcher + ["--host", "127.0.0.1",
               "--distribute-port", str(d.distribute_port), "--collect-port",
               str(d.collect_port), "--batch", str(args.batch if args.worker_batch is None else args.worker_batch),
               "--transport", "tcp"]
        if not args.jpeg:
            cmd.append("--raw")
        if args.inflight:
            cmd += ["--inflight", str(args.inflight)]
        procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
    result = {}
    try:
        t0 = time.time()
        while d.num_workers() < args.workers:
            if time.time() - t0 > 120 or any(p.poll() is not None for p in procs):
                raise RuntimeError("workers did not come up: " +
                                   " | ".join((p.stderr.read() or b"").decode()[-300:] for p in procs if p.poll() is not None))
            time.sleep(0.05)

        # NUMA-local host work: one pool of threads pinned to each slice's node; a frame's copy
        # into its slot and its full check run on the pool of the slot's node, from that node's
        # own copy of the source frames, so neither crosses the socket link
        from concurrent.futures import ThreadPoolExecutor
        from vfilter import numa as vnuma
        wk = d.ordering_stats()["workers"]
        sid_node = {}
        for w_ in wk.values():
            sl = w_.get("slice")
            if sl and w_.get("slice_id") is not None:
                sid_node[w_["slice_id"]] = sl["numa"]
        nodes = sorted({n_ for n_ in sid_node.values() if n_ is not None}) if args.numa_local else []
        per_node = max(2, min(8, (len(os.sched_getaffinity(0)) // max(1, len(nodes))))) if nodes else 0
        node_pool = {n_: ThreadPoolExecutor(max_workers=per_node, thread_name_prefix=f"node{n_}",
                                            initializer=vnuma.pin_thread_to_node, initargs=(n_,)) for n_ in nodes}
        pinned_ok = {n_: bool(node_pool[n_].submit(vnuma.pin_thread_to_node, n_).result()) for n_ in nodes}

        def slot_node(slot):
            return sid_node.get(slot // d.ring_slots) if nodes else None

        rng = np.random.default_rng(0)
        # resident content: each slot's input half holds random bytes once
        if args.producer == "resident":
            for s in range(d.total_slots()):
                d.in_view(s, slot_bytes)[:] = rng.integers(0, 256, slot_bytes, dtype=np.uint8)
        pregen = ([np.frombuffer(j, np.uint8) for j in jpgs] if args.jpeg else
                  [rng.integers(0, 256, fb, dtype=np.uint8) for fb in fbytes])
        # each node's own copy of the sources, first touched by a thread of that node
        pregen_on = {n_: node_pool[n_].submit(lambda: [p_.copy() for p_ in pregen]).result() for n_ in nodes}
        # warmup: every worker maps and page-locks its slice on its first batch (hipHostRegister,
        # ~0.15 s per GB) -- a one-off start-up cost kept out of the timing
        warm = 2 * args.batch * args.workers * len(shapes)
        n = args.frames
        commit_t = np.zeros(warm + n)
        release_t = np.zeros(warm + n)
        errors = []
        started = threading.Event()

        sampler = None
        if args.profile:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            from sampler import Sampler
            sampler = Sampler().start()
        nprod = args.producers or min(8, args.workers)
        # the frame a reservation gets decides what goes in it: index i carries content i % len(shapes)
        # (the distributor fixes the index at reservation, in call order across producers)
        count_lock = threading.Lock()
        counter = [0]

        group = max(1, min(16, args.batch // 2))  # reservations and commits per lock hold
        # frames below this are copied on the producer thread itself: a pool hand-off (submit, wake,
        # join: ~50-60 us) per 182 KB JPEG capped the system at 16-20 k fps;
        # a 1080p / 4K raw frame's copy (0.3-2 ms) still goes to its slice's node pool
        INLINE_COPY = 1 << 20

        # JPEG frames through the native engine: the producer works in columns -- one reservation,
        # one vfd_fill (every frame's copy into its slot) and one commit per group -- where a
        # Python step per frame (index lookup, view, copy call) held the leg at 100-160 k fps on
        # one producer thread (r06_small_legs_profile.txt)
        # (frames of 1 MiB and more -- hard q95 1080p JPEGs are 2 MB -- keep the node pools' parallel copies)
        columnar = (args.jpeg and args.producer == "copy" and getattr(d, "engine", "python") == "native"
                    and max(fbytes) < INLINE_COPY)
        if columnar:
            group = max(1, args.batch)
            src_addr = np.array([p_.ctypes.data for p_ in pregen], np.uint64)
            src_nb = np.array([p_.nbytes for p_ in pregen], np.int64)

        def produce_columns(i0, g):
            done_ = 0
            while done_ < g:
                slots, idxs = d.reserve_frames_array(max_nb, g - done_)
                if not len(slots):
                    return
                nb = src_nb[idxs % len(shapes)]
                d.fill_frames(slots, src_addr[idxs % len(shapes)], nb)
                commit_t[idxs] = time.perf_counter()
                d.commit_frames(slots, nb)
                done_ += len(slots)

        def produce():
            while True:
                with count_lock:
                    i0 = counter[0]
                    if i0 >= warm + n:
                        return
                    g = min(group, warm + n - i0, warm - i0 if i0 < warm else group)
                    counter[0] += g
                if i0 >= warm:
                    started.wait()
                if columnar:
                    produce_columns(i0, g)
                    continue
                done_ = 0
                while done_ < g:
                    slots = d.reserve_frames(max_nb, g - done_)
                    nbs, shs, idxs, futs = [], [], [], []
                    for j, slot in enumerate(slots):
                        idx = d.reserved_index(slot)
                        idx = i0 + done_ + j if idx is None else idx
                        idxs.append(idx)
                        k = idx % len(shapes)
                        nb = fbytes[k]
                        if args.producer == "copy":
                            nd_ = slot_node(slot)
                            if nb < INLINE_COPY:  # a JPEG / 480p frame: a hand-off costs more than the copy
                                copy_into(d.frame_view(slot, nb), (pregen_on[nd_] if nd_ in node_pool else pregen)[k],
                                          threads=1)
                            elif nd_ in node_pool:  # on the slice's own node, frames of a group in parallel
                                futs.append(node_pool[nd_].submit(copy_into, d.frame_view(slot, nb), pregen_on[nd_][k],
                                                                  1))
                            else:
                                copy_into(d.frame_view(slot, nb), pregen[k], threads=1 if nprod > 1 else 4)
                        nbs.append(nb)
                        shs.append(None if args.jpeg else [shapes[k][0], shapes[k][1], 3])
                    for f_ in futs:
                        f_.result()
                    commit_t[idxs] = time.perf_counter()
                    d.commit_frames(slots, nbs, shs)
                    done_ += len(slots)

        max_nb = max(fbytes)
        ths = [threading.Thread(target=produce, daemon=True) for _ in range(nprod)]
        for th in ths:
            th.start()
        # full checks (np.bitwise_not of a whole 4K frame: ~5 ms of one core) run on a pool
        # beside the consumer, which releases a slot once its check is done
        from concurrent.futures import ThreadPoolExecutor
        vpool = ThreadPoolExecutor(max_workers=max(4, min(16, 2 * args.workers)), thread_name_prefix="verify")
        pending = []

        def full_check(i, idx, view, src):
            if not np.array_equal(view, np.bitwise_not(src)):
                errors.append(f"frame {i} differs")
            d.release_frame(idx)

        total_bytes = 0
        # results are taken a batch at a time (get_next_batch) and checked with array operations
        # where the engine gives addresses (native): index order and lengths for every frame, the
        # first and last ENDS bytes of every JPEG gathered from the ring slices in one fancy index
        # per slice, whole frames every verify_every-th; a Python step per frame could not keep up
        # with eight GPUs' worth of JPEG frames (VERDICT r04 missing #1)
        ENDS = 1024
        native_eng = getattr(d, "engine", "python") == "native"
        if args.jpeg:
            want_len = np.asarray([w_.nbytes for w_ in want_np], np.int64)
            want_head = np.stack([w_[:ENDS] for w_ in want_np])
            want_tail = np.stack([w_[-ENDS:] for w_ in want_np])
            span = np.arange(ENDS)

        def check_ends(b, kk, idxs):
            """Head and tail of every JPEG result in batch ``b`` (rows kk) against the expected."""
            if native_eng:
                rec = b.rec[kk]
                sid = rec["slot"] // d.ring_slots
                for s_ in np.unique(sid).tolist():
                    m_ = sid == s_
                    arr = d._slice_arr(int(s_))
                    off = rec["data"][m_].astype(np.int64) - arr.ctypes.data
                    nb_ = rec["nbytes"][m_]
                    wk = idxs[m_] % len(want_np)
                    h_ok = (arr[off[:, None] + span] == want_head[wk]).all(axis=1)
                    t_ok = (arr[(off + nb_ - ENDS)[:, None] + span] == want_tail[wk]).all(axis=1)
                    for j in np.flatnonzero(~(h_ok & t_ok)).tolist():
                        errors.append(f"frame {int(idxs[m_][j])} differs")
                return
            for r_, i_ in zip(kk.tolist(), idxs.tolist()):
                v_ = b.view(r_)
                w_ = want[i_ % len(want_np)]
                if not (v_[:ENDS].tobytes() == w_[:ENDS] and v_[-ENDS:].tobytes() == w_[-ENDS:]):
                    errors.append(f"frame {i_} differs")

        pool_verify = args.verify_pool == 1 or (args.verify_pool < 0 and args.workers > 1)

        def verify_jpeg(b, idxs):
            """Lengths of every JPEG result in batch ``b``, whole frames every verify_every-th, head and
            tail of the rest; then the batch's slots go back."""
            try:
                bad = np.flatnonzero(b.nbytes != want_len[idxs % len(want_np)])
                for j in bad.tolist():
                    errors.append(f"frame {int(idxs[j])}: {int(b.nbytes[j])} B, expected {int(want_len[idxs[j] % len(want_np)])}")
                full = np.flatnonzero(idxs % args.verify_every == 0)
                for j in full.tolist():
                    if not np.array_equal(b.view(j), want_np[int(idxs[j]) % len(want_np)]):
                        errors.append(f"frame {int(idxs[j])} differs")
                rest = np.flatnonzero(idxs % args.verify_every != 0)
                if len(rest):
                    check_ends(b, rest, idxs[rest])
            finally:
                d.release_frames(idxs)

        i = 0
        t_start = None
        while i < warm + n:
            if t_start is None and i >= warm:
                if sampler is not None:
                    sampler.clear()
                d_stats0 = d.ordering_stats()
                t_start = time.perf_counter()
                i_start = i
                started.set()
            b = d.get_next_batch(args.consume, timeout=120)
            k = len(b)
            if not k:
                raise RuntimeError(f"frame {i} never arrived: {d.ordering_stats()}")
            idxs = b.index
            if idxs[0] != i or idxs[-1] != i + k - 1:
                errors.append(f"order: got {idxs[:4].tolist()}... expected from {i}")
            release_t[i:i + k] = time.perf_counter()
            if args.jpeg:
                if i >= warm:
                    total_bytes += int(np.asarray(fbytes)[idxs % len(fbytes)].sum())
                # verified and released on the verification pool, a batch per task, so the
                # checks of several GPUs' worth of results do not serialise on this thread (with
                # one worker the hand-off costs more than it saves: inline)
                if not pool_verify:
                    verify_jpeg(b, idxs)
                    i += k
                    continue
                pending.append(vpool.submit(verify_jpeg, b, idxs))
                if len(pending) >= 64:
                    for f_ in pending[:32]:
                        f_.result()
                    del pending[:32]
                i += k
                continue
            rel = []
            for j in range(k):
                ii = int(idxs[j])
                view, info = b.view(j), b.info(j)
                if ii >= warm:
                    total_bytes += view.nbytes
                src = d.in_view(info["slot"], view.nbytes)
                if ii % args.verify_every == 0:
                    nd_ = slot_node(info["slot"])
                    pending.append((node_pool.get(nd_) or vpool).submit(full_check, ii, ii, view, src))
                else:
                    if not (np.array_equal(view[:4096], np.bitwise_not(src[:4096])) and
                            np.array_equal(view[-4096:], np.bitwise_not(src[-4096:]))):
                        errors.append(f"frame {ii} differs")
                    rel.append(ii)
            d.release_frames(rel)
            i += k
        n_t = i - i_start  # frames timed
        t_end = time.perf_counter()
        if sampler is not None:
            sampler.stop()
            with open(args.profile + ".distributor", "w") as f:
                f.write(sampler.report(60) + "\n")
        for f in pending:
            f.result()
        vpool.shutdown()
        for th in ths:
            th.join()
        for p_ in node_pool.values():
            p_.shutdown()
        el = t_end - t_start
        lat = (release_t[warm:] - commit_t[warm:]) * 1e3
        st = d.ordering_stats()
        st["max_depth"] = max(st["max_depth"], d_stats0["max_depth"])
        slices = [w["slice"] for w in st["workers"].values() if w["slice"]]
        result = {"kind": "pipeline_jpeg" if args.jpeg else "pipeline", "size": args.size, "producers": nprod, "consume": args.consume, "worker_batch": args.worker_batch, "verify_pool": bool(args.jpeg and pool_verify),
                  "workers": args.workers, "gpus": min(ngpu, args.workers),
                  "inflight_per_worker": inflight,
                  "policy": args.policy, "producer": args.producer, "producer_form": "columns" if columnar else "per frame",
                  "batch": args.batch, "frames": n_t,
                  "ring_slots_per_worker": slots, "verify_full_every": args.verify_every,
                  "slice_bytes_per_worker": slices[0]["bytes"] if slices else None,
                  "slice_numa": [sl["numa"] for sl in slices], "slice_numa_bound": [sl["numa_bound"] for sl in slices],
                  "host_work_placement": ({"per_node_threads": per_node, "nodes": nodes,
                                           "pinned": {str(k_): v_ for k_, v_ in pinned_ok.items()},
                                           "node_cpus": {str(n_): len(vnuma.node_cpus(n_)) for n_ in nodes}}
                                          if nodes else "unpinned (one pool)"),
                  "content": args.content if args.jpeg else "random",
                  "evictions": st["evictions"], "frames_lost": st["frames_lost"], "fps": round(n_t / el, 1), "GBps_each_way": round(total_bytes / el / 1e9, 2),
                  "latency_ms_mean": round(float(lat.mean()), 3), "latency_ms_p99": round(float(np.percentile(lat, 99)), 3),
                  "reorder_wait_mean_ms": round(st["reorder_wait_mean_ms"], 3),
                  "reorder_wait_max_ms": round(st["reorder_wait_max_ms"], 3), "max_buffer_depth": st["max_depth"],
                  "out_of_order_arrivals": st["out_of_order"], "errors": errors[:5], "n_errors": len(errors)}
        if args.jpeg:
            result["jpeg_bytes_in_mean"] = round(float(np.mean(fbytes)))
            result["GBps_note"] = "compressed bytes in"
        print(json.dumps(result), flush=True)
        if args.out:
            with open(args.out, "a") as f:
                f.write(json.dumps(result) + "\n")
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(15)
            except subprocess.TimeoutExpired:
                p.kill()
        d.cleanup()
    return 0 if result and not result["n_errors"] else 1


if __name__ == "__main__":
    sys.exit(main())
