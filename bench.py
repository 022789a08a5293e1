#!/usr/bin/env python3
"""Benchmark: 1080p RGB invert frames/s on 1..N MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], kernel-only): batches of 32 frames of 1920x1080x3 uint8,
resident in HBM.  One *step* = one launch of the invert kernel over one 32-frame batch
(199,065,600 B read + 199,065,600 B written).  Steps rotate over a ring of distinct
batches (default 2.4 GB in+out) so the 256 MiB Infinity Cache cannot serve them: the rate is
an HBM rate.  Each rank (one process per GPU) processes its own frame-index shard (global
batch b goes to rank b % N); there is no collective on the data path, so scaling is weak.

Launched as  python bench.py --gpus N --steps K --warmup W  (torch.distributed.run for N>1).
Prints ONE JSON line on rank 0 (contract in the task statement), including
  roofline      algorithmic bytes per launch / mean per-launch hipEvent duration, vs 8 TB/s;
                traffic = HBM bytes per launch from rocprofv3 PMC (FETCH_SIZE x 2 per the
                gfx950 correction in MI355X_MICROARCH.md §HBM, + WRITE_SIZE), rank 0 at N=1
  cpu_baseline  the oracle's numpy restatement of inverter.py:41 (np.bitwise_not per frame,
                a new array each call, like cv2.bitwise_not), 1 host core, ~10 s sample; plus
                multi_process: the same arithmetic in up to 16 processes at once (BASELINE.md plan),
                process_scaling_fps: 1, 2, 4, 8 and 16 processes; sizes: 1 core at 480p and 4K
  sizes         kernel-only frames/s and HBM fraction at 480p / 1080p / 4K on this run's GPUs
                (north star: every size at 1/2/4/8 GPUs), same timing rules as the headline
  configs4_sweep  BASELINE configs[4]: 1080p batches of 256 ... 4096 frames resident per rank
  end_to_end    host->host rate through vf_invert_batch_host (pageable and pinned): PCIe-bound,
                reported beside value, never as value.
  jpeg_mode     the reference's default use_jpeg=True path (decode -> invert -> encode) on 1080p
                JPEGs: GPU-resident and host->host frames/s (in a child process without torch, as
                a worker process runs it), per-stage roofline, libjpeg-turbo on 1 core beside it.
  distributor   configs[2] (4K, batch 16, frame-index shards, in-order reassembly) and configs[3]
                (mixed 480p/1080p/4K stream, ordering overhead) through the distributor with one
                worker process per GPU of this run, and the JPEG deployment (1080p scenes and hard
                content, the reference app's 512 x 512 frames, 480p) with each leg's worker-form
                rate and the distributor's own control-plane rate beside it: host->host frames/s,
                never the headline.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-video-filter_amd"))
sys.path.insert(0, ROOT)

H, W, C = 1080, 1920, 3
FRAME_BYTES = H * W * C
METRIC = "frames/sec (1080p RGB invert) at 1/2/4/8 GPUs; kernel HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=32, help="frames per step (configs[1]: 32)")
    ap.add_argument("--ring-gb", type=float, default=2.4, help="in+out bytes the steps rotate over")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline sample length (0 = skip)")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host->host end-to-end leg")
    ap.add_argument("--no-jpeg", action="store_true", help="skip the JPEG-mode leg (use_jpeg=True path)")
    ap.add_argument("--no-distributor", action="store_true",
                    help="skip the configs[2]/[3] distributor leg (worker process per GPU)")
    ap.add_argument("--no-sizes", action="store_true", help="skip the 480p / 1080p / 4K kernel leg")
    ap.add_argument("--no-sweep", action="store_true", help="skip the configs[4] 256..4096-frame resident sweep")
    ap.add_argument("--no-per-frame", action="store_true", help="skip the one-frame-per-call drop-in leg")
    ap.add_argument("--dist-reps", type=int, default=5,
                    help="repetitions of each JPEG distributor leg (median reported, min/max in the detail; "
                         "the small-frame legs swing 0.8-1.2x run to run, profiles/r06_small_legs_spread.txt)")
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="processes of the multi-process CPU baseline (capped by the CPU affinity; 0 = skip)")
    ap.add_argument("--probe", action="store_true", help=argparse.SUPPRESS)  # child under rocprofv3
    ap.add_argument("--cpu-worker", type=float, default=0.0, help=argparse.SUPPRESS)  # cpu_baseline_multi child
    ap.add_argument("--host-copy-child", type=float, default=0.0, help=argparse.SUPPRESS)  # host_copy_ceiling child
    ap.add_argument("--jpeg-child", type=int, default=-1, help=argparse.SUPPRESS)  # jpeg leg on device N
    return ap.parse_args()


# ---------------------------------------------------------------------------------------
# device ring
# ---------------------------------------------------------------------------------------

def make_ring(ctx, batch, ring_gb, np, rank=0, world=1, hw=(H, W), distinct=97):
    """Ring slot k of this rank holds the frames of global batch k*world + rank (its
    frame-index shard, vfilter.sharding); step s processes slot s % nbuf, i.e. the frames
    of global batch s*world + rank up to the ring's reuse of synthetic content."""
    from vfilter import sharding
    from vfilter.synthetic import synthetic_frame
    fb = hw[0] * hw[1] * C
    batch_bytes = batch * fb
    nbuf = max(2, int(ring_gb * 1e9 // (2 * batch_bytes)))
    cache = {}
    host = np.empty(batch_bytes, np.uint8)
    srcs, dsts = [], []
    for k in range(nbuf):
        for j, i in enumerate(sharding.batch_frames(sharding.batch_of_step(k, rank, world), batch)):
            seed = sharding.synthetic_seed(i, distinct)
            if seed not in cache:
                cache[seed] = synthetic_frame(seed, hw[0], hw[1]).reshape(-1)
            host[j * fb:(j + 1) * fb] = cache[seed]
        s, d = ctx.alloc_device(batch_bytes), ctx.alloc_device(batch_bytes)
        ctx.upload(s, host, batch_bytes)
        ctx.sync()  # host buffer is reused for the next slot
        srcs.append(s)
        dsts.append(d)
    return srcs, dsts, batch_bytes, host


def probe(args):
    """Child of rocprofv3 --pmc: launch the same kernel on the same ring, nothing else."""
    import numpy as np
    from vfilter import Context
    ctx = Context(int(os.environ.get("VF_DEVICE", "0")))
    srcs, dsts, batch_bytes, _ = make_ring(ctx, args.batch, args.ring_gb, np)
    ctx.bench_device_ring(srcs, dsts, batch_bytes, args.steps)
    ctx.close()


def pmc_traffic(args, device=0):
    """HBM bytes per launch from two separate rocprofv3 --pmc passes (FETCH_SIZE needs 3 TCC
    slots and WRITE_SIZE 2, so they cannot share a pass), on rank 0's GPU.  Returns (bytes,
    detail) or (None, why)."""
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        out = tempfile.mkdtemp(prefix="vf_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = ["timeout", "-s", "KILL", "90", rp, "--pmc", ctr, "--output-format", "csv", "-d", out,
               "-o", "pmc", "--", sys.executable, os.path.abspath(__file__), "--probe",
               "--steps", "20", "--batch", str(args.batch), "--ring-gb", str(args.ring_gb)]
        r = subprocess.run(cmd, capture_output=True, text=True, env=dict(os.environ, VF_DEVICE=str(device)))
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files:
            shutil.rmtree(out, ignore_errors=True)
            return None, f"rocprofv3 --pmc {ctr} failed (rc={r.returncode}): {r.stderr[-300:]}"
        per = []
        for fn in files:
            with open(fn) as f:
                for row in csv.DictReader(f):
                    if "invert_stream_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                        per.append(float(row["Counter_Value"]))
        shutil.rmtree(out, ignore_errors=True)
        if not per:
            return None, f"no {ctr} rows for invert_stream_kernel"
        per.sort()
        vals[ctr] = per[len(per) // 2]  # median over dispatches, KB per launch
    # gfx950: FETCH_SIZE counts 64 B per 128-B wide streaming read request -> x2 (guide §HBM)
    fetch = vals["FETCH_SIZE"] * 1024.0 * 2.0
    write = vals["WRITE_SIZE"] * 1024.0
    return fetch + write, {"fetch_size_kb": vals["FETCH_SIZE"], "write_size_kb": vals["WRITE_SIZE"],
                           "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024"}


# kernels of each stage of the fused JPEG pass (vf_jpeg_host.hip run_decode / run_encode; the
# speculative sync at 1080p), for the per-stage issue fractions
JPEG_STAGE_KERNELS = {
    "unstuff": ("k_unstuff_count", "k_unstuff_write"),
    "huffman_sync": ("k_spec", "k_wglink", "k_resolve", "k_finalize", "k_sync", "k_syncg"),
    "huffman_write": ("k_write", "k_write4"),
    "dc_idct": ("k_idct",),
    "color_invert": ("k_color", "k_idct_color422"),
    "fdct_huffman": ("k_fdct", "k_len", "k_zero_stream", "k_pack"),
    "stuffing": ("k_ff_count", "k_ff_write", "k_compact"),
}


def pmc_jpeg(device=0, content="scene"):
    """One per-dispatch rocprofv3 PMC pass over the 1080p JPEG batch (tools/jpeg_bench.py, the
    jpeg_mode workload: 32 frames of the 8 camera-like scenes, q85 4:2:2; content "hard": the
    hard_content workload, 32 noisy scenes at q95), run as a child before anything in this
    process touches the GPU.  Per kernel, from its last dispatch: VALU / LDS / SALU instructions
    and waves, and the shader clock (tools/pmc_issue.py).  Returns {kernel: {...}} or
    {"error": why}."""
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return {"error": "rocprofv3 not found"}
    out = tempfile.mkdtemp(prefix="vf_pmcj_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = ["timeout", "-s", "KILL", "120", rp, "--kernel-trace", "--pmc", "SQ_WAVES", "SQ_INSTS_VALU",
           "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT",
           "--output-format", "csv", "-d", out, "-o", "pmc", "--", sys.executable,
           os.path.join(ROOT, "tools", "jpeg_bench.py"), "--sizes", "1080p", "--batch", "32", "--iters", "3",
           "--cpu-seconds", "0", "--resident-only", "--content", content]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, env=dict(os.environ, VF_DEVICE=str(device)),
                           timeout=240)
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files:
            return {"error": f"rocprofv3 --pmc failed (rc={r.returncode}): {r.stderr[-300:]}"}
        import importlib.util
        spec = importlib.util.spec_from_file_location("pmc_issue", os.path.join(ROOT, "tools", "pmc_issue.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod.per_kernel(files[0], min_waves=1)
    except Exception as e:  # reported in the line, never raised
        return {"error": repr(e)[:300]}
    finally:
        shutil.rmtree(out, ignore_errors=True)


def jpeg_issue_fractions(roofline, per_kernel):
    """Per stage of jpeg_mode.roofline: the VALU and LDS issue fractions -- the compute-side
    bound beside the HBM fraction.  valu_issue_frac = the stage's VALU instructions x 2 cycles
    (a wave64 instruction holds a SIMD-32 for two) / (1,024 SIMDs x the stage's hipEvent time
    x the shader clock); lds_issue_frac = its LDS instructions / (256 CUs x the same cycles),
    one LDS instruction per CU and cycle at best (b64 / b128 accesses take more, so a lower
    bound).  Instruction counts: pmc_jpeg's pass over the same workload."""
    if not per_kernel or "error" in per_kernel:
        return
    clocks = sorted(v["clock_GHz"] for v in per_kernel.values() if v.get("duration_us", 0) > 50)
    clk = clocks[len(clocks) // 2] if clocks else 2.4
    for stage, kernels in JPEG_STAGE_KERNELS.items():
        st = roofline.get(stage)
        if not st:
            continue
        valu = sum(per_kernel[k]["valu_total"] for k in kernels if k in per_kernel)
        lds = sum(per_kernel[k]["lds_total"] for k in kernels if k in per_kernel)
        cyc = st["ms"] * 1e-3 * clk * 1e9
        st["valu_issue_frac"] = round(2.0 * valu / (1024 * cyc), 3)
        st["lds_issue_frac"] = round(lds / (256 * cyc), 3)
        st["kernels"] = {k: {x: per_kernel[k][x] for x in ("duration_us", "valu_per_wave", "lds_per_wave",
                                                             "valu_issue_frac", "lds_issue_frac") if x in per_kernel[k]}
                         for k in kernels if k in per_kernel}
    roofline["issue_fraction_note"] = (
        f"valu_issue_frac = VALU instructions x 2 / (1024 SIMDs x stage cycles), lds_issue_frac = LDS "
        f"instructions / (256 CUs x stage cycles); instruction counts per kernel from a rocprofv3 PMC pass "
        f"(SQ_INSTS_VALU / SQ_INSTS_LDS, summed over the dispatches of the last batch) over the same 1080p batch, shader clock "
        f"{clk:.2f} GHz (GRBM_GUI_ACTIVE / duration, median of the kernels above 50 us)")


# ---------------------------------------------------------------------------------------
# CPU baseline: the oracle's restatement of inverter.py:41 on the host
# ---------------------------------------------------------------------------------------

def cpu_baseline(host_batch, batch, seconds, np):
    from oracle import oracle
    frames = host_batch.reshape(batch, H, W, C)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for f in range(batch):
            oracle.invert(frames[f])  # new array per call, as cv2.bitwise_not(frame)
        n += batch
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{n} x 1080p frames ({dt:.1f} s), np.bitwise_not per frame "
                      f"(oracle restatement of cv2.bitwise_not, inverter.py:41), 1 thread"}


def cpu_baseline_sizes(seconds, np):
    """The same 1-core oracle baseline at 480p and 4K (north star: every size is reported next
    to the reference CPU path), `seconds` per size."""
    from oracle import oracle
    from vfilter.synthetic import synthetic_frame
    out = {}
    for name, (hh, ww) in (("480p", (480, 640)), ("4k", (2160, 3840))):
        frames = [synthetic_frame(s, hh, ww) for s in range(4)]
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            oracle.invert(frames[n % 4])
            n += 1
        dt = time.perf_counter() - t0
        out[name] = {"value": round(n / dt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                     "sample": f"{n} x {name} frames ({dt:.1f} s), np.bitwise_not per frame, 1 thread"}
    return out


def cpu_worker(seconds):
    """Child of cpu_baseline_multi: one process, np.bitwise_not(x, out=y) over a contiguous
    1080p batch of 32 (BASELINE.md's CPU-baseline plan) for `seconds`; prints frames done."""
    import numpy as np
    x = np.random.default_rng(os.getpid() % 97).integers(0, 256, (32, H, W, C), dtype=np.uint8)
    y = np.empty_like(x)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        np.bitwise_not(x, out=y)
        n += len(x)
    print(json.dumps({"frames": n, "seconds": time.perf_counter() - t0}), flush=True)


def cpu_baseline_multi(seconds, procs):
    """BASELINE.md plan (ii): the reference's filter arithmetic on `procs` host processes at
    once (the reference scales by worker processes, distributor.py:229-241), each over its
    own contiguous 1080p batch.  Started as child processes (fresh interpreters, no GPU)."""
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-worker", str(seconds)]
    ps = [subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True) for _ in range(procs)]
    rate = 0.0
    for p in ps:
        so, _ = p.communicate(timeout=seconds + 120)
        r = json.loads([ln for ln in so.splitlines() if ln.startswith("{")][-1])
        rate += r["frames"] / r["seconds"]
    return {"value": round(rate, 1), "unit": "frames/s", "cores": procs, "kind": "port",
            "GBps_r_plus_w": round(rate * 2 * FRAME_BYTES / 1e9, 1),
            "sample": f"{procs} processes x {seconds:.0f} s of np.bitwise_not(x, out=y) over a 32-frame "
                      f"1080p batch each (oracle arithmetic of inverter.py:41)"}


def cgroup_cpus():
    """CPUs this process may use by its cgroup's CPU quota (cpu.max), None when unlimited: on
    the GPU box the lease's share (16 per GPU) is far below the machine's CPU count."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            return None if q == "max" else max(1, int(int(q) / int(per)))
        except (OSError, ValueError):
            pass
    return None


def host_copy_child(seconds):
    """Child of host_copy_ceiling: on each NUMA node, threads pinned to the node's CPUs copy
    between two node-local 64 MiB buffers (np.copyto, no GIL) for `seconds`, all nodes at once;
    prints read + write GB/s per node.  Threads per node: the node's CPUs, capped by the
    process's CPU quota shared evenly over the nodes."""
    import threading
    import numpy as np
    from vfilter import numa
    nodes = [n for n in range(numa.node_count()) if numa.node_cpus(n)] or [None]
    quota = cgroup_cpus() or len(os.sched_getaffinity(0))
    per = {n: max(1, min(len(numa.node_cpus(n)) if n is not None else quota, quota // len(nodes))) for n in nodes}
    moved = {n: [0] * per[n] for n in nodes}
    ready = threading.Barrier(sum(per.values()) + 1)
    stop = threading.Event()

    def run(n, i):
        numa.pin_thread_to_node(n)
        a = np.ones(64 << 20, np.uint8)  # first touch after the pin: node-local pages
        b = np.zeros_like(a)
        ready.wait()
        k = 0
        while not stop.is_set():
            np.copyto(b, a)
            k += 1
        moved[n][i] = 2 * k * a.nbytes
    ths = [threading.Thread(target=run, args=(n, i)) for n in nodes for i in range(per[n])]
    for t in ths:
        t.start()
    ready.wait()
    t0 = time.perf_counter()
    time.sleep(seconds)
    stop.set()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    out = {str(n): round(sum(moved[n]) / dt / 1e9, 1) for n in nodes}
    print(json.dumps({"GBps_r_plus_w_per_node": out, "threads_per_node": {str(n): per[n] for n in nodes},
                      "cpu_quota": cgroup_cpus(), "affinity_cpus": len(os.sched_getaffinity(0))}), flush=True)


def host_copy_ceiling(seconds=3.0):
    """The host side's own bound for the distributor legs: node-local copy bandwidth (read +
    write) summed over the NUMA nodes, measured in a fresh child with threads pinned per node
    (host_copy_child).  It replaces round 2's figure from 16 numpy processes, which was bound
    by the lease's CPU share, not by DRAM; when the share still binds it (threads < CPUs), the
    line says so."""
    cmd = [sys.executable, os.path.abspath(__file__), "--host-copy-child", str(seconds)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds + 120)
        d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    except Exception as e:  # reported, never raised
        return {"error": repr(e)[:300]}
    tot = round(sum(d["GBps_r_plus_w_per_node"].values()), 1)
    threads = sum(d["threads_per_node"].values())
    d["GBps_r_plus_w"] = tot
    d["bound"] = ("CPU share (threads < the nodes' CPUs): a lower bound on host DRAM bandwidth"
                  if d.get("cpu_quota") and threads < d["affinity_cpus"] else "host DRAM (all CPUs copying)")
    d["what"] = f"np.copyto between node-local 64 MiB buffers, {threads} pinned threads over all nodes at once"
    return d


def resolution_leg(ctx, np, rank, world, steps, barrier_sync, reduce_max):
    """North star: kernel-only throughput at 480p, 1080p and 4K on this run's GPUs, as
    whole-job frames/s and as a fraction of the HBM roofline.  Same timing rules as the
    headline (warmup, barrier + sync on both sides, max over ranks; hipEvent mean per launch
    for the roofline); batches of ~200-400 MB per launch so no size is launch-bound."""
    out = {}
    for name, (hh, ww), batch in (("480p", (480, 640), 256), ("1080p", (H, W), 32), ("4k", (2160, 3840), 16)):
        srcs, dsts, bb, _ = make_ring(ctx, batch, 2.4, np, rank, world, hw=(hh, ww), distinct=8)
        # warm until a call costs what its kernels cost: the first calls over a fresh ring carry
        # ~8-17 ms of one-off host-side latency (first touch of new allocations)
        for _ in range(5):
            tw = time.perf_counter()
            wr, _ = ctx.bench_device_ring(srcs, dsts, bb, 10)
            tw = time.perf_counter() - tw
            if tw * 1e3 < 1.2 * wr + 0.5:
                break
        barrier_sync()
        t0 = time.perf_counter()
        region_ms, _ = ctx.bench_device_ring(srcs, dsts, bb, steps)
        tc = time.perf_counter() - t0
        ctx.sync()
        barrier_sync()
        elapsed = reduce_max(time.perf_counter() - t0)
        log(f"sizes {name}: warmup call {tw * 1e3:.2f} ms (region {wr:.2f}), timed call {tc * 1e3:.2f} ms "
            f"(region {region_ms:.2f}), wall {elapsed * 1e3:.2f} ms")
        mean_ms = reduce_max(region_ms / steps)
        for s_, d_ in zip(srcs, dsts):
            ctx.free_device(s_)
            ctx.free_device(d_)
        gbs = 2.0 * bb / (mean_ms * 1e-3) / 1e9
        out[name] = {"frame": [hh, ww, C], "batch_per_rank": batch, "steps": steps,
                     "fps": round(world * steps * batch / elapsed, 1),
                     "kernel_GBps_per_gpu": round(gbs, 1), "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4)}
    out["note"] = "kernel-only, HBM-resident, whole job over all ranks; GB/s = slowest rank's mean launch"
    return out


def sweep_leg(ctx, np, host_batch, batch, rank, world, barrier_sync, reduce_max,
              batches=(256, 512, 1024, 2048, 4096), warm_ms=300.0, timed_ms=200.0):
    """BASELINE.json configs[4]: 1080p invert with 256 ... 4096 frames resident in HBM per
    rank (1.6-25.5 GB in, the same out), one launch over the whole batch per step.  Each
    point is warmed for >= warm_ms of kernel time, then >= timed_ms is timed under the
    headline's rules (barrier + sync on both sides, max over ranks)."""
    fb = FRAME_BYTES
    out = {}
    for nb in batches:
        bb = nb * fb
        src, dst = ctx.alloc_device(bb), ctx.alloc_device(bb)
        for off in range(0, nb, batch):  # the rank's synthetic batch, repeated
            k = min(batch, nb - off)
            ctx.upload(src + off * fb, host_batch, k * fb)
        ctx.sync()
        done = 0.0
        while done < warm_ms:
            ms, _ = ctx.bench_device_ring([src], [dst], bb, 2)
            done += ms
        steps = max(3, int(timed_ms / (ms / 2)) + 1)
        barrier_sync()
        t0 = time.perf_counter()
        region, _ = ctx.bench_device_ring([src], [dst], bb, steps)
        ctx.sync()
        barrier_sync()
        elapsed = reduce_max(time.perf_counter() - t0)
        mean_ms = reduce_max(region / steps)
        ctx.free_device(src)
        ctx.free_device(dst)
        gbs = 2.0 * bb / (mean_ms * 1e-3) / 1e9
        out[str(nb)] = {"bytes_in_per_rank": bb, "steps": steps, "fps": round(world * nb * steps / elapsed, 1),
                        "ms_per_launch": round(mean_ms, 4), "kernel_GBps_per_gpu": round(gbs, 1),
                        "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4)}
    out["note"] = "configs[4]: kernel-only, HBM-resident, whole job over all ranks; GB/s = slowest rank's mean launch"
    return out


def end_to_end(ctx, host_batch, batch, np, reps=16, labels=("pageable", "pinned", "pinned_pipelined")):
    """Host->host frames/s (PCIe-inclusive): one synchronous vf_invert_batch_host call per
    batch from pageable numpy memory (staged through the slot ring) and from pinned memory
    (vf_alloc_host: inverted in place over PCIe by one launch, the zero-copy path), and the
    worker's pipelined form (vf_invert_frames_async, two batches in flight, pinned)."""
    import ctypes
    nb = host_batch.nbytes
    out = np.empty_like(host_batch)
    res = {}
    ps = [ctx.alloc_host(nb) for _ in range(2)]
    pd = [ctx.alloc_host(nb) for _ in range(2)]
    try:
        for p in ps:
            np.ctypeslib.as_array((ctypes.c_uint8 * nb).from_address(p))[:] = host_batch
        for label in labels:
            src, dst = (host_batch, out) if label == "pageable" else (ps[0], pd[0])
            ctx.invert_batch_host(src, dst, FRAME_BYTES, batch)  # warm (first DMA touch)
            if label == "pinned_pipelined":
                ctx.invert_batch_host(ps[1], pd[1], FRAME_BYTES, batch)
            t0 = time.perf_counter()
            if label == "pinned_pipelined":
                q = []
                for r in range(reps):
                    q.append(ctx.invert_frames_async([ps[r % 2]], [pd[r % 2]], [nb]))
                    if len(q) == 2:
                        ctx.wait(q.pop(0))
                for t in q:
                    ctx.wait(t)
            else:
                for _ in range(reps):
                    ctx.invert_batch_host(src, dst, FRAME_BYTES, batch)
            dt = time.perf_counter() - t0
            res[f"{label}_fps"] = round(reps * batch / dt, 1)
            res[f"{label}_GBps_each_way"] = round(reps * nb / dt / 1e9, 2)
    finally:
        for p in ps + pd:
            ctx.free_host(p)
    res["pcie_ceiling_fps"] = round(63e9 / FRAME_BYTES, 0)  # Gen5 x16 spec, one direction
    res["pinned_path"] = "zero-copy" if os.environ.get("VF_ZEROCOPY", "1") != "0" else "slot ring (direct DMA)"
    res["note"] = "host->host incl. PCIe both directions; never the headline value"
    return res


def end_to_end_ring(device, host_batch, batch, np, reps=16):
    """The same pinned calls through the slot ring (the north star's double-buffered
    hipMemcpyAsync H2D || kernel || D2H on separate streams), on a context made with
    VF_ZEROCOPY=0, reported next to the zero-copy default."""
    from vfilter import Context
    old = os.environ.get("VF_ZEROCOPY")
    os.environ["VF_ZEROCOPY"] = "0"  # read by vf_create
    try:
        ctx = Context(device, max_frame_bytes=FRAME_BYTES, max_batch=batch)
    finally:
        if old is None:
            os.environ.pop("VF_ZEROCOPY")
        else:
            os.environ["VF_ZEROCOPY"] = old
    try:
        r = end_to_end(ctx, host_batch, batch, np, reps, labels=("pinned", "pinned_pipelined"))
    finally:
        ctx.close()
    return {k: r[k] for k in ("pinned_fps", "pinned_GBps_each_way", "pinned_pipelined_fps",
                              "pinned_pipelined_GBps_each_way")}


SMALL_BATCH = 64  # JPEG frames of the reference app's size (512 x 512, 480p): worker batch


def jpeg_mode(ctx, batch, iters=20):
    """The reference's default mode (use_jpeg=True): decode -> bitwise_not -> encode per frame
    (inverter.py:32 -> :41 -> :44) on 1080p JPEGs made with the PyTurboJPEG defaults (q85,
    4:2:2) from camera-like synthetic scenes.  GPU-resident = the fused GPU pass with the
    compressed batch already in HBM; host_to_host = Python bytes in, bytes out."""
    from vfilter.jpeg import TurboJPEG
    from vfilter.synthetic import synthetic_scene
    tj = TurboJPEG(ctx=ctx)
    scenes = [synthetic_scene(s, H, W) for s in range(8)]
    enc = tj.encode_batch(scenes)  # the app's encode (webcam_app.py:110), on the GPU
    jpgs = [enc[i % len(enc)] for i in range(batch)]
    ctx.jpeg_bench_invert(jpgs, 85, 1, 0, iters=2)
    ms, stages = ctx.jpeg_bench_invert(jpgs, 85, 1, 0, iters=iters)
    tj.invert_batch(jpgs)
    reps = 15
    t0 = time.perf_counter()
    for _ in range(reps):
        tj.invert_batch(jpgs)
    h2h = (time.perf_counter() - t0) / reps
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(2) as ex:  # two host threads, one call each at a time
        list(ex.map(lambda _: tj.invert_batch(jpgs), range(4)))
        t0 = time.perf_counter()
        list(ex.map(lambda _: tj.invert_batch(jpgs), range(30)))
        h2h_pipe = (time.perf_counter() - t0) / 30
    # the worker's form (InverterWorker in JPEG mode): one thread, three batches in flight
    def worker_form(frames, depth=3, reps=21):
        for _ in range(2):  # warm the codecs (a codec's first batch allocates its buffers)
            ts = [tj.invert_batch_submit(frames) for _ in range(depth)]
            for t in ts:
                tj.invert_batch_result(t)
        t0 = time.perf_counter()
        q = [tj.invert_batch_submit(frames) for _ in range(depth - 1)]
        for _ in range(reps):
            q.append(tj.invert_batch_submit(frames))
            tj.invert_batch_result(q.pop(0))
        for t in q:
            tj.invert_batch_result(t)
        return (time.perf_counter() - t0) / (reps - 1 + depth)
    h2h_async = worker_form(jpgs)
    h2h_async2x = worker_form(jpgs + jpgs, reps=11)  # the worker CLI's batch of 64 frames
    outs = tj.invert_batch(jpgs)
    passes = stages.pop("sync_passes", 0.0)
    # the reference app's own frames (webcam_app.py:17,97-111: 512 x 512 crops, PyTurboJPEG's
    # defaults) and 480p: the rates the distributor legs jpeg_512 / jpeg_480p are compared with
    # in batches of SMALL_BATCH: a worker's per-batch host costs (parse, ~25 launches) halve per
    # frame against 32, +30-50 % through the system at these sizes (profiles/r05_small_batch_ab.txt)
    points = {}
    for pname, (ph, pw) in (("512sq", (512, 512)), ("480p", (480, 640))):
        pj = tj.encode_batch([synthetic_scene(s, ph, pw) for s in range(8)])
        pj = [pj[i % len(pj)] for i in range(SMALL_BATCH)]
        ctx.jpeg_bench_invert(pj, 85, 1, 0, iters=2)
        pms, _ = ctx.jpeg_bench_invert(pj, 85, 1, 0, iters=iters)
        wf = sorted(SMALL_BATCH / worker_form(pj) for _ in range(3))  # median of 3
        res = SMALL_BATCH / (pms / 1e3)
        points[pname] = {"frame": [ph, pw, 3], "batch": SMALL_BATCH,
                         "gpu_resident_fps": round(res, 1),
                         "host_to_host_worker_fps": round(wf[1], 1),
                         "host_to_host_worker_fps_runs": [round(x, 1) for x in wf],
                         "worker_of_resident": round(wf[1] / res, 3),
                         "jpeg_bytes_mean": round(sum(len(j) for j in pj) / SMALL_BATCH)}
    # hard content: 32 distinct noisy scenes at q95 (long blocks, dense entropy streams)
    from vfilter.synthetic import synthetic_noisy_scene
    hard = tj.encode_batch([synthetic_noisy_scene(s, H, W) for s in range(batch)], quality=95)
    ctx.jpeg_bench_invert(hard, 85, 1, 0, iters=2)
    hms, hst = ctx.jpeg_bench_invert(hard, 85, 1, 0, iters=iters)
    hpasses = hst.pop("sync_passes", 0.0)
    h_async = worker_form(hard, reps=11)
    hard_out = tj.invert_batch(hard)
    hard_content = {
        "workload": f"1080p noisy scenes (vfilter.synthetic.synthetic_noisy_scene, +-40 noise) encoded at q95 "
                    f"4:2:2, {batch} distinct frames, re-encoded at q85",
        "gpu_resident_fps": round(batch / (hms / 1e3), 1), "gpu_resident_ms_per_batch": round(hms, 3),
        "stages_ms": {k: round(v, 4) for k, v in hst.items()},
        "huffman_sync_mode": "speculative (one pass)" if hpasses == 0 else f"pass-based, {hpasses:.1f} passes",
        "host_to_host_worker_fps": round(batch / h_async, 1),
        "jpeg_bytes_mean": round(sum(len(j) for j in hard) / batch),
        "jpeg_bytes_out_mean": round(sum(len(o) for o in hard_out) / batch),
        "roofline": jpeg_roofline(hst, H, W, batch, sum(len(j) for j in hard), sum(len(o) for o in hard_out))}
    return {"workload": f"1080p JPEG (q85 4:2:2) decode -> bitwise_not -> encode, batch {batch}",
            "gpu_resident_fps": round(batch / (ms / 1e3), 1), "gpu_resident_ms_per_batch": round(ms, 3),
            "stages_ms": {k: round(v, 4) for k, v in stages.items()},
            "huffman_sync_mode": "speculative (one pass)" if passes == 0 else f"pass-based, {passes:.1f} passes",
            "roofline": jpeg_roofline(stages, H, W, batch, sum(len(j) for j in jpgs), sum(len(o) for o in outs)),
            "host_to_host_fps": round(batch / h2h, 1),
            "host_to_host_2threads_fps": round(batch / h2h_pipe, 1),
            "host_to_host_worker_fps": round(batch / h2h_async, 1),
            f"host_to_host_worker_batch{2 * batch}_fps": round(2 * batch / h2h_async2x, 1),
            "host_to_host_note": "1 call at a time | 2 host threads | the worker's form: 1 thread, 3 batches "
                                 "in flight (vf_jpeg_invert_submit / _wait / _fetch)",
            "jpeg_bytes_mean": round(sum(len(j) for j in jpgs) / batch),
            "operating_points": points,
            "hard_content": hard_content}, jpgs


def jpeg_roofline(stages, h, w, batch, j_in, j_out, fused=None):
    """Per-stage algorithmic bytes of the fused JPEG pass (1080p 4:2:2 in and out) against the
    stage's hipEvent time, as a fraction of the 8 TB/s HBM peak, with the resource that binds
    each stage (from the SQ counters in profiles/r02_jpeg_pmc_sq.txt: none of the entropy or
    pixel stages is HBM-bound).  Bytes: J = compressed bytes in / out of the batch; per 4:2:2
    MCU of 16x8 pixels, 4 blocks of 64 coefficients (int16: 128 B) and 64 plane samples."""
    if fused is None:  # the invert path's one-pass IDCT + colour (4:2:2 input; VF_JPEG_FUSE_IDCT=0: two)
        fused = os.environ.get("VF_JPEG_FUSE_IDCT", "1") != "0" and os.environ.get("VF_JPEG_FUSE", "1") != "0"
    mcus = -(-w // 16) * -(-h // 8)
    blocks = batch * mcus * 4
    pix = batch * h * w * 3
    coef, planes = blocks * 128, blocks * 64
    model = {  # stage: (bytes, what, binding resource)
        "unstuff": (2 * j_in, "read J_in, write J_in", "launch/latency (a few MB)"),
        "huffman_sync": (j_in, "read J_in once (the minimum; the speculative decode reads it bpm-fold)",
                         "dependent Huffman table lookups (LDS latency)"),
        "huffman_write": (j_in + coef, "read J_in, write the coefficient blocks",
                          "dependent Huffman table lookups (LDS latency)"),
        "dc_idct": ((8 * blocks, "the DC scan: read + write one int32 per block", "launch/latency (a few MB)")
                    if fused else (coef + planes + 4 * blocks, "read coefficients + DC, write planes",
                                   "load latency + VALU (LDS conflict-free)")),
        # the invert path's colour pass writes the encoder's 4:2:2 sample planes (as many samples
        # as the decoder's) instead of BGR pixels, read back by k_fdct; fused with the IDCT, the
        # decoder's planes stay in LDS
        "color_invert": ((coef + 4 * blocks + planes, "k_idct_color422: read coefficients + DC, write the "
                          "encoder's sample planes (inverted); decoder planes in LDS",
                          "load latency + VALU (IDCT, then colour from LDS)")
                         if fused else (2 * planes, "read planes, write the encoder's sample planes (inverted)",
                                        "load latency per wave")),
        "fdct_huffman": (planes + 3 * j_out + 10 * blocks, "read sample planes, write + pack AC words",
                         "VALU + issue latency"),
        "stuffing": (5 * j_out, "count + write FF00 stuffing, compact", "launch/latency (a few MB)"),
    }
    out = {}
    tot_b, tot_ms = 0, 0.0
    for k, (b, what, bound) in model.items():
        ms = stages.get(k)
        if not ms:
            continue
        gbs = b / (ms * 1e-3) / 1e9
        out[k] = {"bytes": int(b), "ms": round(ms, 4), "GBps": round(gbs, 1),
                  "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4), "bytes_are": what, "bound": bound}
        tot_b += b
        tot_ms += ms
    out["total"] = {"bytes": int(tot_b), "ms": round(tot_ms, 4),
                    "GBps": round(tot_b / (tot_ms * 1e-3) / 1e9, 1) if tot_ms else None,
                    "frac_of_hbm_peak": round(tot_b / (tot_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if tot_ms else None}
    out["note"] = ("algorithmic bytes per stage / hipEvent stage time; the JPEG pass is bound by dependent "
                   "table lookups and VALU latency, not by HBM (no stage above 35 % of peak)")
    return out


def cpu_baseline_jpeg(jpgs, seconds):
    """libjpeg-turbo 2.1.2 (the codec under PyTurboJPEG: the image's libjpeg.so.8, driven as
    TurboJPEG drives it by oracle/jpeg_xcheck.c) decode + np.bitwise_not + encode per frame,
    1 host core — the reference's default per-frame work (inverter.py:32-44)."""
    import numpy as np
    from oracle import jpeg as J
    ok, why = J.libjpeg_available()
    if not ok:
        return {"value": None, "why": why}
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        J.libjpeg_encode(np.bitwise_not(J.libjpeg_decode(jpgs[n % len(jpgs)])), 85, J.TJPF_BGR, 1, False)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 2), "unit": "frames/s", "cores": 1, "kind": "reference",
            "sample": f"{n} x 1080p JPEG frames ({dt:.1f} s) through libjpeg-turbo 2.1.2, 1 thread"}


def control_plane_rate(nworkers, nbytes, frames=150000, timeout_s=120, **kw):
    """tools/distributor_overhead.py --no-copy: the distributor's own frames/s at this frame size
    and worker count (echo workers that leave results in place: no GPU, no host copy)."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "distributor_overhead.py"), "--workers", str(nworkers),
           "--no-copy", "--bytes", str(int(nbytes)), "--frames", str(frames)]
    for k, v in kw.items():
        cmd += [f"--{k}", str(v)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
        line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        return {k: line[k] for k in ("engine", "fps", "distributor_cpu_us_per_frame", "workers", "frame_bytes")}
    except Exception as e:  # reported, never raised
        return {"error": repr(e)[:200]}


def distributor_leg(nworkers, ngpu, host_gbps=None, pcie_gbps=None, frames_scale=1.0, timeout_s=150, jpeg=None,
                    reps=3):
    """BASELINE.json configs[2] and configs[3] at this run's GPU count, host->host through the
    whole fan-out: one Distributor (lossless, in-order reassembly, one NUMA-bound shared-memory
    ring slice per worker) and one `python -m vfilter.inverter` worker process per GPU
    (tools/pipeline_bench.py).
      configs[2]           4K frames, batch 16, frame-index shards (policy "shard"); the
                           producer copies every frame into its slot ("copy")
      configs[2]_resident  the same with frames committed in place (no producer copy)
      configs[3]           480p / 1080p / 4K interleaved 1:1:1, batch 16, pull policy,
                           producer copy, reporting the ordering overhead
      jpeg_1080p           the reference's default deployment: 1080p JPEG frames (q85 4:2:2),
                           workers in JPEG mode (3 batches of 32 in flight), pull policy
      jpeg_1080p_hard      the same on hard content (noisy scenes at q95)
      jpeg_512, jpeg_480p  the reference app's own frame sizes, in batches of SMALL_BATCH (64)
    Every 8th frame is verified in full, the others on their first and last 4 KiB.  Beside each
    leg: the ceilings for this many GPUs — PCIe (the pinned pipelined rate measured in
    end_to_end, each way, per GPU) and host DRAM (the host's measured r+w bandwidth from the
    multi-process CPU baseline over the host bytes each frame costs: producer copy read+write,
    H2D read, D2H write, verification reads).  Run by rank 0 as a child process group with a
    time limit, so a stuck worker cannot outlive the bench; a failure is reported in the line,
    never raised."""
    import signal
    tool = os.path.join(ROOT, "tools", "pipeline_bench.py")
    k4 = 2160 * 3840 * 3
    legs = {"configs[2]": (["--size", "4k", "--batch", "16", "--policy", "shard", "--producer", "copy",
                            "--frames", str(int(768 * nworkers * frames_scale))], k4, 4.25),
            "configs[2]_resident": (["--size", "4k", "--batch", "16", "--policy", "shard", "--producer",
                                     "resident", "--frames", str(int(768 * nworkers * frames_scale))], k4, 2.25),
            "configs[3]": (["--size", "mixed", "--batch", "16", "--policy", "pull", "--producer", "copy",
                            "--frames", str(int(1152 * nworkers * frames_scale))],
                           (640 * 480 + 1920 * 1080 + 3840 * 2160) * 3 // 3, 4.25),
            # the reference's default deployment: JPEG frames, workers in JPEG mode
            "jpeg_1080p": (["--jpeg", "--size", "1080p", "--batch", "32", "--policy", "pull",
                            "--frames", str(int(24576 * nworkers * frames_scale))], 181876, None),
            # the same deployment on hard content: 32 distinct noisy scenes at q95
            "jpeg_1080p_hard": (["--jpeg", "--content", "hard", "--size", "1080p", "--batch", "32", "--policy",
                                 "pull", "--frames", str(int(4608 * nworkers * frames_scale))], None, None),
            # the reference app's own operating point (webcam_app.py:17,97-111: 512 x 512, q85 4:2:2)
            "jpeg_512": (["--jpeg", "--size", "512sq", "--batch", str(SMALL_BATCH), "--policy", "pull",
                          "--frames", str(int(98304 * nworkers * frames_scale))], None, None),
            "jpeg_480p": (["--jpeg", "--size", "480p", "--batch", str(SMALL_BATCH), "--policy", "pull",
                           "--frames", str(int(98304 * nworkers * frames_scale))], None, None)}
    worker_form = {"jpeg_1080p": (jpeg or {}).get("host_to_host_worker_fps")}
    for k_, pn in (("jpeg_512", "512sq"), ("jpeg_480p", "480p")):
        worker_form[k_] = ((jpeg or {}).get("operating_points") or {}).get(pn, {}).get("host_to_host_worker_fps")
    def run_once(cmd):
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             start_new_session=True)
        try:
            so, se = p.communicate(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            so, se = p.communicate()
            return {"error": f"timed out after {timeout_s} s: " + (se or "")[-300:]}
        lines = [ln for ln in so.splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not lines:
            return {"error": f"rc={p.returncode}: {se[-300:]}"}
        return json.loads(lines[-1])

    out = {}
    for name, (extra, fbytes, host_x) in legs.items():
        cmd = [sys.executable, tool, "--workers", str(nworkers), "--gpus", str(ngpu)] + extra
        t0 = time.time()
        # JPEG legs swing between runs (host scheduling of the worker's submit thread): the
        # median of `reps` runs is reported, with every run's rate beside it
        runs = []
        for i in range(reps if host_x is None else 1):
            runs.append(run_once(cmd))
            # a progress line per run: a leg at N > 1 can run for minutes
            log(f"distributor {name} run {i}: " + (f"{runs[-1]['fps']:.1f} fps" if "fps" in runs[-1]
                                                     else str(runs[-1].get("error"))[:200])
                + f" ({time.time() - t0:.1f} s)")
        good = sorted((r for r in runs if "error" not in r), key=lambda r: r["fps"])
        if not good:
            out[name] = runs[-1]
            continue
        r = good[(len(good) - 1) // 2]
        fps_runs = [g["fps"] for g in good]
        if len(runs) > 1:
            r["fps_runs"] = [x.get("fps", x.get("error")) for x in runs]
            r["fps_min"], r["fps_max"] = fps_runs[0], fps_runs[-1]
            r["n_errors"] = sum(g.get("n_errors", 0) for g in good)
        keep = ("kind", "size", "content", "workers", "gpus", "policy", "producer", "producers", "batch",
                "inflight_per_worker", "host_work_placement",
                "ring_slots_per_worker", "frames", "fps", "GBps_each_way",
                "latency_ms_mean", "latency_ms_p99", "reorder_wait_mean_ms", "reorder_wait_max_ms",
                "max_buffer_depth", "out_of_order_arrivals", "n_errors", "verify_full_every",
                "slice_bytes_per_worker", "slice_numa", "slice_numa_bound", "evictions", "frames_lost",
                "fps_runs", "fps_min", "fps_max")
        leg = {k: r[k] for k in keep if k in r}
        leg["fps_per_gpu"] = round(r["fps"] / max(1, min(ngpu, nworkers)), 1)
        if host_x is not None:
            ceil = {"frame_bytes_mean": fbytes, "host_bytes_per_frame": f"{host_x} x frame"}
            if pcie_gbps:
                ceil["pcie_fps"] = round(min(ngpu, nworkers) * pcie_gbps * 1e9 / fbytes, 1)
            if host_gbps:
                ceil["host_dram_fps"] = round(host_gbps * 1e9 / (host_x * fbytes), 1)
            leg["ceilings"] = ceil
        else:  # JPEG: bound by the GPU codec, compared with its worker-form rate in jpeg_mode
            leg["jpeg_bytes_in_mean"] = r.get("jpeg_bytes_in_mean")
            wf = worker_form.get(name)
            if wf:
                leg["worker_form_fps_per_gpu"] = wf
                leg["of_worker_form"] = round(r["fps"] / (min(ngpu, nworkers) * wf), 3)
            if r.get("jpeg_bytes_in_mean"):  # the distributor's own rate at this frame size beside it
                leg["control_plane"] = control_plane_rate(nworkers, r["jpeg_bytes_in_mean"])
        leg["wall_s"] = round(time.time() - t0, 1)
        out[name] = leg
    out["note"] = ("host->host through distributor + per-worker shared-memory ring slices + one worker process "
                   "per GPU; bound by host memory and PCIe, not HBM; never the headline value. ceilings: pcie = "
                   "GPUs x end_to_end.pinned_pipelined GB/s each way / frame bytes; host_dram = "
                   "cpu_baseline.host_copy_ceiling's node-local r+w GB/s (pinned threads on every node; its "
                   "'bound' says whether the lease's CPU share limited it) / host bytes per frame")
    return out


def jpeg_child(args):
    """The JPEG leg in a fresh interpreter without torch, as a worker process runs it
    (`python -m vfilter.inverter` imports no torch); prints one JSON object."""
    from vfilter import Context
    from vfilter.inverter import pin_to_gpu_node
    pin_to_gpu_node(args.jpeg_child)  # as the worker process pins itself (its "worker form" is measured here)
    ctx = Context(args.jpeg_child)
    jpeg, jpgs = jpeg_mode(ctx, args.batch)
    ctx.close()
    if args.cpu_seconds > 0:
        jpeg["cpu_reference"] = cpu_baseline_jpeg(jpgs, min(5.0, args.cpu_seconds))
    print(json.dumps(jpeg), flush=True)


def run_jpeg_child(device, batch, cpu_seconds, timeout_s=300):
    cmd = [sys.executable, os.path.abspath(__file__), "--jpeg-child", str(device), "--batch", str(batch),
           "--cpu-seconds", str(cpu_seconds)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout_s} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"rc={r.returncode}: {r.stderr[-300:]}"}
    return json.loads(lines[-1])


def per_frame_leg(device, pcie_gbps=None, timeout_s=120):
    """north_star's own entry point: one uint8 HxWx3 numpy frame in, the same-shape frame out
    (vfilter.bitwise_not in place of cv2.bitwise_not, inverter.py:41), median per-call latency at
    480p / 1080p / 4K from tools/per_frame_probe.py in a child without torch: the drop-in
    (pageable frame in, result in the pinned arena), pinned in/out, and numpy on 1 core.
    pcie_floor_ms = frame bytes / the pinned pipelined GB/s each way (both directions overlapped)."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "per_frame_probe.py")]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s,
                           env=dict(os.environ, VF_DEVICE=str(device)))
        rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not rows:
            return {"error": f"rc={r.returncode}: {r.stderr[-300:]}"}
    except Exception as e:  # reported, never raised
        return {"error": repr(e)[:300]}
    out = {}
    for row in rows:
        if pcie_gbps:
            row["pcie_floor_ms"] = round(row["frame_bytes"] / (pcie_gbps * 1e9) * 1e3, 4)
        out[row.pop("size")] = row
    out["note"] = ("median ms per call over 60-200 calls; dropin = vfilter.bitwise_not(frame) on an ordinary "
                   "numpy frame (inverter.py:41's call shape), cpu = np.bitwise_not on 1 core")
    return out


HEADLINE_MAX_BYTES = 7000  # the driver parses the last stdout line from a bounded tail
DETAIL_DEFAULT = os.path.join(ROOT, "gpurun_out", "bench_detail.json")


def _pick(d, *keys):
    """The keys of dict d that are present (None-safe)."""
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _leg_summary(leg):
    if not isinstance(leg, dict):
        return None
    if "error" in leg:
        return {"error": str(leg["error"])[:120]}
    s = _pick(leg, "fps", "fps_min", "fps_max", "n_errors", "frames_lost", "of_worker_form", "workers", "gpus")
    if "reorder_wait_mean_ms" in leg:
        s["reorder_wait_ms"] = leg["reorder_wait_mean_ms"]
    cp = leg.get("control_plane")
    if isinstance(cp, dict) and "fps" in cp:
        s["control_plane_fps"] = cp["fps"]
    ceil = leg.get("ceilings")
    if isinstance(ceil, dict):
        s["ceilings_fps"] = _pick(ceil, "pcie_fps", "host_dram_fps")
    return s


def headline(line):
    """The compact last stdout line (<= HEADLINE_MAX_BYTES) built from the full bench record
    `line`: the contract keys, roofline (with traffic) and cpu_baseline, and one-number
    summaries of every leg.  Everything else stays in the detail file (bench_detail.json)."""
    h = {k: line.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                   "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")}
    rf = line.get("roofline") or {}
    h["roofline"] = _pick(rf, "bound", "achieved", "peak", "unit", "frac", "traffic", "algorithmic_bytes_per_launch",
                          "mean_launch_ms", "isolated_launch_ms_median", "timing")
    td = rf.get("traffic_detail")
    if isinstance(td, dict):
        h["roofline"]["traffic_pmc_kb"] = _pick(td, "fetch_size_kb", "write_size_kb")
    elif td is not None:
        h["roofline"]["traffic_detail"] = str(td)[:160]
    cpu = line.get("cpu_baseline")
    if isinstance(cpu, dict):
        c = _pick(cpu, "value", "unit", "cores", "kind", "sample")
        mp = cpu.get("multi_process")
        if isinstance(mp, dict):
            c["multi_process"] = _pick(mp, "value", "cores", "GBps_r_plus_w")
        if isinstance(cpu.get("process_scaling_fps"), dict):
            c["process_scaling_fps"] = cpu["process_scaling_fps"]
        if isinstance(cpu.get("sizes"), dict):
            c["sizes_fps"] = {k: v.get("value") for k, v in cpu["sizes"].items() if isinstance(v, dict)}
        hc = cpu.get("host_copy_ceiling")
        if isinstance(hc, dict):
            c["host_copy_GBps"] = hc.get("GBps_r_plus_w", hc.get("error"))
        h["cpu_baseline"] = c
    else:
        h["cpu_baseline"] = cpu
    sz = line.get("sizes")
    if isinstance(sz, dict):  # whole-job fps and the slowest rank's HBM fraction per size
        h["sizes"] = {k: _pick(v, "fps", "batch_per_rank", "kernel_GBps_per_gpu", "frac_of_hbm_peak")
                      for k, v in sz.items() if isinstance(v, dict)}
    sw = line.get("configs4_sweep")
    if isinstance(sw, dict):
        h["configs4_sweep"] = {k: _pick(v, "fps", "frac_of_hbm_peak") for k, v in sw.items() if isinstance(v, dict)}
    e2e = line.get("end_to_end")
    if isinstance(e2e, dict):
        h["end_to_end"] = _pick(e2e, "pageable_fps", "pinned_fps", "pinned_pipelined_fps",
                                "pinned_pipelined_GBps_each_way", "pcie_ceiling_fps")
    pf = line.get("per_frame")
    if isinstance(pf, dict):
        h["per_frame_ms"] = {k: (_pick(v, "dropin_ms", "pinned_ms", "cpu_ms", "pcie_floor_ms")
                                 if isinstance(v, dict) else v) for k, v in pf.items() if k != "note"}
    jm = line.get("jpeg_mode")
    if isinstance(jm, dict):
        if "error" in jm:
            h["jpeg_mode"] = {"error": str(jm["error"])[:160]}
        else:
            j = _pick(jm, "gpu_resident_fps", "host_to_host_worker_fps")
            j["stages_ms"] = jm.get("stages_ms")
            hc = jm.get("hard_content")
            if isinstance(hc, dict):
                j["hard"] = _pick(hc, "gpu_resident_fps", "host_to_host_worker_fps", "huffman_sync_mode")
                j["hard"]["huffman_sync_ms"] = (hc.get("stages_ms") or {}).get("huffman_sync")
            op = jm.get("operating_points")
            if isinstance(op, dict):
                j["operating_points"] = {k: _pick(v, "gpu_resident_fps", "host_to_host_worker_fps",
                                                  "worker_of_resident") for k, v in op.items()}
            cr = jm.get("cpu_reference")
            if isinstance(cr, dict):
                j["cpu_reference"] = _pick(cr, "value", "cores", "kind")
            h["jpeg_mode"] = j
    dl = line.get("distributor")
    if isinstance(dl, dict):
        h["distributor"] = {k: _leg_summary(v) for k, v in dl.items() if k != "note"}
    h["detail"] = line.get("detail")
    return h


def emit(line, path=None):
    """Write the full record to the detail file (and stderr), then print the compact headline
    as the LAST stdout line; returns the headline."""
    path = path or os.environ.get("BENCH_DETAIL", DETAIL_DEFAULT)
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(line, f)
        line["detail"] = os.path.relpath(path, ROOT) if path.startswith(ROOT) else path
    except OSError as e:
        line["detail"] = f"not written: {e}"
    print("[bench] detail: " + json.dumps(line), file=sys.stderr, flush=True)
    h = headline(line)
    s = json.dumps(h)
    if len(s) > HEADLINE_MAX_BYTES:  # never lose the headline: drop the leg summaries first
        for k in ("distributor", "configs4_sweep", "jpeg_mode", "per_frame_ms", "sizes", "end_to_end"):
            h.pop(k, None)
            s = json.dumps(h)
            if len(s) <= HEADLINE_MAX_BYTES:
                break
    print(s, flush=True)
    return h


def main():
    args = parse()
    if args.probe:
        return probe(args)
    if args.jpeg_child >= 0:
        return jpeg_child(args)
    if args.cpu_worker:
        return cpu_worker(args.cpu_worker)
    if args.host_copy_child:
        return host_copy_child(args.host_copy_child)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus {args.gpus}; using WORLD_SIZE")

    import numpy as np
    import torch
    import torch.distributed as dist
    from vfilter import Context

    # one GPU per rank (LOCAL_RANK); VF_DEVICE + BENCH_DIST_BACKEND=gloo rehearse N ranks on
    # one card (the timing barrier is the only cross-rank operation, so gloo is enough)
    device = int(os.environ.get("VF_DEVICE", local_rank))
    have_gpu = torch.cuda.device_count() > 0  # counts devices without initialising HIP
    backend = os.environ.get("BENCH_DIST_BACKEND") or ("nccl" if have_gpu else "gloo")
    cpu_group = None
    if world > 1:
        dist.init_process_group(backend, rank=rank, world_size=world)
        cpu_group = dist.new_group(backend="gloo")  # host-only barrier before any GPU work

    # PMC passes run before ANY rank touches a GPU: rank 0's profiler child owns rank 0's GPU
    # (the others wait on a host-only barrier, so nothing else runs on the card being counted)
    traffic, traffic_detail = None, "skipped"
    jpeg_pmc = jpeg_pmc_hard = None
    if rank == 0 and not args.no_traffic:
        t0 = time.time()
        traffic, traffic_detail = pmc_traffic(args, device)
        log(f"pmc traffic: {traffic} ({traffic_detail}) in {time.time() - t0:.1f}s")
        if not args.no_jpeg:
            t0 = time.time()
            jpeg_pmc = pmc_jpeg(device)
            jpeg_pmc_hard = pmc_jpeg(device, "hard")
            log(f"pmc jpeg: {len(jpeg_pmc)} + {len(jpeg_pmc_hard)} (hard) kernels in {time.time() - t0:.1f}s")
    if world > 1:
        dist.barrier(group=cpu_group)
    have_gpu = torch.cuda.is_available()
    if have_gpu:
        torch.cuda.set_device(device)

    def barrier_sync():
        if have_gpu:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            if have_gpu:
                torch.cuda.synchronize()

    ctx = Context(device, max_frame_bytes=FRAME_BYTES, max_batch=args.batch)
    srcs, dsts, batch_bytes, host_batch = make_ring(ctx, args.batch, args.ring_gb, np, rank, world)
    log(f"rank {rank}: ring {len(srcs)} x 2 x {batch_bytes / 1e6:.1f} MB on device {device}")

    if args.warmup:
        ctx.bench_device_ring(srcs, dsts, batch_bytes, args.warmup)
    barrier_sync()
    t0 = time.perf_counter()
    # the K steps, back to back on one stream; a hipEvent pair brackets them on that stream
    region_ms, _ = ctx.bench_device_ring(srcs, dsts, batch_bytes, args.steps)  # returns synchronised
    barrier_sync()
    elapsed = time.perf_counter() - t0
    # untimed: isolated per-launch durations (event pair around each launch) for reference
    _, isolated = ctx.bench_device_ring(srcs, dsts, batch_bytes, min(args.steps, 60), per_launch=True)

    def reduce_max(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda" if (have_gpu and backend == "nccl") else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    elapsed = reduce_max(elapsed)

    # average launch duration over the timed region (includes the ~1-2 us kernel boundaries)
    mean_ms = region_ms / args.steps if args.steps else float("nan")
    achieved = 2.0 * batch_bytes / (mean_ms * 1e-3) / 1e9
    for s_, d_ in zip(srcs, dsts):  # the sizes leg needs the HBM
        ctx.free_device(s_)
        ctx.free_device(d_)
    sizes = None
    if not args.no_sizes:
        sizes = resolution_leg(ctx, np, rank, world, 100, barrier_sync, reduce_max)
        if rank == 0:
            log(f"sizes: {sizes}")
    e2e = None
    cpu = None
    if rank == 0 and not args.no_e2e:  # before the sweep's 51 GB of allocations come and go
        e2e = end_to_end(ctx, host_batch, args.batch, np)
        e2e["slot_ring"] = end_to_end_ring(device, host_batch, args.batch, np)
        log(f"end-to-end: {e2e}")
    sweep = None
    if not args.no_sweep:
        sweep = sweep_leg(ctx, np, host_batch, args.batch, rank, world, barrier_sync, reduce_max)
        if rank == 0:
            log(f"configs[4] sweep: {sweep}")
    if world > 1 and rank != 0:
        # No collective follows: the other ranks leave here, so that their idle GPU contexts
        # (and their hardware queues) are gone while rank 0 runs the JPEG, per-frame and
        # distributor legs.  Rehearsing N ranks on one card, the idle contexts' queues slowed the
        # workers' JPEG kernels about 4x, past the legs' time limits.
        ctx.close()
        try:  # local teardown: rank 0 runs no collective after this point
            dist.destroy_process_group()
        except Exception as e:  # reported, never raised
            log(f"rank {rank}: destroy_process_group: {e!r}"[:200])
        return
    jpeg = None
    if rank == 0 and not args.no_jpeg:
        jpeg = run_jpeg_child(device, args.batch, args.cpu_seconds)
        if isinstance(jpeg.get("roofline"), dict):
            jpeg_issue_fractions(jpeg["roofline"], jpeg_pmc)
        hc = jpeg.get("hard_content")
        if isinstance(hc, dict) and isinstance(hc.get("roofline"), dict):
            jpeg_issue_fractions(hc["roofline"], jpeg_pmc_hard)
        log(f"jpeg mode: {jpeg}")
    if rank == 0 and args.cpu_seconds > 0:
        # after every timed region (the other ranks have left); at N > 1 a shorter sample
        # without the process-count series keeps the run bounded
        full = world == 1
        cpu = cpu_baseline(host_batch, args.batch, args.cpu_seconds if full else min(3.0, args.cpu_seconds), np)
        procs = min(args.cpu_procs, len(os.sched_getaffinity(0)))
        if procs > 1:
            cpu["multi_process"] = cpu_baseline_multi(min(5.0 if full else 2.0, args.cpu_seconds), procs)
            if full:  # BASELINE.md plan: 1, 2, 4, ... processes, to show where host memory saturates
                series = {}
                p_ = 1
                while p_ < procs:
                    series[str(p_)] = cpu_baseline_multi(min(2.0, args.cpu_seconds), p_)["value"]
                    p_ *= 2
                series[str(procs)] = cpu["multi_process"]["value"]
                cpu["process_scaling_fps"] = series
        if full:
            cpu["sizes"] = cpu_baseline_sizes(min(3.0, args.cpu_seconds), np)
        cpu["host_copy_ceiling"] = host_copy_ceiling(3.0 if full else 1.5)
        log(f"cpu baseline: {cpu}")

    ctx.close()

    per_frame = None
    if rank == 0 and not args.no_per_frame:
        per_frame = per_frame_leg(device, (e2e or {}).get("pinned_pipelined_GBps_each_way"))
        log(f"per frame: {per_frame}")

    fanout = None
    if not args.no_distributor:
        if rank == 0:
            # one worker per rank; workers share GPUs only when rehearsing N ranks on fewer cards
            host_gbps = (cpu or {}).get("host_copy_ceiling", {}).get("GBps_r_plus_w")
            pcie_gbps = (e2e or {}).get("pinned_pipelined_GBps_each_way")
            fanout = distributor_leg(world, max(1, min(world, torch.cuda.device_count())), host_gbps, pcie_gbps,
                                     jpeg=jpeg if isinstance(jpeg, dict) else None, reps=max(1, args.dist_reps))
            log(f"distributor leg: {fanout}")

    if rank == 0:
        frames = world * args.steps * args.batch
        line = {
            "metric": METRIC,
            "value": round(frames / elapsed, 1),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded uniform uint8 frames, seed = frame index mod 97, resident in HBM)",
            "config": {"workload": "configs[1]: 1080p RGB invert, batch=32, kernel-only, HBM-resident",
                       "frame": [H, W, C], "global_batch": world * args.batch,
                       "frames_per_rank_step": args.batch,
                       "ring_bytes_in_plus_out": 2 * batch_bytes * len(srcs),
                       "parallelism": f"frame-index shard x{world}: rank r step s = global batch s*{world}+r "
                                      "(vfilter.sharding; no collective)",
                       "kernel": "invert_stream_kernel<4,nt,nt>, grid 32 WG/CU (vf_kernels.hip)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "algorithmic_bytes_per_launch": 2 * batch_bytes,
                         "mean_launch_ms": round(mean_ms, 5),
                         "timing": "hipEvent pair around the K back-to-back launches on their stream / K",
                         "isolated_launch_ms_median": round(float(np.median(isolated)), 5),
                         "traffic_detail": traffic_detail},
            "cpu_baseline": cpu,
            "sizes": sizes,
            "configs4_sweep": sweep,
            "end_to_end": e2e,
            "jpeg_mode": jpeg,
            "distributor": fanout,
            "per_frame": per_frame,
        }
        emit(line)
    if world > 1:
        try:  # the other ranks have left (after the last collective); the line is out already
            dist.destroy_process_group()
        except Exception as e:
            log(f"destroy_process_group: {e!r}"[:200])


if __name__ == "__main__":
    main()
