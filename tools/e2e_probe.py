#!/usr/bin/env python3
"""Host->host rates of vf_invert_batch_host (pageable, pinned, pinned pipelined) at 1080p x 32
and 4K x 16 in this process (bench.end_to_end), plus where the library put its pinned pages.
  VF_NUMA=0 python tools/e2e_probe.py    # hipHostMalloc placement instead of the GPU's node"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-video-filter_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from vfilter import Context  # noqa: E402
from vfilter.numa import gpu_numa_node, node_count  # noqa: E402

dev = int(os.environ.get("VF_DEVICE", "0"))
for name, (h, w, b) in {"1080p": (1080, 1920, 32), "4k": (2160, 3840, 16)}.items():
    bench.H, bench.W = h, w
    bench.FRAME_BYTES = h * w * 3
    ctx = Context(dev, max_frame_bytes=h * w * 3, max_batch=b)
    host = np.random.default_rng(0).integers(0, 256, b * h * w * 3, dtype=np.uint8)
    r = bench.end_to_end(ctx, host, b, np)
    r.update({"size": name, "batch": b, "VF_NUMA": os.environ.get("VF_NUMA", "1"),
              "VF_ZEROCOPY": os.environ.get("VF_ZEROCOPY", "1"), "VF_SCATTER": os.environ.get("VF_SCATTER", "1"),
              "gpu_numa_node": gpu_numa_node(dev), "numa_nodes": node_count(),
              "cpu": os.sched_getaffinity(0).__len__()})
    r.pop("note", None)
    print(json.dumps(r), flush=True)
    ctx.close()
