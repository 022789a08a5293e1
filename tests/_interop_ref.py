"""Interop with the real reference over ZeroMQ (run by tests/test_reference_interop.py under
/opt/conda/bin/python3.9, the only interpreter here with pyzmq; the reference lives only in
the build container, so these tests skip on the GPU box).

  python3.9 -B _interop_ref.py <reference_dir> <repo_dir> ref-distributor|ref-worker

ref-distributor  the reference's Distributor (distributor.py) feeds this build's Worker
                 speaking protocol v0 over zmq; prints what the reference collected.
ref-worker       this build's Distributor (zmq, latest policy, display reassembly) feeds the
                 reference's Worker loop (worker.py) with a byte-inverting plugin.
The plugins compute ~x with numpy; the point is the wire and the loop semantics.
"""
import json
import os
import socket
import sys
import threading
import time

import numpy as np


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def wait_until(cond, timeout=15.0):
    t0 = time.time()
    while not cond():
        if time.time() - t0 > timeout:
            return False
        time.sleep(0.005)
    return True


def frames():
    return [np.random.default_rng(500 + k).integers(0, 256, (h, w, 3), dtype=np.uint8)
            for k, (h, w) in enumerate([(480, 480), (120, 160), (17, 13), (480, 640)])]


def main():
    ref_dir, repo, mode = sys.argv[1], sys.argv[2], sys.argv[3]
    sys.path.insert(0, ref_dir)
    sys.path.insert(0, os.path.join(repo, "distributed-video-filter_amd"))
    out = {"mode": mode, "frames": []}
    if mode == "ref-distributor":
        from distributor import Distributor as RefDistributor
        from vfilter.worker import Worker

        class NumpyInverter(Worker):
            def __call__(self, frame):
                return np.bitwise_not(np.frombuffer(frame, np.uint8)).tobytes()

        dport, cport = free_port(), free_port()
        d = RefDistributor(dport, cport, 0, False)
        d.start()
        w = NumpyInverter("127.0.0.1", dport, cport, protocol="v0", transport="zmq")
        t = threading.Thread(target=w.start, daemon=True)
        t.start()
        for f in frames():
            idx = d.frame_index_counter
            d.add_frame_for_distribution(f.tobytes())
            ok = wait_until(lambda: idx in d.received_frames)
            e = d.received_frames.get(idx, {})
            out["frames"].append({"index": idx, "ok": ok,
                                  "exact": ok and bytes(e["frame_data"]) == np.bitwise_not(f).tobytes(),
                                  "pid_is_worker": e.get("process_id") == str(os.getpid()),
                                  "start_le_end": ok and e["start_time"] <= e["end_time"]})
        w.stop()
        d.stop()
        time.sleep(0.1)
    else:
        from worker import Worker as RefWorker
        from vfilter.distributor import Distributor

        class RefByteInverter(RefWorker):
            def __call__(self, frame_bytes):
                return np.bitwise_not(np.frombuffer(frame_bytes, np.uint8)).tobytes()

        d = Distributor(free_port(), free_port(), 0, False, transport="zmq", verbose=False)
        d.start()
        w = RefByteInverter("127.0.0.1", d.distribute_port, d.collect_port)
        t = threading.Thread(target=w.start, daemon=True)
        t.start()
        for f in frames():
            idx = d.frame_index_counter
            d.add_frame_for_distribution(f.tobytes())
            ok = wait_until(lambda: idx in d.received_frames)
            e = d.received_frames.get(idx, {})
            out["frames"].append({"index": idx, "ok": ok,
                                  "exact": ok and bytes(e["frame_data"]) == np.bitwise_not(f).tobytes(),
                                  "pid_is_worker": e.get("process_id") == str(os.getpid()),
                                  "start_le_end": ok and e["start_time"] <= e["end_time"]})
        out["display_update"] = d.update_display_frame()
        out["stats"] = d.get_frame_stats()
        w.running = False
        d.cleanup()
    print(json.dumps(out))
    sys.stdout.flush()
    os._exit(0)  # the reference's threads are non-daemon-safe; leave without joining them


if __name__ == "__main__":
    main()
