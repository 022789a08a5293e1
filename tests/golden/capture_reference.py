"""Capture golden traces from the REAL reference plumbing (distributor.py / worker.py).

Run in the build container only (the reference is not on the GPU box):

    env -u PYTHONHOME -u PYTHONPATH /opt/conda/bin/python3.9 -B \
        tests/golden/capture_reference.py /root/reference tests/golden

``/opt/conda/bin/python3.9`` is the only interpreter here with pyzmq (22.2.1 / libzmq 4.3.4),
which the reference imports at module level.  ``-B`` keeps ``__pycache__`` out of the
read-only reference tree.  Nothing of the reference is copied: this script imports it,
drives it through its public methods and sockets, and writes only observed inputs and
outputs as JSON fixtures:

  ref_ingest.json    add_frame_for_distribution (distributor.py:173-203) with the dispatch
                     thread idle: which frame indices the bounded queue keeps.
  ref_display_*.json the collect thread (distributor.py:253-289) fed through its real PULL
                     socket, one 5-part message at a time (worker.py:63-67 layout), with
                     update_display_frame / get_frame_to_display (distributor.py:309-344)
                     called between messages: the reorder/display policy, op by op.
  ref_dispatch.json  the dispatch thread (distributor.py:205-251) answering READY from a
                     real DEALER: latest-wins slot, at-most-once, monotonic indices.
  ref_worker.json    the reference Worker loop (worker.py:30-76) with a plugin subclass
                     (the reference's own extension point, worker.py:78-80) that inverts
                     bytes, against the reference Distributor: the 5-part result layout and
                     the payload bytes for seeded frames.
"""
import json
import os
import random
import socket
import sys
import threading
import time

import numpy as np


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def payload_for(idx: int) -> bytes:  # same as oracle.payload_for
    return b"F" + int(idx).to_bytes(4, "little")


def payload_index(payload) -> int:
    return int.from_bytes(bytes(payload)[1:5], "little")


def wait_until(cond, timeout=5.0):
    t0 = time.time()
    while not cond():
        if time.time() - t0 > timeout:
            raise TimeoutError("reference did not reach the expected state")
        time.sleep(0.001)


def capture_ingest(Distributor, out_dir):
    d = Distributor(free_port(), free_port(), 5, False)  # threads never started
    cases = []
    for n in (0, 1, 9, 10, 11, 15, 37):
        d.frame_index_counter = 0
        while not d.frame_queue.empty():
            d.frame_queue.get_nowait()
        for i in range(n):
            d.add_frame_for_distribution(b"x%d" % i, 1000.0 + i)
        kept = []
        while not d.frame_queue.empty():
            item = d.frame_queue.get_nowait()
            kept.append([item["frame_index"], item["frame"].decode(), item["timestamp"]])
        cases.append({"n_added": n, "kept": kept, "frame_index_counter": d.frame_index_counter})
    d.cleanup()
    with open(os.path.join(out_dir, "ref_ingest.json"), "w") as f:
        json.dump({"source": "distributor.py:173-203", "queue_maxsize": 10, "cases": cases}, f, indent=1)


def make_ops(rng, n_frames, max_jitter):
    """A stream of results arriving out of order (bounded jitter, some frames lost),
    interleaved with display updates and reads like the app's on_draw (webcam_app.py:135-137)."""
    order = list(range(n_frames))
    keyed = sorted(order, key=lambda i: i + rng.uniform(0, max_jitter))
    ops = []
    for idx in keyed:
        if rng.random() < 0.1:  # lost frame (dropped by a worker, worker.py:74-76)
            continue
        ops.append(["recv", idx])
        r = rng.random()
        if r < 0.5:
            ops.append(["update"])
            ops.append(["get"])
        elif r < 0.6:
            ops.append(["get"])
    ops.append(["update"])
    ops.append(["get"])
    return ops


def capture_display(zmq, Distributor, out_dir, name, frame_delay, buffer_size, ops):
    d = Distributor(free_port(), free_port(), frame_delay, True)
    d.frame_buffer_size = buffer_size
    collect_port = d.collect_socket.getsockopt_string(zmq.LAST_ENDPOINT).rsplit(":", 1)[1]
    d.running = True
    d.inverter_thread.start()  # only the collect thread; dispatch stays idle
    ctx = zmq.Context()
    push = ctx.socket(zmq.PUSH)
    push.connect("tcp://127.0.0.1:%s" % collect_port)
    records = []
    for op in ops:
        rec = {"op": op}
        if op[0] == "recv":
            idx = op[1]
            before = len(d.frame_timings)
            push.send_string(str(idx), zmq.SNDMORE)
            push.send_string("4242", zmq.SNDMORE)
            push.send_string(str(1.0 + idx), zmq.SNDMORE)
            push.send_string(str(1.5 + idx), zmq.SNDMORE)
            push.send(payload_for(idx))
            wait_until(lambda: len(d.frame_timings) > before)
            time.sleep(0.001)  # let cleanup_old_frames (called after the log) finish
            wait_until(lambda: d.latest_received_frame >= idx)
        elif op[0] == "update":
            rec["ret"] = bool(d.update_display_frame())
        elif op[0] == "get":
            fd = d.get_frame_to_display()
            rec["ret"] = None if fd is None else payload_index(fd)
        rec["keys"] = sorted(d.received_frames)
        rec["current_display_frame"] = d.current_display_frame
        rec["latest_received_frame"] = d.latest_received_frame
        records.append(rec)
    # one stored entry, to pin the dict layout of distributor.py:271-276
    sample = None
    if d.received_frames:
        k = max(d.received_frames)
        e = d.received_frames[k]
        sample = {"index": k, "process_id": e["process_id"], "start_time": e["start_time"],
                  "end_time": e["end_time"], "frame_data_index": payload_index(e["frame_data"])}
    ev = d.frame_timings[-1]
    d.running = False
    time.sleep(0.05)
    push.close(0)
    ctx.term()
    d.enable_trace_export = False
    d.cleanup()
    with open(os.path.join(out_dir, "ref_display_%s.json" % name), "w") as f:
        json.dump({"source": "distributor.py:253-344", "frame_delay": frame_delay,
                   "frame_buffer_size": buffer_size, "ops": ops, "records": records,
                   "stored_entry": sample,
                   "trace_event": {k: ev[k] for k in ("frame_index", "begin_time", "end_time",
                                                       "event_type", "event_ph", "pid")}}, f, indent=1)


def capture_dispatch(zmq, Distributor, out_dir):
    d = Distributor(free_port(), free_port(), 5, False)
    dist_port = d.distribute_socket.getsockopt_string(zmq.LAST_ENDPOINT).rsplit(":", 1)[1]
    d.start()
    ctx = zmq.Context()
    dealer = ctx.socket(zmq.DEALER)
    dealer.connect("tcp://127.0.0.1:%s" % dist_port)
    time.sleep(0.2)
    steps = []

    def ready(label):
        dealer.send_string("READY")
        if dealer.poll(300):
            parts = dealer.recv_multipart()
            steps.append({"step": label, "reply": [parts[0].decode(), parts[1].decode()],
                          "n_parts": len(parts)})
        else:
            steps.append({"step": label, "reply": None})

    def add(i):
        d.add_frame_for_distribution(b"frame-%d" % i, 2000.0 + i)
        time.sleep(0.1)  # dispatch loop moves it into the current slot (<= 10 ms poll)

    ready("ready-before-any-frame")
    add(0)
    ready("ready-after-frame-0")
    ready("ready-again-no-new-frame")
    for i in (1, 2, 3):  # one frame per dispatch iteration: the slot ends at the newest
        add(i)
    ready("ready-after-frames-1-2-3")
    add(4)
    add(5)
    ready("ready-after-frames-4-5")
    ready("ready-again-no-new-frame-2")
    d.stop()
    time.sleep(0.05)
    dealer.close(0)
    ctx.term()
    d.cleanup()
    with open(os.path.join(out_dir, "ref_dispatch.json"), "w") as f:
        json.dump({"source": "distributor.py:205-251", "steps": steps}, f, indent=1)


def capture_worker(zmq, Distributor, Worker, out_dir):
    class ByteInverter(Worker):  # the reference's plugin extension point (worker.py:78-80)
        def __call__(self, frame_bytes):
            return np.bitwise_not(np.frombuffer(frame_bytes, dtype=np.uint8)).tobytes()

    dport, cport = free_port(), free_port()
    d = Distributor(dport, cport, 0, True)
    d.start()
    w = ByteInverter("127.0.0.1", dport, cport)
    t = threading.Thread(target=w.start, daemon=True)
    t.start()
    frames = []
    shapes = [(4, 4), (17, 13), (1, 1), (16, 16)]
    for k, (h, wd) in enumerate(shapes):
        frm = np.random.default_rng(100 + k).integers(0, 256, (h, wd, 3), dtype=np.uint8)
        before = len(d.received_frames) + len([e for e in d.frame_timings if e["event_ph"] == "X"])
        idx = d.frame_index_counter
        d.add_frame_for_distribution(frm.tobytes(), 3000.0 + k)
        wait_until(lambda: idx in d.received_frames, timeout=10)
        e = d.received_frames[idx]
        frames.append({"index": idx, "shape": [h, wd, 3], "seed": 100 + k,
                       "input_hex": frm.tobytes().hex(), "output_hex": bytes(e["frame_data"]).hex(),
                       "process_id_is_worker_pid": e["process_id"] == str(os.getpid()),
                       "start_le_end": e["start_time"] <= e["end_time"]})
    w.running = False
    d.stop()
    time.sleep(0.1)
    d.enable_trace_export = False
    d.cleanup()
    with open(os.path.join(out_dir, "ref_worker.json"), "w") as f:
        json.dump({"source": "worker.py:30-76 + distributor.py:205-289", "frames": frames}, f, indent=1)


def main():
    ref_dir, out_dir = sys.argv[1], sys.argv[2]
    sys.path.insert(0, ref_dir)
    import zmq  # noqa: E402
    from distributor import Distributor  # noqa: E402
    from worker import Worker  # noqa: E402

    capture_ingest(Distributor, out_dir)
    rng = random.Random(20250718)
    for name, fd, bs, n, jit in (("d5_b50", 5, 50, 120, 6.0), ("d0_b50", 0, 50, 60, 3.0),
                                 ("d3_b8", 3, 8, 80, 12.0), ("d5_b50_inorder", 5, 50, 30, 0.0)):
        capture_display(zmq, Distributor, out_dir, name, fd, bs, make_ops(rng, n, jit))
    capture_dispatch(zmq, Distributor, out_dir)
    capture_worker(zmq, Distributor, Worker, out_dir)
    print("captured into", out_dir)


if __name__ == "__main__":
    main()
