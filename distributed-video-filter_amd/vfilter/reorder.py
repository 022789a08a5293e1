"""Reassembly of results that come back from workers out of order.

``DisplayBuffer``  the reference's policy, unchanged (distributor.py:253-344): keep results
                   by index, drop indices below the display index and cap at the newest
                   ``frame_buffer_size``; the display index trails the newest result by
                   ``frame_delay``; a missing frame is replaced by the nearest index.  Lossy by
                   design (a live view).  Checked op-for-op against traces of the real
                   reference (tests/golden/ref_display_*.json).
``OrderedBuffer``  lossless in-order release for batch pipelines (BASELINE configs[2]/[3]):
                   every index is released exactly once, in index order; it measures the
                   ordering overhead (how long a result waits for its predecessors, and how
                   deep the buffer gets).

Neither holds a lock; the distributor serialises access.
"""
from __future__ import annotations

import heapq
import time
from typing import Any, Dict, List, Optional, Tuple


class DisplayBuffer:
    def __init__(self, frame_delay: int = 5, frame_buffer_size: int = 50):
        self.received_frames: Dict[int, dict] = {}
        self.current_display_frame = 0          # distributor.py:21
        self.latest_received_frame = -1         # distributor.py:22
        self.frame_buffer_size = frame_buffer_size  # distributor.py:23
        self.frame_delay = frame_delay          # distributor.py:24

    def receive(self, frame_index: int, frame_data: Any, process_id: str, start_time: float,
                end_time: float) -> None:
        """Store one result (distributor.py:270-282)."""
        self.received_frames[frame_index] = {"frame_data": frame_data, "process_id": process_id,
                                             "start_time": float(start_time), "end_time": float(end_time)}
        if frame_index > self.latest_received_frame:
            self.latest_received_frame = frame_index
        self.cleanup_old_frames()

    def cleanup_old_frames(self) -> None:
        """distributor.py:291-307."""
        cur = self.current_display_frame
        stale = [i for i in self.received_frames if i < cur]
        for i in stale:
            del self.received_frames[i]
        excess = len(self.received_frames) - self.frame_buffer_size
        if excess > 0:
            for i in sorted(self.received_frames)[:excess]:
                del self.received_frames[i]

    def get_frame_to_display(self):
        """distributor.py:309-322 (ties between two nearest indices go to the lower one)."""
        target = self.current_display_frame
        hit = self.received_frames.get(target)
        if hit is not None:
            return hit["frame_data"]
        if not self.received_frames:
            return None
        best = min(self.received_frames, key=lambda i: (abs(i - target), i))
        return self.received_frames[best]["frame_data"]

    def update_display_frame(self) -> bool:
        """distributor.py:324-344."""
        latest = self.latest_received_frame
        if latest >= self.frame_delay:
            self.current_display_frame = latest - self.frame_delay
            return True
        if latest > 0 and self.current_display_frame < latest:
            self.current_display_frame = latest
            return True
        return False

    def __len__(self) -> int:
        return len(self.received_frames)


class OrderedBuffer:
    """Release results strictly in index order, each exactly once.

    ``push`` stores a result (or marks an index lost); ``pop_ready`` returns every result
    whose predecessors have all been released.  Ordering overhead = per-result time between
    arrival and release, plus the buffer's depth.
    """

    def __init__(self, first_index: int = 0):
        self.next_index = first_index
        self._heap: List[Tuple[int, float]] = []
        self._items: Dict[int, Tuple[Any, dict]] = {}
        self._lost = set()
        self.released = 0
        self.lost_count = 0
        self.max_depth = 0
        self.wait_total = 0.0
        self.wait_max = 0.0
        self.out_of_order = 0  # results that arrived while a predecessor was missing

    def push(self, index: int, data: Any, info: Optional[dict] = None, now: Optional[float] = None) -> None:
        if index < self.next_index or index in self._items:
            return  # duplicate or already skipped
        t = time.monotonic() if now is None else now
        self._items[index] = (data, info or {})
        heapq.heappush(self._heap, (index, t))
        if index != self.next_index:
            self.out_of_order += 1
        if len(self._items) > self.max_depth:
            self.max_depth = len(self._items)

    def mark_lost(self, index: int) -> None:
        if index >= self.next_index and index not in self._items:
            self._lost.add(index)

    def pop_ready(self, now: Optional[float] = None) -> List[Tuple[int, Any, dict]]:
        t = time.monotonic() if now is None else now
        out = []
        while True:
            if self.next_index in self._lost:
                self._lost.discard(self.next_index)
                self.lost_count += 1
                self.next_index += 1
                continue
            if not self._heap or self._heap[0][0] != self.next_index:
                break
            idx, t_in = heapq.heappop(self._heap)
            data, info = self._items.pop(idx)
            w = t - t_in
            self.wait_total += w
            if w > self.wait_max:
                self.wait_max = w
            self.released += 1
            self.next_index += 1
            out.append((idx, data, info))
        return out

    def __len__(self) -> int:
        return len(self._items)

    def stats(self) -> dict:
        return {"released": self.released, "lost": self.lost_count, "buffered": len(self._items),
                "max_depth": self.max_depth, "out_of_order": self.out_of_order,
                "reorder_wait_mean_ms": 1e3 * self.wait_total / self.released if self.released else 0.0,
                "reorder_wait_max_ms": 1e3 * self.wait_max, "next_index": self.next_index}
