"""Frame-index sharding across GPUs.

Frames are independent (inverter.py:29-46 keeps no cross-frame state), so the path
partitions by frame index with no collective.  Two layouts, both deterministic:

  batch round-robin   global batch b = frames [b*B, (b+1)*B) goes to rank b % N; step s of
                      rank r processes global batch s*N + r (used by bench.py: each rank's
                      batches stay contiguous, one launch each).
  chunk round-robin   index i goes to shard (i // chunk) % N (Distributor policy="shard").

The reference gives each frame to whichever worker asked first (distributor.py:229-241);
with uniform work per frame both layouts give every GPU the same load without that
round trip, and the in-order reassembly is host-side (``reorder.OrderedBuffer``).
"""
from __future__ import annotations

from typing import List


def batch_of_step(step: int, rank: int, world: int) -> int:
    """Global batch id processed by ``rank`` at ``step``."""
    return step * world + rank


def batch_frames(batch_id: int, batch: int) -> range:
    return range(batch_id * batch, (batch_id + 1) * batch)


def rank_frames(rank: int, world: int, steps: int, batch: int) -> List[int]:
    """Every frame index ``rank`` processes in ``steps`` steps."""
    out: List[int] = []
    for s in range(steps):
        out.extend(batch_frames(batch_of_step(s, rank, world), batch))
    return out


def chunk_owner(index: int, chunk: int, nshards: int) -> int:
    """Shard of frame ``index`` under chunk round-robin."""
    return (index // chunk) % nshards


def synthetic_seed(index: int, distinct: int = 97) -> int:
    """Seed of the synthetic frame with global index ``index`` (a small prime number of
    distinct frames keeps generation cheap while neighbouring frames differ)."""
    return index % distinct
