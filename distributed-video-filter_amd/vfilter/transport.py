"""Message transport between distributor and workers.

The reference uses ZeroMQ over TCP: the distributor binds a ROUTER (dispatch,
distributor.py:30-31) and a PULL (collect, :34-35); each worker connects a DEALER
(worker.py:20-21) and a PUSH (:24-25).  Two interchangeable implementations of those four
roles live here:

  "zmq"  pyzmq, exactly the reference's sockets and multipart framing, so this build's
         distributor and workers interoperate with the reference's (needs pyzmq; on this
         image only /opt/conda/bin/python3.9 has it);
  "tcp"  stdlib sockets with the same roles and semantics (multipart messages; ROUTER
         prefixes the peer identity; DEALER/PUSH connect lazily and retry), for
         interpreters without pyzmq — e.g. the GPU box's main python3.

Large frames should not ride either of them between processes of one node: see
``shm.FrameRing`` (frames in a page-locked shared-memory ring, only indices on the wire).

Wire framing of "tcp": message = u32 nparts, then per part u64 length + bytes (little endian).
"""
from __future__ import annotations

import collections
import itertools
import os
import select
import selectors
import socket
import struct
import threading
import time
from typing import List, Optional, Sequence, Tuple

_HDR = struct.Struct("<I")
_LEN = struct.Struct("<Q")


def zmq_available() -> bool:
    try:
        import zmq  # noqa: F401
        return True
    except Exception:
        return False


def resolve(kind: str) -> str:
    if kind == "auto":
        return "zmq" if zmq_available() else "tcp"
    if kind not in ("zmq", "tcp"):
        raise ValueError(f"unknown transport {kind!r} (zmq | tcp | auto)")
    return kind


# ---------------------------------------------------------------------------------------
# stdlib TCP implementation
# ---------------------------------------------------------------------------------------

def _recv_exact(sock: socket.socket, n: int, alloc=None):
    """n bytes from ``sock``: into a new bytearray, or into ``alloc(n)`` (a writable buffer the
    caller provides, e.g. a pinned arena array the GPU reads directly)."""
    buf = alloc(n) if alloc is not None else bytearray(n)
    view = memoryview(buf).cast("B")
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed")
        got += k
    return buf


# what a reader accepts before it allocates anything: a peer's length field is never trusted
# (a u64 of 2^62 is a MemoryError, 2^63 an OverflowError in bytearray())
MAX_PARTS = 1 << 16
MAX_PART = int(os.environ.get("VF_TCP_MAX_PART", str(1 << 30)))


def _check_nparts(nparts: int) -> None:
    if nparts > MAX_PARTS:
        raise ValueError(f"malformed message: {nparts} parts (at most {MAX_PARTS})")


def _check_len(n: int, cap: int) -> None:
    if n > cap:
        raise ValueError(f"malformed message: a part of {n} B (at most {cap})")


def _recv_msg(sock: socket.socket, alloc=None, max_part: int = MAX_PART) -> List[bytes]:
    (nparts,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    _check_nparts(nparts)
    parts = []
    for _ in range(nparts):
        (n,) = _LEN.unpack(_recv_exact(sock, _LEN.size))
        _check_len(n, max_part)
        parts.append(bytes(_recv_exact(sock, n)) if n < (1 << 16) else _recv_exact(sock, n, alloc))
    return parts


def _send_msg(sock: socket.socket, parts: Sequence) -> None:
    bufs = [_HDR.pack(len(parts))]
    for p in parts:
        mv = memoryview(p).cast("B") if not isinstance(p, (bytes, bytearray)) else p
        bufs.append(_LEN.pack(len(mv)))
        bufs.append(mv)
    # gather-write; sendmsg may send partially, so finish with sendall on the remainder
    total = sum(len(b) for b in bufs)
    sent = sock.sendmsg(bufs)
    if sent < total:
        for b in bufs:
            if sent >= len(b):
                sent -= len(b)
                continue
            sock.sendall(memoryview(b)[sent:])
            sent = 0


class _RecvState:
    """One peer's message being received by the select loop: u32 nparts, then per part u64
    length + bytes, read as far as the socket has data (MSG_DONTWAIT per call, so the socket
    itself stays blocking for the senders on other threads)."""

    def __init__(self, pid: bytes, conn: socket.socket, max_part: int = MAX_PART):
        self.pid, self.conn, self.max_part = pid, conn, max_part
        self._start(_HDR.size, "hdr")

    def _start(self, n: int, stage: str) -> None:
        self.stage, self.buf, self.got = stage, bytearray(n), 0

    def feed(self) -> List[List[bytes]]:
        """Read what is available; returns the messages completed (raises on disconnect)."""
        done = []
        while True:
            n = len(self.buf)
            if self.got < n:
                try:
                    k = self.conn.recv_into(memoryview(self.buf)[self.got:], n - self.got, socket.MSG_DONTWAIT)
                except (BlockingIOError, InterruptedError):
                    return done
                if k == 0:
                    raise ConnectionError("peer closed")
                self.got += k
                if self.got < n:
                    continue
            if self.stage == "hdr":
                (self.nparts,) = _HDR.unpack(self.buf)
                _check_nparts(self.nparts)
                self.parts = []
                if self.nparts == 0:
                    done.append(self.parts)
                    self._start(_HDR.size, "hdr")
                else:
                    self._start(_LEN.size, "len")
            elif self.stage == "len":
                (m,) = _LEN.unpack(self.buf)
                _check_len(m, self.max_part)
                self._start(m, "part")
                if m == 0:
                    continue
            else:
                self.parts.append(bytes(self.buf) if len(self.buf) < (1 << 16) else self.buf)
                if len(self.parts) == self.nparts:
                    done.append(self.parts)
                    self._start(_HDR.size, "hdr")
                else:
                    self._start(_LEN.size, "len")


# VF_TCP_READER=thread (default): one reader thread per peer connection.  "select": one thread
# per listener accepts and reads every peer, so N workers' messages are handled by one thread
# instead of N contending for the GIL and the distributor's lock -- 8 echo workers with JPEG-size
# frames 102-104 k fps against 70-95 k, the JPEG system leg 41.1-41.5 k against 38.0-41.1 k
# (profiles/r04_reader_ab.txt).  Safe with payload dispatches since round 5: the distributor
# sends outside its lock, so a handler blocked in a large send to a worker that is itself busy
# sending results no longer holds what the result reader needs (the round-4 hang of
# test_configs3_mixed_resolution_pull_tcp_payloads; tests/test_plumbing.py covers both readers).
_READER = os.environ.get("VF_TCP_READER", "thread")


def _bind_addr(host: str) -> str:
    return "0.0.0.0" if host in ("*", "", None) else host


# VF_TCP_UNIX=1: same-host peers skip the TCP stack.  A listener also answers on the abstract
# Unix socket "\0vfd-tcp-<port>" (the native engine's listeners always do, csrc/vf_dist.cc), and a
# connecting side whose host is 127.0.0.1 / localhost tries it before TCP.  Same framing, same
# roles.  Not the default: a Unix socket buffers ~200 KB where loopback TCP autotunes to MBs, so a
# sender of large socket payloads blocks sooner (harmless to the distributor, which never sends
# under its lock, but a behaviour change for payload deployments).
_UNIX = os.environ.get("VF_TCP_UNIX", "0") == "1" and hasattr(socket, "AF_UNIX")


def _unix_name(port: int) -> str:
    return f"\0vfd-tcp-{port}"


def _nodelay(conn: socket.socket) -> None:
    if conn.family != getattr(socket, "AF_UNIX", None):
        conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)


class _Listener:
    """Accepts peers; every message from any peer lands in one queue as (peer_id, parts).
    ``poll`` sleeps on a condition the readers (and ``wake``) notify: it returns the moment a
    message lands, and an idle poll costs no GIL hand-offs (round 3 slept in 0.2 ms steps,
    and every step took the GIL from the distributor's other threads)."""

    def __init__(self, host: str, port: int):
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((_bind_addr(host), port))
        self.sock.listen(64)
        self.port = self.sock.getsockname()[1]
        self.usock = None
        if _UNIX:
            try:
                u = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                u.bind(_unix_name(self.port))
                u.listen(64)
                self.usock = u
            except OSError:  # the name is taken: TCP only
                self.usock = None
        self.inbox: "collections.deque[Tuple[bytes, Optional[List[bytes]]]]" = collections.deque()
        self._cond = threading.Condition(threading.Lock())
        self._woken = False
        # set_handler: messages are handled on the peer's reader thread as they arrive, instead
        # of queued for a polling thread (one thread hand-off less per message)
        self.handler = None
        self.max_part = MAX_PART  # largest part a peer may announce (the distributor lowers it)
        self.peers = {}
        self._ids = itertools.count(1)
        self._lock = threading.Lock()
        self._closed = False
        if _READER == "thread":
            threading.Thread(target=self._accept_loop, args=(self.sock,), daemon=True).start()
            if self.usock is not None:
                threading.Thread(target=self._accept_loop, args=(self.usock,), daemon=True).start()
        else:
            threading.Thread(target=self._select_loop, daemon=True, name="tcp-select").start()

    def _select_loop(self):
        sel = selectors.DefaultSelector()
        try:
            sel.register(self.sock, selectors.EVENT_READ, None)
            if self.usock is not None:
                sel.register(self.usock, selectors.EVENT_READ, None)
        except (ValueError, OSError):  # closed before this thread started
            sel.close()
            return
        try:
            while not self._closed:
                try:
                    events = sel.select(timeout=0.5)
                except (ValueError, OSError):
                    return
                for key, _ in events:
                    st = key.data
                    if st is None:  # a listening socket: a new peer
                        try:
                            conn, _ = key.fileobj.accept()
                        except OSError:
                            if self._closed:
                                return
                            continue
                        _nodelay(conn)
                        pid = b"\x00" + next(self._ids).to_bytes(4, "big")
                        with self._lock:
                            self.peers[pid] = (conn, threading.Lock())
                        sel.register(conn, selectors.EVENT_READ, _RecvState(pid, conn, self.max_part))
                        continue
                    try:
                        msgs = st.feed()
                    except (ConnectionError, OSError):
                        msgs = None  # closed
                    except Exception as e:  # a malformed frame: drop that peer, keep serving the others
                        print(f"transport: dropping peer {st.pid.hex()}: {type(e).__name__}: {e}")
                        msgs = None
                    for msg in msgs or ():
                        h = self.handler
                        if h is not None:
                            h(st.pid, msg)
                        else:
                            self._put((st.pid, msg))
                    if msgs is None:
                        try:
                            sel.unregister(st.conn)
                        except (KeyError, ValueError, OSError):
                            pass
                        self._gone(st.pid, st.conn)
        finally:
            sel.close()

    def _gone(self, pid, conn):
        with self._lock:
            self.peers.pop(pid, None)
        try:
            conn.close()
        except OSError:
            pass
        if not self._closed:
            h = self.handler
            if h is not None:
                h(pid, None)
            else:
                self._put((pid, None))  # disconnect notice (ZeroMQ gives none; see RouterEnd.recv)

    def _accept_loop(self, lsock):
        while not self._closed:
            try:
                conn, _ = lsock.accept()
            except OSError:
                return
            _nodelay(conn)
            pid = b"\x00" + next(self._ids).to_bytes(4, "big")  # ZeroMQ-style 5-byte identity
            with self._lock:
                self.peers[pid] = (conn, threading.Lock())
            threading.Thread(target=self._read_loop, args=(pid, conn), daemon=True).start()

    def _read_loop(self, pid, conn):
        try:
            while not self._closed:
                msg = _recv_msg(conn, max_part=self.max_part)
                h = self.handler
                if h is not None:
                    h(pid, msg)
                else:
                    self._put((pid, msg))
        except (ConnectionError, OSError):
            pass
        except Exception as e:  # a malformed frame (absurd length or part count): drop this peer
            print(f"transport: dropping peer {pid.hex()}: {type(e).__name__}: {e}")
        finally:
            self._gone(pid, conn)

    def _put(self, item) -> None:
        with self._cond:
            self.inbox.append(item)
            self._cond.notify()

    def wake(self) -> None:
        """End the current (or the next) ``poll`` early, e.g. because frames were committed for
        a worker waiting on its credit."""
        with self._cond:
            self._woken = True
            self._cond.notify()

    def poll(self, timeout_ms: float) -> bool:
        """True when a message is waiting; returns at the first message, ``wake`` or timeout."""
        if self.inbox:
            return True
        with self._cond:
            if not self.inbox and not self._woken and timeout_ms > 0:
                self._cond.wait(timeout_ms / 1000.0)
            self._woken = False
            return bool(self.inbox)

    def recv(self, timeout_ms: Optional[int] = None):
        with self._cond:
            if not self.inbox and timeout_ms != 0:
                self._cond.wait_for(lambda: self.inbox, None if timeout_ms is None else timeout_ms / 1000.0)
            return self.inbox.popleft() if self.inbox else None

    def send_to(self, pid: bytes, parts: Sequence) -> bool:
        with self._lock:
            ent = self.peers.get(pid)
        if ent is None:
            return False  # ROUTER drops messages to unknown peers
        conn, lk = ent
        with lk:
            try:
                _send_msg(conn, parts)
                return True
            except OSError:
                return False

    def close(self):
        self._closed = True
        for ls in (self.sock, self.usock):
            if ls is None:
                continue
            try:
                ls.shutdown(socket.SHUT_RDWR)  # wakes a thread blocked in accept
            except OSError:
                pass
            try:
                ls.close()
            except OSError:
                pass
        with self._lock:
            for conn, _ in self.peers.values():
                try:
                    conn.close()
                except OSError:
                    pass
            self.peers.clear()


class _Connection:
    """Connecting side (DEALER / PUSH): connects lazily, retrying until the peer binds."""

    def __init__(self, host: str, port: int, connect_timeout: float = 30.0):
        self.addr = ("127.0.0.1" if host in ("localhost", "*") else host, port)
        self.connect_timeout = connect_timeout
        self.sock: Optional[socket.socket] = None
        self._lock = threading.Lock()

    def _ensure(self):
        if self.sock is not None:
            return
        deadline = time.monotonic() + self.connect_timeout
        while True:
            if _UNIX and self.addr[0] in ("127.0.0.1", "localhost"):
                u = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                try:
                    u.connect(_unix_name(self.addr[1]))
                    self.sock = u
                    return
                except OSError:  # no such listener on this host: TCP
                    u.close()
            try:
                s = socket.create_connection(self.addr, timeout=2.0)
                s.settimeout(None)
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                self.sock = s
                return
            except OSError:
                if time.monotonic() > deadline:
                    raise
                time.sleep(0.05)

    def send(self, parts: Sequence) -> None:
        with self._lock:
            self._ensure()
            _send_msg(self.sock, parts)

    def poll(self, timeout_ms: int) -> bool:
        self._ensure()
        r, _, _ = select.select([self.sock], [], [], timeout_ms / 1000.0)
        return bool(r)

    def recv(self, alloc=None) -> List[bytes]:
        self._ensure()
        return _recv_msg(self.sock, alloc)

    def close(self):
        if self.sock is not None:
            try:
                self.sock.close()
            except OSError:
                pass
            self.sock = None


# ---------------------------------------------------------------------------------------
# role objects used by the distributor and the worker
# ---------------------------------------------------------------------------------------

def _zmq_ms(timeout_ms: float) -> int:
    """zmq_poll takes whole milliseconds: a sub-millisecond wait (the runtime's short polls while
    batches are in flight) becomes 1 ms there instead of 0, which would spin."""
    return 0 if timeout_ms <= 0 else max(1, int(-(-timeout_ms // 1)))


class RouterEnd:
    """Distributor dispatch socket (reference: ROUTER bind, distributor.py:30-31)."""

    def __init__(self, kind: str, host: str, port: int, ctx=None):
        self.kind = resolve(kind)
        if self.kind == "zmq":
            import zmq
            self._zmq = zmq
            self.sock = ctx.socket(zmq.ROUTER)
            self.sock.bind(f"tcp://{host if host not in ('localhost',) else '127.0.0.1'}:{port}")
            self.port = int(self.sock.getsockopt_string(zmq.LAST_ENDPOINT).rsplit(":", 1)[1])
        else:
            self.sock = _Listener(host, port)
            self.port = self.sock.port

    def poll(self, timeout_ms: float) -> bool:
        return bool(self.sock.poll(_zmq_ms(timeout_ms) if self.kind == "zmq" else timeout_ms))

    def wake(self) -> None:
        """"tcp": end the dispatch thread's poll now (frames were committed).  "zmq": nothing
        (its polls are short: ``wakeable`` is False)."""
        if self.kind != "zmq":
            self.sock.wake()

    @property
    def wakeable(self) -> bool:
        return self.kind != "zmq"

    def set_handler(self, fn) -> bool:
        """"tcp": call fn(peer, parts) on the peer's reader thread for every message (parts None:
        the peer disconnected) instead of queueing it for ``poll`` / ``recv``.  False for "zmq"."""
        if self.kind == "zmq":
            return False
        self.sock.handler = fn
        return True

    def recv(self) -> Tuple[bytes, Optional[List[bytes]]]:
        """(peer, parts); parts is None when "tcp" saw the peer disconnect (the distributor
        then re-queues that worker's frames at once instead of waiting for their deadline)."""
        if self.kind == "zmq":
            parts = self.sock.recv_multipart(self._zmq.NOBLOCK)
            return parts[0], parts[1:]
        got = self.sock.recv(0)
        if got is None:
            raise BlockingIOError
        return got

    def send(self, peer: bytes, parts: Sequence) -> bool:
        if self.kind == "zmq":
            self.sock.send_multipart([peer] + list(parts), copy=False)
            return True
        return self.sock.send_to(peer, parts)

    def close(self):
        self.sock.close()


class PullEnd:
    """Distributor collect socket (reference: PULL bind, distributor.py:34-35)."""

    def __init__(self, kind: str, host: str, port: int, ctx=None):
        self.kind = resolve(kind)
        if self.kind == "zmq":
            import zmq
            self._zmq = zmq
            self.sock = ctx.socket(zmq.PULL)
            self.sock.bind(f"tcp://{host if host not in ('localhost',) else '127.0.0.1'}:{port}")
            self.port = int(self.sock.getsockopt_string(zmq.LAST_ENDPOINT).rsplit(":", 1)[1])
        else:
            self.sock = _Listener(host, port)
            self.port = self.sock.port

    def poll(self, timeout_ms: float) -> bool:
        return bool(self.sock.poll(_zmq_ms(timeout_ms) if self.kind == "zmq" else timeout_ms))

    def recv(self) -> List[bytes]:
        if self.kind == "zmq":
            return self.sock.recv_multipart(self._zmq.NOBLOCK)
        got = self.sock.recv(0)
        if got is None or got[1] is None:  # nothing, or a PUSH peer's disconnect notice
            raise BlockingIOError
        return got[1]

    def set_handler(self, fn) -> bool:
        """"tcp": call fn(parts) on the peer's reader thread for every result message."""
        if self.kind == "zmq":
            return False
        self.sock.handler = lambda pid, parts: None if parts is None else fn(parts)
        return True

    def close(self):
        self.sock.close()


class DealerEnd:
    """Worker request socket (reference: DEALER connect, worker.py:20-21)."""

    def __init__(self, kind: str, host: str, port: int, ctx=None):
        self.kind = resolve(kind)
        if self.kind == "zmq":
            import zmq
            self._zmq = zmq
            self.sock = ctx.socket(zmq.DEALER)
            self.sock.connect(f"tcp://{host}:{port}")
        else:
            self.sock = _Connection(host, port)
        # "tcp": parts of 64 KiB or more are received into recv_alloc(n) when it is set (a GPU
        # worker gives its pinned arena, so a received frame is a source the kernel reads in place)
        self.recv_alloc = None

    def send(self, parts: Sequence) -> None:
        if self.kind == "zmq":
            self.sock.send_multipart(list(parts), self._zmq.NOBLOCK)
        else:
            self.sock.send(parts)

    def poll(self, timeout_ms: float) -> bool:
        return bool(self.sock.poll(_zmq_ms(timeout_ms) if self.kind == "zmq" else timeout_ms))

    def recv(self) -> List[bytes]:
        if self.kind == "zmq":
            return self.sock.recv_multipart(self._zmq.NOBLOCK)
        return self.sock.recv(self.recv_alloc)

    def close(self):
        self.sock.close(0) if self.kind == "zmq" else self.sock.close()


class PushEnd:
    """Worker result socket (reference: PUSH connect, worker.py:24-25)."""

    def __init__(self, kind: str, host: str, port: int, ctx=None):
        self.kind = resolve(kind)
        if self.kind == "zmq":
            import zmq
            self._zmq = zmq
            self.sock = ctx.socket(zmq.PUSH)
            self.sock.connect(f"tcp://{host}:{port}")
        else:
            self.sock = _Connection(host, port)

    def send(self, parts: Sequence) -> None:
        if self.kind == "zmq":
            self.sock.send_multipart(list(parts), self._zmq.NOBLOCK, copy=False)
        else:
            self.sock.send(parts)

    def close(self):
        self.sock.close(0) if self.kind == "zmq" else self.sock.close()


def make_context(kind: str):
    """A zmq.Context for the "zmq" transport, else None."""
    if resolve(kind) == "zmq":
        import zmq
        return zmq.Context()
    return None
