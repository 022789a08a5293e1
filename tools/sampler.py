"""A tiny sampling profiler for the plumbing (tools only): every ~0.5 ms, each thread's
innermost vfilter frame and its innermost frame; a report of the top entries per thread.
  from sampler import Sampler; s = Sampler(); s.start(); ...; print(s.report())"""
import os
import sys
import threading
import time
import traceback


class Sampler:
    def __init__(self, period=0.0005, match=("vfilter", "tools")):
        self.period, self.match = period, match
        self.samples = {}
        self._stop = threading.Event()
        self._names = {}

    def _run(self):
        me = threading.get_ident()
        while not self._stop.is_set():
            for tid, fr in sys._current_frames().items():
                if tid == me:
                    continue
                name = self._names.get(tid)
                if name is None:
                    name = next((t.name for t in threading.enumerate() if t.ident == tid), str(tid))
                    self._names[tid] = name
                st = traceback.extract_stack(fr)
                key = next((f"{os.path.basename(f.filename)}:{f.lineno} {f.name}" for f in reversed(st)
                            if any(m in f.filename for m in self.match)), None)
                inner = f"{os.path.basename(st[-1].filename)}:{st[-1].lineno} {st[-1].name}"
                k = (name, key, inner)
                self.samples[k] = self.samples.get(k, 0) + 1
            time.sleep(self.period)

    def start(self):
        threading.Thread(target=self._run, daemon=True, name="sampler").start()
        return self

    def clear(self):
        self.samples.clear()

    def stop(self):
        self._stop.set()

    def report(self, top=40):
        tot = {}
        for (th, _, _), c in self.samples.items():
            tot[th] = tot.get(th, 0) + c
        lines = []
        for (th, key, inner), c in sorted(self.samples.items(), key=lambda kv: -kv[1])[:top]:
            lines.append(f"{100 * c / tot[th]:5.1f}%  {th:22s} {key}  <- {inner}")
        return "\n".join(lines)
