#!/usr/bin/env python3
"""``python -m vfilter.inverter`` with tools/sampler.py running; the report goes to
$VF_SAMPLER_OUT.<pid> when the worker exits (tools/pipeline_bench.py --profile)."""
import atexit
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sampler import Sampler  # noqa: E402

_out = os.environ.get("VF_SAMPLER_OUT", "/tmp/vf_sampler")
_err = open(f"{_out}.{os.getpid()}.stderr", "w")  # the library's VF_JPEG_TRACE lines land here
os.dup2(_err.fileno(), 2)
s = Sampler().start()


@atexit.register
def _dump():
    out = os.environ.get("VF_SAMPLER_OUT", "/tmp/vf_sampler")
    with open(f"{out}.{os.getpid()}", "w") as f:
        f.write(s.report(60) + "\n")


from vfilter.inverter import main  # noqa: E402

if os.environ.get("VF_CPROFILE"):  # deterministic per-function profile of the worker's main thread
    import cProfile
    import pstats
    prof = cProfile.Profile()
    try:
        rc = prof.runcall(main, sys.argv[1:])
    finally:
        with open(f"{_out}.{os.getpid()}.cprofile", "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(35)
    sys.exit(rc)
sys.exit(main(sys.argv[1:]))
