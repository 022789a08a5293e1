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

sys.exit(main(sys.argv[1:]))
