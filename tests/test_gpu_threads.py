"""GPU: launch code entered concurrently by several host threads (loopback ranks, one planner per thread).

The racing must happen on each kernel's FIRST launch in the process (its once-per-kernel LDS attribute, the
per-device CU count, the occupancy cache), so it runs in a fresh child process (tests/_race_first_launch.py):
4 threads, MLP steps over a 4-rank loopback communicator and independent f16 U-Net samplers, all released
together by a barrier; results must equal a single planner's."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_first_launches_racing_from_four_threads():
    r = subprocess.run([sys.executable, os.path.join(HERE, "_race_first_launch.py")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-2000:] + r.stderr[-4000:]
