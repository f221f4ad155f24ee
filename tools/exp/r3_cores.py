"""Round 3: which kernels run beside a waiting lane slab fill, by the fill's workgroup count
(tests/test_coresidency_gpu.py at growing occupancy).  python tools/exp/r3_cores.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("GA_LANE_COLS_PER_LANE", "2")
os.environ.setdefault("GA_FILL_NWC", "4")
os.environ.setdefault("GA_FILL_MODE", "lane")
from tests.test_coresidency_gpu import run_coresidency  # noqa: E402

cfgs = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or [(64, 1), (200, 1), (240, 1), (245, 0)]
for wgs, heavy in cfgs:
    r = run_coresidency(m=20_000, n=2048 + wgs * 512, split=2048, heavy=0 if heavy else None, deadline_s=3.0)
    print(f"wgs {wgs:3d} heavy {heavy!s:5} done {r['all_done_while_waiting']!s:5} waited {r['waited_s']:.3f}s "
          f"still_waiting {r['fill_still_waiting']} halo_ok {r['halo_ok']} kind {r['kind']} prio {r['priority']}",
          flush=True)
