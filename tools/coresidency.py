#!/usr/bin/env python3
"""Experiment: does a kernel on a later stream run beside a slab fill that waits on its halo?

Runs tests/test_coresidency_gpu.run_coresidency with the engine's stream at the device's
greatest priority (the default) and at normal priority (GA_STREAM_PRIORITY=normal), with
more torch streams than GPU_MAX_HW_QUEUES, and prints one JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.test_coresidency_gpu import oracle_cost, run_coresidency  # noqa: E402

for prio in ("high", "normal"):
    for nstreams in (2, 8, 16):
        if prio == "normal":
            os.environ["GA_STREAM_PRIORITY"] = "normal"
        else:
            os.environ.pop("GA_STREAM_PRIORITY", None)
        r = run_coresidency(nstreams=nstreams, deadline_s=5.0)
        r["cost_ok"] = r["cost"] == oracle_cost(*r.pop("seqs"))
        print(json.dumps(dict(priority_mode=prio, nstreams=nstreams, GPU_MAX_HW_QUEUES=os.environ.get("GPU_MAX_HW_QUEUES"),
                              **r)), flush=True)
