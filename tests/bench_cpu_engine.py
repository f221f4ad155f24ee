"""CPU slab engine for rehearsing ``bench.py --gpus N`` without GPUs (TEST INFRASTRUCTURE ONLY).

``GA_BENCH_ENGINE=tests.bench_cpu_engine:make_engine GA_DIST_BACKEND=gloo python bench.py --gpus 2``
runs the real launcher, rank processes and slab orchestration (globalign_amd/distributed.py)
with the oracle-backed engine of tests/test_distributed.py under them."""
import time

from tests.test_distributed import OracleSlabEngine


class TimedOracleSlabEngine(OracleSlabEngine):
    def slab_launch(self, traceback=True):
        self._t0 = time.perf_counter()
        super().slab_launch(traceback)

    def slab_finish(self):
        cost = super().slab_finish()
        self._fill_ms = (time.perf_counter() - self._t0) * 1e3
        return cost

    def timings(self):
        return {"fill_ms": getattr(self, "_fill_ms", 0.0), "walk_ms": 0.0, "rng_ms": 0.0, "call_ms": 0.0}

    def synchronize(self):
        pass

    def torch_device(self):
        return "cpu"


def make_engine(tables):
    K = tables.K
    cmat = {x: {y: int(tables.sub[tables.code[x] * K + tables.code[y]]) for y in tables.keys} for x in tables.keys}
    return TimedOracleSlabEngine(cmat, tables.gap_open)
