"""A rank process for tests/test_bench_ranks_cpu.py's spawner tests: what `python bench.py` runs as a spawned rank
(WORLD_SIZE / RANK / ... set by bench.spawn_ranks), with the stand-in wcpt device API of that test file in place of
libwcpt.so. Not a test module itself."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "wc-path-tracer_amd"), HERE]

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
if os.environ.get("WCPT_TEST_FAIL_RANK") == str(rank):
    sys.stderr.write(f"rank {rank}: failing on purpose\n")
    sys.exit(7)
import wcpt  # noqa: E402,F401  (the real package: its scene module builds the Cornell box on the host)
import wcpt.rdzv  # noqa: E402,F401
from test_bench_ranks_cpu import _fake_wcpt  # noqa: E402

log = []
sys.modules["wcpt"] = _fake_wcpt(rank, world, log)
import bench  # noqa: E402

rc = bench.main(sys.argv[1:])
keys = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
        "WCPT_BENCH_LAUNCH")
json.dump({"env": {k: os.environ.get(k) for k in keys}, "log": [list(x) for x in log], "torch": "torch" in sys.modules},
          open(os.path.join(os.environ["WCPT_TEST_OUT"], f"rank{rank}.json"), "w"))
sys.exit(rc or 0)
