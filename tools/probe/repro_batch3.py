"""Probe (not product): tests/test_batch_replay_gpu.py::test_batched_replay_whole_digest_bit_exact[3]
run `reps` times in one process against the library VN_LIB selects; each run reports pass or the
first differing digest.  Stops at the first engine error (a GPU fault ends the process's use of the
device)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_batch_replay_gpu import _check  # noqa: E402
from veneur_amd.engine import EngineError  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
batches = int(sys.argv[2]) if len(sys.argv) > 2 else 3
fails = 0
for r in range(reps):
    try:
        _check(["lognormal", "falling", "rising", "ints", "seven", "heavy"], 300_000, 11 + batches, batches)
        print("rep %d: pass" % r, flush=True)
    except AssertionError as e:
        fails += 1
        print("rep %d: FAIL %s" % (r, str(e)[:300]), flush=True)
    except EngineError as e:
        print("rep %d: ENGINE ERROR %s" % (r, e), flush=True)
        sys.exit(2)
print("fails %d of %d" % (fails, reps))
