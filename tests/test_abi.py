"""CPU checks of the drop-in boundary: the HIP library loads, exports every symbol the
public headers declare, and its host-side utilities behave (no GPU compute here)."""
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in ("veneur_amd.h", "veneur_amd_synth.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        syms |= set(re.findall(r"\b(vn_[a-z0-9_]+)\s*\(", src))
    return syms


def test_library_exports_every_declared_symbol():
    import veneur_amd._abi as A
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in sorted(syms):
        assert hasattr(A.lib, s), "missing export %s" % s
    assert set(A.EXPORTED) == syms
    assert A.lib.vn_abi_version() == 6


def test_struct_layouts_match_header():
    import ctypes as C
    import veneur_amd._abi as A
    # sizes derived from the C declarations (LP64)
    assert C.sizeof(A.Config) == 4 + 16 + 4 + 8 + 4 + 4 + 16 * 8 + 8 + 8 + 4 + 4 + 4 + 4 + 8 + 8 + 4 + 4 + 4 * 8  # (+ padding)
    assert C.sizeof(A.Batch) == 16 * 8
    assert C.sizeof(A.SplitBatch) == 9 * 8
    assert C.sizeof(A.SetState) == 4 + 5 * 4
    # and the library's own sizeof of every struct the binding passes (vn_struct_size)
    for which, st in ((0, A.Config), (1, A.Batch), (2, A.FlushResult), (3, A.Timing), (4, A.SplitBatch),
                      (5, A.Stage)):
        assert A.lib.vn_struct_size(which) == C.sizeof(st), st.__name__
    assert A.lib.vn_struct_size(99) == 0


def test_synth_deterministic_and_thread_independent():
    import veneur_amd as V
    a = V.synth(seed=7, n_keys=500, n_samples=20000, threads=1)
    b = V.synth(seed=7, n_keys=500, n_samples=20000, threads=5)
    for k in ("c_slot", "c_val", "c_rate", "g_slot", "g_val", "h_slot", "h_val", "h_rate", "s_slot", "s_off",
              "s_bytes"):
        assert np.array_equal(a[k], b[k]), k
    assert sum(len(a[k]) for k in ("c_slot", "g_slot", "h_slot", "s_slot")) == 20000
    assert a["s_off"][-1] == len(a["s_bytes"])


def test_synth_sharding_partitions_keys():
    import oracle
    import veneur_amd as V
    full = V.synth(seed=9, n_keys=2000, n_samples=1000)
    tot = [0, 0, 0, 0]
    for shard in range(4):
        d = V.synth(seed=9, n_keys=2000, n_samples=1000, shard=shard, n_shards=4)
        for c in range(4):
            tot[c] += d["n_slots"][c]
            assert np.all(d["digest_of_slot"][c] % 4 == shard)
        # digest is veneur's FNV-1a(name || type || joinedTags) (samplers/parser.go:213-304)
        tn = ("counter", "gauge", "histogram", "set")
        for c in range(4):
            for s in range(min(3, d["n_slots"][c])):
                key = int(d["key_of_slot"][c][s])
                assert oracle.metric_digest("k%07d" % key, tn[c]) == int(d["digest_of_slot"][c][s])
    assert tuple(tot) == full["n_slots"]


def test_oracle_processes_synth_stream():
    import veneur_amd as V
    from tests.util import run_oracle
    d = V.synth(seed=11, n_keys=300, n_samples=30000)
    w = run_oracle(d, d["n_slots"])
    s = int(d["c_slot"][0])
    assert w.touched(0, s)
    # counters are integers 1..10 times 1, 2 or 10
    vals = [w.counter_value(int(x)) for x in np.unique(d["c_slot"])]
    assert all(v > 0 for v in vals)


def test_graft_build_entry_checks_the_current_abi():
    """__graft_entry__.build() compares the library's ABI with the binding's, not a fixed number."""
    import inspect
    import __graft_entry__ as g
    src = inspect.getsource(g.build)
    assert "A.ABI_VERSION" in src
