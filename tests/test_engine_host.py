"""Host logic of Engine.run's plan cache (CPU: plans are stand-ins, no device)."""

from collections import OrderedDict

import numpy as np


def _engine(cache_size=1):
    from classical_speech_enhancement_amd.engine import Engine
    eng = Engine.__new__(Engine)  # no device: only the cache logic runs
    eng._plan_cache = OrderedDict()
    eng.plan_cache_size = cache_size
    eng._side = None
    built = []

    class Plan:
        def __init__(self, specs):
            self.specs, self.runs = specs, 0

        def execute(self, noisy, clean=None, on_plan=None):
            self.runs += 1
            if on_plan is not None:
                on_plan(self)

        def results(self):
            return {"plan": self}

    def plan(S, L, specs, *args, **kw):
        built.append(Plan(specs))
        return built[-1]
    eng.plan = plan
    return eng, built


X = np.zeros((2, 16000))


def test_reuse_hits_and_evicts_at_size_one():
    eng, built = _engine()
    a1 = eng.run(X, [("a",)], reuse="A")["plan"]
    a2 = eng.run(X, [("a",)], reuse="A")["plan"]
    assert a1 is a2 and len(built) == 1 and a1.runs == 2
    b = eng.run(X, [("b",)], reuse="B")["plan"]
    assert b is not a1 and len(eng._plan_cache) == 1
    a3 = eng.run(X, [("a",)], reuse="A")["plan"]  # A was evicted by B
    assert a3 is not a1 and len(built) == 3


def test_two_entries_alternate_without_rebuilding():
    eng, built = _engine(cache_size=2)
    seen = [eng.run(X, [(k,)], reuse=k)["plan"] for k in "ABABAB"]
    assert len(built) == 2
    assert seen[0] is seen[2] is seen[4] and seen[1] is seen[3] is seen[5]


def test_no_reuse_builds_every_call_and_keeps_cache():
    eng, built = _engine()
    eng.run(X, [("a",)], reuse="A")
    eng.run(X, [("a",)])
    eng.run(X, [("a",)])
    assert len(built) == 3 and list(eng._plan_cache) and len(eng._plan_cache) == 1


def test_callable_specs_are_built_only_on_a_miss():
    eng, built = _engine()
    calls = []

    def specs():
        calls.append(1)
        return [("a",)]
    eng.run(X, specs, reuse="A", keep=object())
    eng.run(X, specs, reuse="A")
    assert len(calls) == 1 and len(built) == 1


def test_on_plan_reaches_the_plan():
    eng, _ = _engine()
    got = []
    eng.run(X, [("a",)], reuse="A", on_plan=got.append)
    assert len(got) == 1


def test_structure_digest_and_fingerprint():
    """Plan-reuse keys: the digest object hashes numpy buffers without a copy
    (xxh3 when importable, blake2b otherwise) and equal structures give equal
    fingerprints, different ones different."""
    import numpy as np
    from classical_speech_enhancement_amd.engine import spec_fingerprint, structure_digest
    a, b = structure_digest(), structure_digest()
    x = np.arange(1000, dtype=np.int64)
    a.update(x)
    b.update(x.tobytes())
    assert a.hexdigest() == b.hexdigest() and len(a.hexdigest()) == 32
    p, q = {"n_fft": 512}, {"n_fft": 1024}
    s1 = [(0, "wiener", p), (1, "mmse", q)]
    assert spec_fingerprint(s1) == spec_fingerprint(list(s1))
    assert spec_fingerprint(s1) != spec_fingerprint([(0, "wiener", p), (1, "mmse", p)])
