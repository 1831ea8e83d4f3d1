"""The oracle is pinned before it is trusted: both restatements (C and Python)
must reproduce every known-answer test in tests/golden/kats.json (restated
reference unit tests + hand-derived edge cases) and agree with each other."""
import math

import numpy as np
import pytest

from golden_io import kat_arrays, load_kats, load_traces
from oracle.coracle import COracle
from oracle.rl_oracle import PyOracle

KATS = load_kats()


def _check(case, res):
    a, rem, tok = res[0], res[1], res[2]
    for i, (ea, er, et) in enumerate(case["expected"]):
        assert int(a[i]) == ea, (case["name"], i, "allowed")
        assert int(rem[i]) == er, (case["name"], i, "remaining", int(rem[i]), er)
        if et is not None:
            assert float(tok[i]) == et, (case["name"], i, "tokens", float(tok[i]), et)


@pytest.mark.parametrize("case", KATS, ids=[c["name"] for c in KATS])
def test_c_oracle_kat(case, coracle_lib):
    o = COracle(case["limiters"])
    _check(case, o.run(*kat_arrays(case)))


@pytest.mark.parametrize("case", KATS, ids=[c["name"] for c in KATS])
def test_py_oracle_kat(case):
    o = PyOracle()
    for l in case["limiters"]:
        o.add_limiter(*l)
    _check(case, o.run(*kat_arrays(case)))


def test_kat_coverage():
    names = {c["name"] for c in KATS}
    for must in ["ref:shouldAllowRequestsUnderLimit", "ref:shouldRejectWhenLimitExceeded",
                 "ref:shouldHandleMultiplePermits", "ref:shouldReportAvailablePermits",
                 "ref:shouldResetLimits", "ref:shouldRejectInvalidPermits",
                 "hand:sw:fmaDiscriminator", "hand:tb:expiryBoundary", "hand:tb:fmaFlip0",
                 "doc:apiRemaining97", "doc:rateLimitExceededRemaining0",
                 "doc:loginRemainingAttempts7", "doc:batchTokensRemaining30",
                 "hand:sw:regressionPrevWindow", "hand:tb:deepNegative"]:
        assert must in names


@pytest.mark.parametrize("name", sorted(load_traces()))
def test_trace_fixtures_reproduce(name, coracle_lib):
    d = load_traces()[name]
    o = COracle(d["limiters"])
    a, r, t, _ = o.run(d["keys"], d["permits"], d["now_ns"], d["limiter"], d["op"])
    assert np.array_equal(a, d["allowed"])
    assert np.array_equal(r, d["remaining"])
    m = ~np.isnan(d["tokens"])
    assert np.array_equal(np.isnan(t), ~m)
    assert np.array_equal(t[m].view(np.uint64), d["tokens"][m].view(np.uint64))


def test_sharded_oracle_matches_sequential(coracle_lib):
    d = load_traces()["mixed_small"]
    seq = COracle(d["limiters"]).run(d["keys"], d["permits"], d["now_ns"], d["limiter"], d["op"])
    par = COracle(d["limiters"], nthreads=4).run(d["keys"], d["permits"], d["now_ns"],
                                                  d["limiter"], d["op"])
    for x, y in zip(seq[:2], par[:2]):
        assert np.array_equal(x, y)


def test_config_validation():
    # SlidingWindowRateLimiterTest.java:178-198 + RateLimitConfig.java:46-56
    o = COracle()
    with pytest.raises(ValueError):
        o.add_limiter(0, -1, 1000)
    with pytest.raises(ValueError):
        o.add_limiter(0, 10, 0)
    with pytest.raises(ValueError):
        o.add_limiter(1, 10, 1000, 0.0)   # TokenBucketRateLimiter.java:77-79
    assert o.add_limiter(0, 10, 1000) == 0
