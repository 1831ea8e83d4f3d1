"""CPU checks of the oracle's Redis-keyspace export (the checker of rl_export_state):
every live key appears once with its PEXPIRE deadline, expired keys do not, and
keyspace -> load_keyspace -> keyspace is the identity."""
import numpy as np

from oracle.rl_oracle import SW, TB, PyOracle

NS = 1_000_000
T0 = 1_700_000_000_000


def test_keyspace_deadlines_and_round_trip():
    o = PyOracle()
    o.add_limiter(SW, 3, 1000)
    o.add_limiter(TB, 5, 1000, 2.0)
    keys = np.array([11, 11, 11, 12, 11, 12], np.uint64)
    lim = np.array([0, 0, 0, 0, 1, 1], np.uint16)
    now = (T0 + np.array([10, 20, 1010, 1500, 1600, 1700])) * NS
    a, r, t = o.run(keys, np.array([1, 1, 1, 1, 2, 1], np.int32), now, lim)
    assert list(a) == [1, 1, 1, 1, 1, 1]
    w0 = (T0 // 1000) * 1000
    assert o.keyspace(T0 + 1015)[:2] == [
        (0, 11, 0, w0, 2, 0.0, 0, T0 + 20 + 1000),
        (0, 11, 0, w0 + 1000, 1, 0.0, 0, T0 + 1010 + 1000)]
    ks = o.keyspace(T0 + 1700)
    assert ks == [
        (0, 11, 0, w0 + 1000, 1, 0.0, 0, T0 + 1010 + 1000),
        (0, 12, 0, w0 + 1000, 1, 0.0, 0, T0 + 1500 + 1000),
        (1, 11, 1, 0, 0, 3.0, T0 + 1600, T0 + 1600 + 2000),
        (1, 12, 1, 0, 0, 4.0, T0 + 1700, T0 + 1700 + 2000),
    ]
    # the first window's bucket lapses 1000 ms after its last INCR
    assert [k[3] for k in o.keyspace(T0 + 1021) if k[0] == 0 and k[1] == 11] == [w0 + 1000]
    o2 = PyOracle()
    o2.add_limiter(SW, 3, 1000)
    o2.add_limiter(TB, 5, 1000, 2.0)
    o2.load_keyspace(o.keyspace(T0 + 1015))
    assert o2.keyspace(T0 + 1015) == o.keyspace(T0 + 1015)
    assert o2.keyspace(T0 + 1700) == ks
    assert o.keyspace(T0 + 10_000) == []
