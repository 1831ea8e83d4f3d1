"""Loading helpers for tests/golden fixtures (JSON + npz, no pickle)."""
import json
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_kats():
    with open(os.path.join(HERE, "kats.json")) as f:
        return json.load(f)["cases"]


def kat_arrays(case):
    r = case["requests"]
    keys = np.array([x[0] for x in r], np.uint64)
    permits = np.array([x[1] for x in r], np.int32)
    now = np.array([x[2] for x in r], np.int64)
    lim = np.array([x[3] for x in r], np.uint16)
    ops = np.array([x[4] for x in r], np.uint8)
    return keys, permits, now, lim, ops


def load_traces():
    z = np.load(os.path.join(HERE, "traces.npz"), allow_pickle=False)
    names = sorted({k.split("__")[0] for k in z.files})
    out = {}
    for n in names:
        d = {k.split("__")[1]: z[k] for k in z.files if k.startswith(n + "__")}
        d["limiters"] = [[int(l[0]), int(l[1]), int(l[2]), float(l[3])] for l in d["limiters"]]
        out[n] = d
    return out
