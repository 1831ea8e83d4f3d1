"""Config 1 (RateLimiterBenchmark.java:48-71) stage breakdown: the 100k single-key SW stream
with the local cache, on a fresh engine (bench.py's figure) and on an engine whose scratch
was allocated by an earlier batch of another key, with per-stage hipEvent times."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-rate-limiter_amd", "python"))
import rl_amd  # noqa: E402

NS = 1_000_000


def main():
    dev = torch.device("cuda:0")
    n = 100_000
    t0 = (1_700_000_000_000 // 60000) * 60000 + 5000
    keys = np.full(n, rl_amd.key_hash("user123"), np.uint64)
    now = (t0 * NS + np.arange(n, dtype=np.int64) * 12_500).astype(np.int64)
    permits = np.ones(n, np.int32)
    lim = (rl_amd.SW, 100_000, 60_000, 0.0, 0, 50)
    d = [torch.from_numpy(x).to(dev) for x in (keys.view(np.int64), permits, now)]
    other = torch.from_numpy(np.full(n, rl_amd.key_hash("warm"), np.uint64).view(np.int64)).to(dev)
    early = torch.from_numpy(now - 600_000 * NS).to(dev)
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    r = torch.empty(n, dtype=torch.int64, device=dev)
    for warm in (False, True):
        for timing in (False, True):
            e = rl_amd.Engine(device=0, max_batch=n, capacity=1 << 10, stage_timing=timing)
            e.add_limiter(*lim)
            if warm:
                e.execute_device(n, other, d[1], early, None, None, a, r)
                e.sync()
            torch.cuda.synchronize()
            g0 = time.perf_counter()
            e.execute_device(n, *d, None, None, a, r)
            e.sync()
            dt = time.perf_counter() - g0
            st = e.stage_times() if timing else {}
            print(f"warm={warm} timing={timing} wall {dt * 1e3:.3f} ms "
                  f"{n / dt:.3e}/s allowed {int(a.sum())}", flush=True)
            if st:
                print("   " + " ".join(f"{k}={v:.3f}" for k, v in st.items()), flush=True)
            e.close()


if __name__ == "__main__":
    main()
