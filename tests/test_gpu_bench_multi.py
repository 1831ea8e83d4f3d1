"""bench.py's N>1 path (torchrun, one rank per GPU, the C-ABI router) rehearsed on the box's
one GPU: RL_BENCH_REHEARSE=1 puts both ranks on cuda:0 and moves the all-to-alls through
gloo on the host. Checks the plumbing the driver's multi-GPU scaling run uses — engine
sizing to the router's receive capacity, the hot-key directory, split rounds — and that the
JSON line reports them (numbers from a rehearsal mean nothing)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(*extra, nproc=2):
    env = dict(os.environ, RL_BENCH_REHEARSE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--steps", "3", "--warmup", "1",
           *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + "\n".join(
        l for l in r.stderr.splitlines() if l.startswith("[rank"))[-6000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


def test_bench_rehearsal_two_ranks_zipf():
    d = _bench("--config", "zipf_1b", "--batch", str(1 << 21))
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["status"] == "ok"
    assert "hot-key directory" in d["config"]["parallelism"]
    rt = d["router"]
    assert rt["recv_cap"] == 2 << 21 and rt["split_steps"] == 0 and rt["rounds_per_step"] == 1.0


def test_bench_rehearsal_split_rounds():
    # receive capacity below what an owner gets: every step runs in several rounds
    d = _bench("--config", "mixed_tenants", "--batch", str(1 << 20), "--recv-cap", str(300_000))
    assert d["status"] == "ok"
    rt = d["router"]
    assert rt["split_steps"] == 4 and rt["rounds_per_step"] > 2


def _bench1(*extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "2",
           "--no-extra", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_bench_footprint_model_matches_device():
    """bench.hbm_footprint (the model test_bench_model checks at --gpus 8) against the device
    bytes the run really holds (hipMemGetInfo before the engine and after the timed steps)."""
    d = _bench1("--config", "zipf_1b", "--batch", str(1 << 23))
    fp = d["hbm_footprint_gb"]
    model = fp["total"] - fp["tables"] + fp["tables_now"]
    assert abs(fp["measured"] - model) <= 0.6 + 0.05 * model, fp
    # pass-1 kernels are charged for the records pass 1 partitions: no io_frac above 1
    for k, v in d["roofline"]["kernels"].items():
        assert v["io_frac"] is None or v["io_frac"] <= 1.0, (k, v)
    assert d["roofline"]["traffic"] is None          # no profile of this batch size
    assert d["parity"].startswith("bit-exact")
