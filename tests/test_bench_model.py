"""CPU checks of bench.py's accounting (no GPU): the per-GPU HBM footprint of the driver's
runs fits 288 GB at every world size, pass-1 kernels are charged for the records pass 1
actually partitions, and `roofline.traffic` is only taken from a profile of the same
workload."""
import json
import os

import pytest

import bench

DRIVER = dict(steps=20, warm=5)          # the driver's `bench.py --steps 20 --warmup 5`


@pytest.mark.parametrize("ws", [1, 2, 4, 8])
@pytest.mark.parametrize("name", sorted(bench.CONFIGS))
def test_footprint_fits_288gb(name, ws):
    n = bench.CONFIGS[name]["batch"]
    fp = bench.hbm_footprint(name, n, ws, DRIVER["steps"], DRIVER["warm"],
                             parity_tokens=ws == 1)
    # one doubling of every table on top (on-demand growth) and 4 GB of runtime slack
    worst = fp["total"] + fp["tables"] + 4e9
    assert worst <= bench.HBM_BYTES_PER_GPU, (name, ws, {k: v / 1e9 for k, v in fp.items()
                                                          if not isinstance(v, bool)})
    assert fp["fits_288GB"]


def test_footprint_sw_zipf_gpus8_components():
    """The verdict's case: --gpus 8 --config sw_zipf --steps 20 --warmup 5."""
    n = 1 << 28
    fp = bench.hbm_footprint("sw_zipf", n, 8, 20, 5)
    assert fp["inputs"] == 25 * n * 20
    # the router reserves its send side for n and its receive side for 2n (rl_router_create_ex)
    assert fp["router"] > n * 58 + 2 * n * 63 - 1
    assert fp["total"] < 240e9


def test_pass1_io_uses_normal_records():
    n, nn = 1 << 28, 110_000_000
    assert bench.kernel_io_bytes("group", n, 0, 1, 1, nn) == nn * 52
    assert bench.kernel_io_bytes("scatter0", n, 0, 1, 1, nn) == n * 40


def test_traffic_keyed_by_workload(tmp_path, monkeypatch):
    d = json.load(open(os.path.join(bench.ROOT, "profiles", "pmc_summary.json")))
    for name in ("sw_zipf", "tb_uniform", "zipf_1b", "mixed_tenants"):
        assert d[name]["batch"] == bench.CONFIGS[name]["batch"] and d[name]["world"] == 1
        v, src = bench.load_pmc(name, "step", bench.CONFIGS[name]["batch"], 1)
        assert v > 0 and src == d["_meta"][name] and os.path.isdir(os.path.join(bench.ROOT, src))
        assert bench.load_pmc(name, "step", bench.CONFIGS[name]["batch"], 2) == (None, None)
        assert bench.load_pmc(name, "step", 1 << 21, 1) == (None, None)


def test_walk_tables_only_where_a_key_can_walk():
    # tb_uniform (and the minute-window configs) never walk, so the engine
    # holds no walk tables for them; mixed_tenants' TB 1000 @ 100/s can
    walks = {name: bench.walk_possible(cfg) for name, cfg in bench.CONFIGS.items()}
    assert walks == {"tb_uniform": False, "sw_zipf": False, "zipf_1b": False, "mixed_tenants": True}
    fp = bench.hbm_footprint("tb_uniform", 1 << 26, 1, 20, 5)
    assert fp["walk_tables"] == 0
