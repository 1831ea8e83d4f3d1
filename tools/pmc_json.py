#!/usr/bin/env python3
"""Fold a tools/profile.sh output directory into profiles/pmc_summary.json, the file
bench.py reads `roofline.traffic` from.

Per pipeline stage (bench.py's stage names) it records the rocprofv3 kernel-trace
average duration and the per-launch HBM-side byte counters, corrected as
/opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes:
  * FETCH_SIZE / WRITE_SIZE are reported in KiB            -> x 1024
  * FETCH_SIZE counts half the bytes of wide streaming reads on gfx950 -> x 2
  * WRITE_SIZE is exact for streaming stores               -> x 1
Both counters are taken from their own --pmc pass (they do not fit one pass). They
count L2 -> fabric traffic, so Infinity-Cache hits are included: the figure is an
upper bound on HBM bytes. The x2 is calibrated for 16-B/lane streaming reads only; the
engine's 2-B gathers and scattered stores are calibrated by tools/calib_fetch.sh
(profiles/r04_calib). TCC_EA0_ATOMIC_sum (its own pass) is the L2's fabric-side atomic
request count (north_star's atomic profile).

usage: tools/pmc_json.py <profile dir> <config name> [--out profiles/pmc_summary.json] [--tag DIR]

The entry and _meta[config] always name the directory the values came from (--tag, else the
profile directory as given): tests/test_pmc_provenance.py recomputes `step` from it.
"""
import argparse
import collections
import csv
import json
import os


# bench.py CONFIGS[...]["batch"] (requests per GPU per step)
DEFAULT_BATCH = {"tb_uniform": 1 << 26, "sw_zipf": 1 << 28, "mixed_tenants": 1 << 27,
                 "zipf_1b": 1 << 27}


def stage_of(name: str):
    def raw(n):  # second template argument: pass 0 reads the raw request arrays
        args = n.split("<", 1)[1].split(">")[0].split(",")
        return len(args) > 1 and args[1].strip() == "true"
    if "k_upsweep<" in name:
        return "upsweep0" if raw(name) else "upsweep1"
    if "k_scatter<" in name or "k_scatter_split<" in name:
        return "scatter0" if raw(name) else "scatter1"
    if "k_regions<" in name:
        return "region"
    if "k_unpermute<" in name or "k_unpermute_split<" in name:
        return "unpermute"
    if "k_group<" in name:
        return "group"
    if "k_unpermute_mid<" in name:
        return "unpermute_mid"
    if "k_hot_chains<" in name:
        return "hot_chains"
    if "k_hot_summ<" in name:
        return "hot_summ"
    if "k_hot_fill<" in name:
        return "hot_fill"
    if "k_solo<" in name:
        return "solo"
    return None


def _csv(base, f, name):
    """A pass's CSV in a tools/profile.sh output directory (gpurun_out/prof_<tag>/<f>/) or in
    its committed copy (profiles/<tag>/, flattened)."""
    for p in (f"{base}/{f}/{name}", f"{base}/{name}"):
        if os.path.exists(p):
            return p
    return None


def summarize(base):
    """Per-stage kernel-trace averages and PMC means of one profile directory, plus the
    whole step's bytes (the entry bench.py reads as roofline.traffic)."""
    base = base.rstrip("/")
    st = {}
    for r in csv.DictReader(open(_csv(base, "trace", "trace_kernel_stats.csv"))):
        s = stage_of(r["Name"])
        if s:
            st[s] = {"kernel": r["Name"], "calls": int(r["Calls"]),
                     "avg_us": float(r["AverageNs"]) / 1e3}
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in ("fetch", "write", "tcc", "sq", "atomic"):
        p = _csv(base, f, f"{f}_counter_collection.csv")
        if p is None:
            continue
        for r in csv.DictReader(open(p)):
            s = stage_of(r["Kernel_Name"])
            if s:
                counters[s][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for s, cs in counters.items():
        d = st.setdefault(s, {})
        mean = {k: sum(v) / len(v) for k, v in cs.items()}
        if "FETCH_SIZE" in mean:
            d["fetch_kib_raw"] = mean["FETCH_SIZE"]
            d["fetch_bytes"] = mean["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in mean:
            d["write_bytes"] = mean["WRITE_SIZE"] * 1024
        if "fetch_bytes" in d and "write_bytes" in d:
            d["hbm_bytes_per_launch"] = d["fetch_bytes"] + d["write_bytes"]
        if "TCC_EA0_ATOMIC_sum" in mean:
            d["l2_fabric_atomics"] = mean["TCC_EA0_ATOMIC_sum"]
        if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
            tot = mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"]
            d["l2_hit_rate"] = mean["TCC_HIT_sum"] / tot if tot else None
        for k in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_ANY",
                  "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES"):
            if k in mean:
                d[k] = mean[k]
    # the whole step: every kernel of the bench's timed and warmup steps except the
    # trace generator, divided by the number of steps (unpermute launches)
    steps = st.get("unpermute", {}).get("calls")
    tot = collections.defaultdict(float)
    for f, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = _csv(base, f, f"{f}_counter_collection.csv")
        if p is None:
            continue
        for r in csv.DictReader(open(p)):
            if "k_synth" not in r["Kernel_Name"] and r["Counter_Name"] == ctr:
                tot[ctr] += float(r["Counter_Value"])
    if steps and "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
        st["step"] = {"fetch_bytes": tot["FETCH_SIZE"] * 1024 * 2 / steps,
                      "write_bytes": tot["WRITE_SIZE"] * 1024 / steps, "steps": steps}
        st["step"]["hbm_bytes_per_launch"] = st["step"]["fetch_bytes"] + st["step"]["write_bytes"]
    # The steady state: batches 1.. only (batch 0 is the bench's first warmup step: no routed
    # regions yet, so every record takes the grouping pass; the timed steps all route). A
    # batch starts at its pass-0 upsweep (dispatch order).
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = _csv(base, f, f"{f}_counter_collection.csv")
        if p is None:
            continue
        b = -1
        for r in sorted(csv.DictReader(open(p)), key=lambda r: int(r["Dispatch_Id"])):
            if stage_of(r["Kernel_Name"]) == "upsweep0":
                b += 1
            if b >= 0 and "k_synth" not in r["Kernel_Name"] and r["Counter_Name"] == ctr:
                per[b][ctr] += float(r["Counter_Value"])
    bs = [b for b in sorted(per) if b >= 1 and "FETCH_SIZE" in per[b] and "WRITE_SIZE" in per[b]]
    if bs:
        fb = sum(per[b]["FETCH_SIZE"] for b in bs) * 1024 * 2 / len(bs)
        wb = sum(per[b]["WRITE_SIZE"] for b in bs) * 1024 / len(bs)
        st["step_steady"] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
                             "batches": bs}
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("config")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "pmc_summary.json"))
    ap.add_argument("--tag", default="",
                    help="the directory the values are cited from (default: prof_dir as given, "
                         "e.g. profiles/r06_sw_zipf); always recorded in _meta and the entry")
    ap.add_argument("--batch", type=int, default=0,
                    help="requests per GPU per step of the profiled run (default: the config's)")
    ap.add_argument("--world", type=int, default=1, help="ranks of the profiled run")
    a = ap.parse_args()
    st = summarize(a.prof_dir)
    tag = a.tag or a.prof_dir.rstrip("/")
    st["source"] = tag
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    # bench.py reports `roofline.traffic` only for the workload the profile was taken on
    st["batch"] = a.batch or DEFAULT_BATCH[a.config]
    st["world"] = a.world
    out[a.config] = st
    out.setdefault("_meta", {})["note"] = (
        "per-launch means; fetch_bytes = FETCH_SIZE KiB x1024 x2 (gfx950 wide-read "
        "correction), write_bytes = WRITE_SIZE KiB x1024; L2->fabric bytes, Infinity-Cache "
        "hits included (upper bound on HBM bytes)")
    out["_meta"][a.config] = tag                    # provenance: where the values came from
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1, sort_keys=True)
    for s, d in sorted(st.items()):
        if not isinstance(d, dict):
            continue
        print(f"{s:10s} {d.get('avg_us', 0):9.1f} us  hbm/launch "
              f"{d.get('hbm_bytes_per_launch', 0) / 1e9:.3f} GB  l2hit {d.get('l2_hit_rate') or 0:.2f}")


if __name__ == "__main__":
    main()
