#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for the engine's access widths (tools/calib_fetch.hip), one
# --pmc pass per counter; prints each kernel's counter bytes over its known HBM-side bytes.
# usage (GPU box, repo root): tools/calib_fetch.sh <out dir>
set -o pipefail
OUT=${1:-gpurun_out/calib}
mkdir -p $OUT
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 -o $OUT/calib_fetch tools/calib_fetch.hip || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $c -d $OUT/$c -o $c --output-format csv -- $OUT/calib_fetch > $OUT/$c.log 2>&1 || { echo "$c pass failed"; tail -5 $OUT/$c.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
lines = 1 << 23
known = {  # kernel -> (counter, known bytes: lines touched x 128 B, or the streamed bytes)
    "stream16": ("FETCH_SIZE", 1 << 30),
    "gather<unsigned short>": ("FETCH_SIZE", lines * 128),
    "gather<unsigned long>": ("FETCH_SIZE", lines * 128),
    "scatter<unsigned short>": ("WRITE_SIZE", lines * 128),
    "scatter<HIP_vector_type<unsigned int, 4u> >": ("WRITE_SIZE", lines * 128),
}
rows = []
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        rows += [(r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), r["Grid_Size"]) for r in csv.DictReader(open(f))]
for name, ctr, val, grid in rows:
    short = name.split("(")[0].replace("void ", "")
    kb = val * 1024
    note = ""
    for k, (kc, kbytes) in known.items():
        if short.startswith(k) and kc == ctr:
            note = f"counter/known-lines-x128B = {kb / kbytes:.3f}"
    print(f"{short:50s} grid {grid:>10s} {ctr:10s} {kb / 1e9:8.3f} GB  {note}")
PY
