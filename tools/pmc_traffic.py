"""Turn a rocprofv3 `--pmc FETCH_SIZE` counter CSV into profiles/<tag>_traffic.json for bench.py.

    python tools/pmc_traffic.py gpurun_out/pmc_r01/run_counter_collection.csv r01 deep_kernel 1024x4194304:sha1+crc32

HBM bytes per launch = median over the kernel's dispatches of FETCH_SIZE (KiB) x 1024 x 2:
on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read
(MI355X_MICROARCH.md, section HBM), so it is doubled.  The same x 2 holds for WIDE's per-lane
pattern (16 B per lane, 64 distinct lines per instruction): calibrated on a known byte count with
tools/microbench/mb_wide_fetch (profiles/r04_fetch/: FETCH_SIZE x 2 = TCC_EA0_RDREQ x 128 B, no
32-B requests, and = the bytes read for every shape whose lines are fetched once).  WRITE_SIZE
(digests/states, < 200 KiB per launch) needs its own pass and is not included.
"""
import csv
import json
import os
import statistics
import sys


def main(path, tag, kernel, workload_key):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == "FETCH_SIZE" and kernel in r["Kernel_Name"]]
    if not vals:
        sys.exit(f"no FETCH_SIZE rows for {kernel} in {path}")
    kib = statistics.median(vals)
    out = {
        "kernel": kernel,
        "workload_key": workload_key,
        "bytes_per_launch": kib * 1024 * 2,
        "fetch_size_kib_median": kib,
        "dispatches": len(vals),
        "correction": "FETCH_SIZE (KiB) x 1024 x 2 (gfx950 reports half of a streaming read; the same factor "
                      "calibrated for WIDE's per-lane pattern, profiles/r04_fetch/)",
        "source": os.path.relpath(path),
    }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles", f"{tag}_traffic.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(dst, out)


if __name__ == "__main__":
    main(*sys.argv[1:5])
