#!/usr/bin/env python3
"""HBM traffic per launch of the SMA kernels from rocprofv3 PMC passes.

Reads the ``*_counter_collection.csv`` files of separate ``rocprofv3 --pmc``
passes (one counter group per pass: FETCH_SIZE in one, WRITE_SIZE in another,
as MI355X_MICROARCH.md "rocprofv3 PMC slots" requires) and writes, per kernel,
the mean bytes per dispatch.  gfx950 corrections (MI355X_MICROARCH.md "HBM"):

* FETCH_SIZE (KiB) reports half the bytes of a wide (16 B/lane) coalesced
  streaming read, so read bytes = 2 * FETCH_SIZE * 1024;
* WRITE_SIZE (KiB) is exact for 16 B/lane streaming stores.

hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.

Usage: pmc_traffic.py --out traffic.json --key-suffix resnet50/R8/m1 DIR [DIR...]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short_name(kernel: str) -> str:
    m = re.search(r"(sma_\w+_kernel|copy_kernel|fill_normal_kernel)", kernel)
    return m.group(1) if m else kernel.split("(")[0]


def collect(dirs):
    # (kernel, counter) -> list of per-dispatch values
    vals = defaultdict(list)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per_dispatch = defaultdict(float)
            with open(path, newline="") as f:
                for row in csv.DictReader(f):
                    k = (short_name(row["Kernel_Name"]), row["Counter_Name"], row.get("Dispatch_Id", ""))
                    per_dispatch[k] += float(row["Counter_Value"])  # sum over dimensions, if any
            for (kern, ctr, _), v in per_dispatch.items():
                vals[(kern, ctr)].append(v)
    return vals


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", required=True)
    p.add_argument("--key-suffix", required=True, help="e.g. resnet50/R8/m1 (matches bench.py)")
    p.add_argument("--alg-bytes", action="append", default=[],
                   help="KERNEL=BYTES algorithmic bytes per launch of KERNEL (repeatable), for the ratio")
    p.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "crossbow_amd", "libcrossbow_sma.so"),
                   help="the library the PMC passes ran (its device-code digest is stored with each entry)")
    p.add_argument("--only", action="append", default=[],
                   help="record only this kernel (repeatable; default: every kernel in the passes)")
    p.add_argument("dirs", nargs="+")
    a = p.parse_args()
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from crossbow_amd.build import code_object_digest
    digest = code_object_digest(a.lib)
    vals = collect(a.dirs)
    kernels = sorted({k for k, _ in vals if not a.only or k in a.only})
    out = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            out = json.load(f)
    for kern in kernels:
        rec = {}
        for (k, ctr), v in vals.items():
            if k == kern and v:
                rec[ctr] = {"mean": sum(v) / len(v), "dispatches": len(v)}
        fetch = rec.get("FETCH_SIZE", {}).get("mean")
        write = rec.get("WRITE_SIZE", {}).get("mean")
        entry = {"counters": rec}
        if fetch is not None and write is not None:
            entry["read_bytes_per_launch"] = 2 * fetch * 1024
            entry["write_bytes_per_launch"] = write * 1024
            entry["hbm_bytes_per_launch"] = 2 * fetch * 1024 + write * 1024
            alg = dict(x.split("=", 1) for x in a.alg_bytes)
            if kern in alg:
                entry["alg_bytes_per_launch"] = float(alg[kern])
                entry["traffic_over_alg"] = entry["hbm_bytes_per_launch"] / float(alg[kern])
        entry["correction"] = "read = 2*FETCH_SIZE KiB (gfx950 half-count of 16B/lane streams), write = WRITE_SIZE KiB"
        entry["code_object_sha256"] = digest  # .hip_fatbin of the library that ran (crossbow_amd.build)
        out[f"{kern}/{a.key_suffix}"] = entry
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
