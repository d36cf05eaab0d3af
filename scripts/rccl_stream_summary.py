#!/usr/bin/env python3
"""Summarise scripts/trace_rccl_streams.sh: per rank, the HIP stream-creation
calls in order, and per kernel kind the (Stream_Id, Queue_Id) pairs it ran on
(the library's kernels vs RCCL's), plus how many event records / stream waits
the process issued."""
import collections
import csv
import glob
import json
import os
import sys


def kind(name):
    for k in ("sma_accumulate", "sma_apply", "sma_fused", "nccl", "rccl", "fill_normal", "order_probe"):
        if k in name.lower():
            return k
    return name.split("(")[0][-40:]


def main(out):
    res = {}
    for rd in sorted(glob.glob(os.path.join(out, "rank*"))):
        if not os.path.isdir(rd):
            continue
        r = {}
        kt = glob.glob(os.path.join(rd, "**", "*kernel_trace.csv"), recursive=True)
        ht = glob.glob(os.path.join(rd, "**", "*hip_api_trace.csv"), recursive=True)
        pairs = collections.defaultdict(collections.Counter)
        if kt:
            for row in csv.DictReader(open(kt[0])):
                pairs[kind(row["Kernel_Name"])][f"stream {row.get('Stream_Id')} queue {row.get('Queue_Id')}"] += 1
        r["kernels"] = {k: dict(v) for k, v in pairs.items()}
        if ht:
            calls = collections.Counter()
            creates = []
            for row in csv.DictReader(open(ht[0])):
                fn = row.get("Function", "")
                if fn.startswith("hipStreamCreate") or fn.startswith("hipExtStreamCreate"):
                    creates.append((int(row["Start_Timestamp"]), fn, row.get("Thread_Id")))
                if fn in ("hipEventRecord", "hipEventRecordWithFlags", "hipStreamWaitEvent", "hipStreamWaitValue64",
                          "hipStreamWriteValue64", "hipExtLaunchKernel", "hipLaunchKernel", "hipModuleLaunchKernel",
                          "hipExtModuleLaunchKernel", "hipStreamCreateWithFlags", "hipStreamCreateWithPriority",
                          "hipStreamCreate", "hipMemcpyAsync", "hipMemsetAsync"):
                    calls[fn] += 1
            creates.sort()
            r["stream_creates_in_order"] = [f"{fn} (thread {t})" for _, fn, t in creates]
            r["calls"] = dict(calls)
        res[os.path.basename(rd)] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
