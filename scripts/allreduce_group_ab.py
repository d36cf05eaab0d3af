#!/usr/bin/env python3
"""All-reduce grouping of the bucketed split path (cbx_set_allreduce_group):
ResNet-50, R = 8, mu 0.9, one GPU, one-rank all-reduce, force split; 8/16
buckets x modes 0, 1, 2 x groups 1, 2, 4, interleaved over 5 rounds, wall ms
per step.  Writes gpurun_out/allreduce_group_ab.json."""
import json, os, statistics, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from crossbow_amd import SYNC_BSP, UPDATE_SMA, TheGPU
from crossbow_amd.variables import MODELS, register
g = TheGPU(); g.init([0]); n = register(g, MODELS["resnet50"]())
g.setUpdateModelType(UPDATE_SMA); g.setEamsgdAlpha(0.1); g.setMomentum(0.9, 0); g.setModelManager(8, SYNC_BSP)
g.set_force_split(True); g.fill_synthetic(1); g.set_timing(True)
clock = 0
def step():
    global clock
    clock += 1; g.lockAny(); g.synchronise(0, clock, 0, False); g.unlockAny()
res = {}
for _ in range(5):
    for nb in (8, 16):
        for mode in (0, 1):
            for grp in (1, 2, 4):
                g.set_allreduce_group(grp)
                g.set_bucket_elements(-(-n // nb)); g.set_pipeline_mode(mode)
                for _ in range(3): step()
                g.wait(); t0 = time.perf_counter()
                for _ in range(30): step()
                g.wait(); res.setdefault((nb, mode, grp), []).append((time.perf_counter() - t0) * 1e3 / 30)
g.free()
out = [dict(buckets=k[0], mode=k[1], allreduce_group=k[2], wall_ms=round(statistics.median(v), 4), rounds=[round(x, 4) for x in v]) for k, v in sorted(res.items())]
for r in out: print(json.dumps(r))
os.makedirs("gpurun_out", exist_ok=True); json.dump(out, open("gpurun_out/allreduce_group_ab.json", "w"), indent=1)
