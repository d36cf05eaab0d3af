"""Does cbx_peer_export / cbx_peer_import work in a process that imported
torch first (so the library runs on torch's bundled HIP runtime), launched by
torch.distributed.run?  Prints one line per stage to stderr (feasibility probe,
not a test).  Usage: torch.distributed.run --nproc-per-node 2 scripts/ipc_torch_probe.py [--no-torch]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def say(*a):
    print(f"[rank {os.environ.get('RANK')} {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def main():
    use_torch = "--no-torch" not in sys.argv
    serial = "--serial" in sys.argv
    n = int(sys.argv[sys.argv.index("--elements") + 1]) if "--elements" in sys.argv else 1 << 20
    R = int(sys.argv[sys.argv.index("--replicas") + 1]) if "--replicas" in sys.argv else 2
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if use_torch:
        import torch
        torch.cuda.set_device(0)
        say("torch HIP", torch.version.hip)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from crossbow_amd import dist as D
    from crossbow_amd import TheGPU, UPDATE_SMA, SYNC_BSP
    D.rehearsal_env(rank)
    gpu = TheGPU()
    uid = D.share_unique_id(rank, world, TheGPU.unique_id)
    gpu.init_rank(0, world, rank, uid)
    say("init_rank done")
    from crossbow_amd import _lib
    shape = [n]
    gpu.setModel(1, 4 * shape[0])
    gpu.setModelVariable(0, 1, shape, 4 * shape[0])
    gpu.setUpdateModelType(UPDATE_SMA)
    gpu.setModelManager(R, SYNC_BSP)
    say("manager set")
    blob = gpu.peer_export()
    say("exported")
    blobs = [None] * world
    dist.all_gather_object(blobs, blob)
    say("gathered; importing" + (" one rank at a time" if serial else ""))
    if serial:
        # the round-4 experiment that found the open-in-turn rule; since then
        # cbx_peer_import runs the turns itself (every rank must call it at
        # once), so this form now ends in the library's 120 s turn timeout
        for r in range(world):
            if r == rank:
                gpu.peer_import(blobs)
            dist.barrier()
    else:
        gpu.peer_import(blobs)
    say("imported")
    gpu.set_allreduce_algorithm(_lib.ALLREDUCE_PEER)
    gpu.set_bucket_elements(1 << 18)
    gpu.fill_synthetic(1)
    for step in range(3):
        gpu.lockAny()
        gpu.synchronise(0, step + 1, 0, False)
        gpu.unlockAny()
    gpu.wait()
    say("3 peer steps done")
    gpu.free()
    say("freed")
    dist.destroy_process_group()


main()
