"""bench.py's multi-rank body on real hardware with one GPU: N processes (default 2) join a
gloo group on 127.0.0.1, each drives the GPU engine on device 0 through ``bench.run`` (the
same per-rank function the driver's ``torch.distributed.run --nproc-per-node N`` launch
uses, with RCCL), and rank 0 prints the single JSON line: barrier + max-over-ranks timing,
the verdict all-gather and weak-scaling aggregation run with the real engine.  RCCL itself
needs one GPU per rank, so the collectives here are gloo over host tensors.  Tool (tools/).

usage: python tools/bench_ranks_one_gpu.py [world] [extra bench args...]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    import bench

    args = bench.parse(sys.argv[2:])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    line = bench.run(args, rank, world, 0, dist, cdev="cpu")
    if line is not None:
        print(json.dumps(line), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    extra = sys.argv[2:] or ["--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--corpus-scenarios", "0",
                             "--keccak-log2", "0"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29533"),
               WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, "-u", __file__, "--child", "--gpus", str(world), *extra],
                              env=dict(env, RANK=str(r), LOCAL_RANK="0"), stdout=subprocess.PIPE, text=True)
             for r in range(world)]
    outs = [p.communicate()[0] for p in procs]
    codes = [p.returncode for p in procs]
    print(outs[0].strip().splitlines()[-1] if outs[0].strip() else "(no line from rank 0)")
    sys.exit(max(abs(c) for c in codes))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
    else:
        main()
