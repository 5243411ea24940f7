"""CPU rehearsal of bench.py's multi-GPU path (replicas only): world_size 2
over gloo -- the timing barriers, the max-over-ranks of the elapsed time and the whole-job
throughput formula that rank 0 reports."""
import os
import socket
import sys

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import bench
    r, w, _ = bench.setup_dist(world, backend="gloo")
    bench.barrier(w)
    elapsed = 1.0 + 0.5 * r  # rank 1 is the slow replica
    e = bench.max_over_ranks(elapsed, w, torch.device("cpu"))
    q.put((r, w, e, bench.job_tflops(w, 2.0 * bench.M * bench.N * bench.K, 10, e)))
    dist.destroy_process_group()


def test_bench_replicas_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    flops = 2.0 * 16384 * 4096 * 4096
    for r, w, e, v in res:
        assert w == world
        assert e == 1.5  # max over ranks
        assert abs(v - world * flops * 10 / 1.5 / 1e12) < 1e-9 * v


def test_bench_cli_spawns_world2():
    """`python bench.py --gpus 2` without a torch.distributed.run environment starts one
    (child process, one rank per device) and reports n_gpus 2; the CPU rehearsal runs the
    same launcher, barriers and max-over-ranks over gloo."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--rehearsal", "--steps", "3", "--warmup", "1"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["value"] > 0
