"""Benchmark of the W4A4 mixed-precision linear on MI355X (BASELINE.json config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--act per_group|per_token]

A "step" is one W4A4Linear.forward over one synthetic batch resident in HBM:
W4A4Linear(4096, 4096), weight per_group (sorted) int4, G=128, 10% salient channels,
x[bs*seq = 16384, 4096] fp16 -- activation quantization (column absmax over the batch,
stable sort, per-(row, group) scales) + the mixed-precision MFMA GEMM with the salient
fp16 side-GEMM.  `value` is whole-job TFLOP/s = N_gpus * 2*M*N*K / max-over-ranks time.

Multi-GPU: the op is per-layer and does not shard ("replicas only"): each rank
runs an independent replica on its own GPU; the only collectives are the timing barriers
and the max-over-ranks of the elapsed time.

Also printed in the same JSON line:
  roofline      the dominant kernel (the GEMM), timed live with HIP events on the stream
                it runs on; achieved = 2*M*N*K / average GEMM duration; peak = dense MFMA
                peak of the dtype the kernel computes in.
  cpu_baseline  the CPU oracle (numpy restatement of fake_quant, oracle/) on a bounded
                sample of the same workload, rank 0, N=1 only.
  prepass       the activation-quantization kernels' time and algorithmic GB/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

M, K, N, G, P = 16384, 4096, 4096, 128, 0.10
PEAK_TFLOPS = {"f16": 2516.6, "bf16": 2516.6, "i8": 5033.2, "f8": 5033.2}  # dense MFMA, 256 CU @ 2.4 GHz
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults long enough for the chip to settle at the clock it holds under this load
    # (DVFS, MI355X_MICROARCH.md): ~0.14 s of warmup and of timed steps
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--act", default="per_group", choices=["per_group", "per_token"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-rows", type=int, default=16384)
    return ap.parse_args()


def setup_dist(n, backend="nccl"):
    """One process per GPU (torch.distributed.run env); backend "nccl" is RCCL on ROCm,
    "gloo" is the CPU rehearsal used by tests/test_bench_dist_cpu.py."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(v, world, dev):
    if world == 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_tflops(world, flops_per_step, steps, elapsed_max):
    """Whole-job throughput: every replica ran `steps` steps; the job took the slowest
    rank's time (max over ranks)."""
    return world * flops_per_step * steps / elapsed_max / 1e12


def make_layer(dev, act, seed):
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(seed)
    lin = torch.nn.Linear(K, N, bias=True).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(N, K, generator=gen, device=dev) * 0.02)
        lin.bias.copy_(torch.randn(N, generator=gen, device=dev) * 0.01)
    outl = torch.randperm(K, generator=gen, device=dev)[: K // 100]
    x = torch.randn(M, K, generator=gen, device=dev)
    x[:, outl] *= 30.0
    x = x.half()
    cal = torch.randn(2048, K, generator=gen, device=dev)
    cal[:, outl] *= 30.0
    imp = cal.abs().mean(0).cpu()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act, importance=imp,
                              salient_prop=P, quant_bits=4, group_size=G)
    return q, x, lin


def time_events(fn, iters, stream):
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record(stream)
    for _ in range(iters):
        fn()
    end.record(stream)
    end.synchronize()
    return start.elapsed_time(end) / iters  # ms


def cpu_baseline(rows, act):
    """The oracle (numpy, fp16 emulation, fp64-accumulated product) on `rows` rows."""
    from oracle import fake_quant_oracle as O
    D = O.DT("fp16")
    g = np.random.default_rng(0)
    W = D.rnd(g.standard_normal((N, K)).astype(np.float32) * 0.02)
    b = D.rnd(g.standard_normal(N).astype(np.float32) * 0.01)
    x = g.standard_normal((rows, K)).astype(np.float32)
    outl = g.permutation(K)[: K // 100]
    x[:, outl] *= 30.0
    x = D.rnd(x)
    imp = np.abs(x).mean(0)
    sal = O.select_salient(imp, P)
    t0 = time.perf_counter()
    w_hat = O.w4a4_from_float(W, "per_group", 4, G, sal, D)  # offline, not timed below
    t_pack = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.w4a4_forward(x, w_hat, b, act, 4, G, sal, False, D)
    dt = time.perf_counter() - t0
    threads = os.environ.get("OMP_NUM_THREADS") or str(os.cpu_count())
    try:
        from threadpoolctl import threadpool_info
        info = threadpool_info()
        if info:
            threads = str(max(i.get("num_threads", 1) for i in info))
    except Exception:
        pass
    return {
        "value": 2.0 * rows * N * K / dt / 1e12,
        "unit": "TFLOP/s",
        "cores": int(threads),
        "kind": "port",
        "sample": (f"oracle/fake_quant_oracle.py W4A4Linear forward, fp16 emulation, "
                   f"act {act}, {rows} of {M} rows (K=N={K}, G={G}, p={P}); "
                   f"{dt:.2f} s forward (+{t_pack:.2f} s offline weight quant, untimed)"),
    }


def main():
    args = parse()
    rank, world, local = setup_dist(args.gpus)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from smoothquant import ops

    q, x, lin = make_layer(dev, args.act, seed=1234 + rank)
    pw = q.packed()
    # what W4A4Linear(kernel="auto") runs for this layer
    use_f8 = ops.F8_AUTO and ops.f8_eligible(pw, args.act, 4)
    use_i8 = not use_f8 and ops.I8_AUTO and ops.i8_eligible(pw, args.act, 4)
    stream = torch.cuda.current_stream(dev)

    def step():
        return q(x)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier(world)
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, world, dev)
    ms_per_step = elapsed / args.steps * 1e3
    flops = 2.0 * M * N * K
    value = job_tflops(world, flops, args.steps, elapsed)

    # ---- dominant kernel: the GEMM, timed alone on the same stream with HIP events
    if use_f8:
        a8, sa, xs = ops.quant_act_f8(x, pw, args.act, 4)
        gemm = lambda: ops.gemm_f8(a8, sa, xs, pw, lin.bias)  # noqa: E731
        quant = lambda: ops.quant_act_f8(x, pw, args.act, 4)  # noqa: E731
        kdt = "f8"
    elif use_i8:
        a8, sa, xs = ops.quant_act_i8(x, pw, args.act, 4)
        gemm = lambda: ops.gemm_i8(a8, sa, xs, pw, lin.bias)  # noqa: E731
        quant = lambda: ops.quant_act_i8(x, pw, args.act, 4)  # noqa: E731
        kdt = "i8"
    else:
        a = ops.quant_act_fp(x, pw, args.act, 4, G)
        gemm = lambda: ops.gemm_fq(a, pw, lin.bias)  # noqa: E731
        quant = lambda: ops.quant_act_fp(x, pw, args.act, 4, G)  # noqa: E731
        kdt = "f16"
    for _ in range(max(3, args.warmup)):
        gemm()
    gemm_ms = time_events(gemm, max(10, args.steps), stream)
    quant_ms = time_events(quant, max(10, args.steps), stream)
    achieved = flops / (gemm_ms * 1e-3) / 1e12
    # reference point: the vendor dense fp16 GEMM (hipBLASLt via torch) on the same shape,
    # unquantized -- what the reference's F.linear costs on this GPU, without any act-quant
    wd = lin.weight.detach()
    dense = lambda: torch.nn.functional.linear(x, wd, lin.bias)  # noqa: E731
    for _ in range(max(3, args.warmup)):
        dense()
    dense_ms = time_events(dense, max(10, args.steps), stream)
    # reference point: the reference's own fake-quant forward (restated in PyTorch ops,
    # tools/torch_fakequant.py) on this GPU, same layer and input
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from torch_fakequant import TorchFakeQuantLinear
    ref = TorchFakeQuantLinear(q.weight, lin.bias.detach(), q.salient_indices, args.act, 4, G)
    y_ref, y_ours = ref(x), q(x.clone())
    ref_rel = float((y_ref.float() - y_ours.float()).norm() / y_ref.float().norm())
    ref_ms = time_events(lambda: ref(x), max(5, args.steps // 5), stream)
    # prepass algorithmic bytes: read x (colmax) + read x (quantize) + write operand(s)
    xbytes = M * K * 2
    if use_i8 or use_f8:
        wbytes = M * pw.Kp + M * 4 + M * pw.S_pad * 2
        reads = 2 if args.act == "per_tensor" else 1
    else:
        wbytes = M * (pw.Kp + pw.S_pad) * 2
        reads = 2 if args.act in ("per_group", "per_tensor") else 1
    prepass_bytes = reads * xbytes + wbytes

    traffic = None
    prof = os.path.join(ROOT, "profiles", f"pmc_gemm_{kdt}_{args.act}.json")
    if os.path.exists(prof):
        try:
            traffic = json.load(open(prof)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": "quantized-Linear TFLOP/s (W4A4Linear 4096x4096, G=128, 10% salient, bs*seq=16384)",
        "value": round(value, 2),
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "e4m3 codes (fp32 accumulate) + fp16 salient tail" if use_f8 else "fp16",
        "data": "synthetic (random-init weights N(0,0.02^2), x N(0,1) with 1% outlier channels x30)",
        "config": {
            "workload": (f"W4A4Linear.forward: weight per_group(sorted) int4 + act {args.act} "
                         f"{'(sorted) ' if args.act == 'per_group' else ''}4-bit, "
                         f"{int(P * 100)}% salient fp16 side-GEMM"),
            "M": M, "K": K, "N": N, "group_size": G, "salient_prop": P,
            "salient_channels": pw.S,
            "kernel": "gemm_f8" if use_f8 else "gemm_i8" if use_i8 else "gemm_fq",
            "parallelism": f"replicas x{world}",
        },
        "roofline": {
            "bound": "mfma",
            "achieved": round(achieved, 1),
            "peak": PEAK_TFLOPS[kdt],
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_TFLOPS[kdt], 4),
            "traffic": traffic,
            "kernel": ("sqmp::gemm_f8_kernel<F16> (e4m3 block-scaled MFMA)" if use_f8 else
                       "sqmp::gemm_i8v2_kernel<F16>" if use_i8 else "sqmp::gemm_fq6_kernel<F16,1>"),
            "avg_ms": round(gemm_ms, 4),
            "algorithmic_flops_per_launch": flops,
        },
        "reference_points": {
            "reference_fakequant_forward_ms": round(ref_ms, 4),
            "reference_fakequant_TFLOP_per_s": round(flops / (ref_ms * 1e-3) / 1e12, 1),
            "speedup_vs_reference_fakequant": round(ref_ms / ms_per_step, 2),
            "reference_vs_ours_rel_err": ref_rel,
            "torch_fp16_linear_ms": round(dense_ms, 4),
            "torch_fp16_linear_TFLOP_per_s": round(flops / (dense_ms * 1e-3) / 1e12, 1),
            "note": "reference fake-quant forward restated in PyTorch ops (tools/torch_fakequant.py) on "
                    "this GPU; fp16 F.linear = unquantized hipBLASLt GEMM of the same shape",
        },
        "prepass": {
            "avg_ms": round(quant_ms, 4),
            "algorithmic_bytes": prepass_bytes,
            "GB_per_s": round(prepass_bytes / (quant_ms * 1e-3) / 1e9, 1),
            "hbm_peak_GB_per_s": HBM_PEAK_GBS,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_rows, args.act)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
