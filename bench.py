"""Benchmark of the W4A4 mixed-precision linear on MI355X (BASELINE.json config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--act per_group|per_token]

A "step" is one W4A4Linear.forward over one synthetic batch resident in HBM:
W4A4Linear(4096, 4096), weight per_group (sorted) int4, G=128, 10% salient channels,
x[bs*seq = 16384, 4096] fp16 -- activation quantization (column absmax over the batch,
stable sort, per-(row, group) scales) + the mixed-precision MFMA GEMM with the salient
fp16 side-GEMM.  `value` is whole-job TFLOP/s = N_gpus * 2*M*N*K / max-over-ranks time.

Multi-GPU: the op is per-layer and does not shard ("replicas only"): each
rank runs an independent replica on its own GPU; the only collectives are the timing
barriers and the max-over-ranks of the elapsed time.  `--gpus N` without a
torch.distributed.run environment starts one as a child process (nothing touches the
GPU before that) and exits with its status.

Also printed in the same JSON line:
  roofline      the dominant kernel (the GEMM), timed live with HIP events on the stream
                it runs on; achieved = 2*M*N*K / average GEMM duration; `peak` = the
                north star's int8-MFMA roofline as a rate, 2*M*N*K / T_roof with BASELINE.md
                §2's T_roof = 2MNK'/P_i8 + 2MNS/P_f16 (about 120 us: the int4 contraction on
                the int8 MFMA, the salient columns on the f16 MFMA), so `frac` = T_roof / GEMM
                time = the "fraction of the int8-MFMA roofline"; `frac_dtype_peak` = achieved
                / the dense MFMA peak of the dtype the kernel computes in (f16 for the
                faithful per_group kernel, whose exact operands rule out the int8 MFMA:
                SURVEY.md §7 hard part 1); `frac_contract_step` = T_roof / step time
  cpu_baseline  the reference's fake-quant layer restated in PyTorch ops (oracle/
                torch_cpu.py, pinned bit-exact to the reference goldens) in fp32 on this
                host's cores: rank 0, N=1 only, median of 3 after 1 warm-up
  prepass       the activation-quantization kernels' time and algorithmic GB/s
  llama_layer   BASELINE config 4's workload: one Llama-2-7B decoder layer's 7 linears at
                2048 tokens (G=64, 5 % salient), W4A4 vs unquantized fp16 F.linear, per
                linear and in total (measured after the timed region)
  per_token     the same layer with per_token 4-bit activations (the FP8 GEMM)
  fp32          the same layer in fp32 (config 3's dtype): step, h2d GEMM, fraction of the
                three-product f16 floor, counter traffic of the same library
  e2e           the metric's Llama-2-7B W4A4 tokens/s (bench_e2e.run: 32 layers, random-init
                fp16 weights, 8 x 2048-token windows, batch 1) next to unquantized fp16, the
                reference fake-quant forward on the GPU, PPL deltas, and the torch-CPU fp32
                baseline (extrapolated from 1 and 2 layers, cores stated)
Secondary measurements (GEMM alone, prepass, vendor dense GEMM, reference fake-quant on
the GPU) run BEFORE the W warm-up steps, followed by --settle-ms (default 300) of untimed
steps, so the timed region starts on a chip that holds the clock it settles at under this
load whatever W is (DVFS: a 20-step run right after a short warm-up measured the GEMM at
510-680 us in its first milliseconds, 445 us once settled -- profiles/r02_bench_driver20_*).
The timed region is still exactly K steps between barriers.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

M, K, N, G, P = 16384, 4096, 4096, 128, 0.10
# dense MFMA peaks (MI355X_MICROARCH.md: 256 CU @ 2.4 GHz): f16/bf16 2.5 PF, i8/fp8 5 PF,
# (fp6/fp4 10 PF: no kernel here)
PEAK_TFLOPS = {"f16": 2516.6, "bf16": 2516.6, "i8": 5033.2, "f8": 5033.2,
               "f32": 157.3}
HBM_PEAK_GBS = 8000.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--act", default="per_group", choices=["per_group", "per_token"])
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed steps run for this long before the W warm-up steps")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "fp32"],
                    help="model dtype of the layer (fp32: the reference's OPT dtype; the GEMM "
                         "runs on the f16 MFMA as sqmp_gemm_h2)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-layer", action="store_true",
                    help="skip the secondary lines (per_token, llama_layer, fp32, e2e)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end Llama-2-7B leg")
    ap.add_argument("--e2e-windows", type=int, default=8)
    ap.add_argument("--rehearsal", action="store_true",
                    help="CPU/gloo rehearsal of the launcher and timing path (no GPU): the "
                         "step is the CPU fake-quant layer on a 64-row batch")
    return ap.parse_args(argv)


def contract_roofline_s(S: int) -> float:
    """T_roof = 2*M*N*K'/P_i8 + 2*M*N*S/P_f16 (seconds)."""
    return (2.0 * M * N * (K - S) / (PEAK_TFLOPS["i8"] * 1e12)
            + 2.0 * M * N * S / (PEAK_TFLOPS["f16"] * 1e12))


# ------------------------------------------------------------------ launcher / dist
def launch_children(args, argv) -> int:
    """Start `torch.distributed.run` with one rank per GPU as a child process (never an
    exec of this process) and return its exit status."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def setup_dist(n, backend="nccl"):
    """One process per GPU (torch.distributed.run env); backend "nccl" is RCCL on ROCm,
    "gloo" the CPU rehearsal."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n:
        raise RuntimeError(f"--gpus {n} but WORLD_SIZE={world}")
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


# ------------------------------------------------------------------ workload
def synthetic_layer(gen, dev, dtype):
    """W ~ N(0, 0.02^2), b ~ N(0, 0.01^2), x ~ N(0, 1) with 1% outlier channels x30, and
    the importance = mean|x| of a separate 2048-row calibration batch."""
    W = torch.randn(N, K, generator=gen, device=dev) * 0.02
    b = torch.randn(N, generator=gen, device=dev) * 0.01
    outl = torch.randperm(K, generator=gen, device=dev)[: K // 100]
    x = torch.randn(M, K, generator=gen, device=dev)
    x[:, outl] *= 30.0
    cal = torch.randn(2048, K, generator=gen, device=dev)
    cal[:, outl] *= 30.0
    imp = cal.abs().mean(0).cpu()
    return W.to(dtype), b.to(dtype), x.to(dtype), imp


def make_layer(dev, act, seed, dtype=torch.float16):
    from smoothquant.fake_quant import W4A4Linear
    gen = torch.Generator(device=dev).manual_seed(seed)
    W, b, x, imp = synthetic_layer(gen, dev, dtype)
    lin = torch.nn.Linear(K, N, bias=True).to(dev, dtype)
    with torch.no_grad():
        lin.weight.copy_(W)
        lin.bias.copy_(b)
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act, importance=imp,
                              salient_prop=P, quant_bits=4, group_size=G)
    return q, x, lin


def time_events(fn, iters, stream):
    """Average ms per call, HIP events recorded on `stream` (the stream the kernels of
    `fn` are launched on)."""
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record(stream)
    for _ in range(iters):
        fn()
    end.record(stream)
    end.synchronize()
    return start.elapsed_time(end) / iters


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CORES_NOTE = ("cores = the torch intra-op threads used = this job's CPU share on the GPU box "
              "(the lease sets OMP_NUM_THREADS=16 and its rules size worker pools to that share: "
              "os.cpu_count() / the process affinity show the whole shared machine, whose other "
              "CPUs serve other jobs), so the baseline runs on every core the job may use")


def cpu_baseline(act, rows=M, runs=3):
    """The reference's fake-quant layer on PyTorch-CPU (oracle/torch_cpu.py, pinned
    bit-exact to the reference goldens), fp32 as in the reference's CPU scripts, every
    thread torch uses on this host: 1 warm-up + median of `runs` forwards."""
    from oracle.torch_cpu import CPUFakeQuantLinear
    gen = torch.Generator().manual_seed(1234)
    W, b, x, imp = synthetic_layer(gen, "cpu", torch.float32)
    x = x[:rows].contiguous()
    layer = CPUFakeQuantLinear(W, b, "per_group", act, 4, G, imp, P)
    layer(x)  # warm-up
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        layer(x)
        ts.append(time.perf_counter() - t0)
    dt = statistics.median(ts)
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {
        "value": round(2.0 * rows * N * K / dt / 1e12, 4),
        "unit": "TFLOP/s",
        "cores": torch.get_num_threads(),
        "host_cpu_count": os.cpu_count(),
        "process_affinity_cpus": affinity,
        "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
        "cores_note": CORES_NOTE,
        "kind": "torch-cpu-fp32",
        "cpu_model": cpu_model(),
        "sample": (f"oracle/torch_cpu.py CPUFakeQuantLinear (the reference's fake_quant ops, "
                   f"bit-exact to its goldens), fp32, weight per_group + act {act}, "
                   f"{rows}x{K}->{N}, G={G}, p={P}; median of {runs} after 1 warm-up: "
                   f"{dt:.3f} s per forward (runs {', '.join(f'{t:.3f}' for t in ts)})"),
    }


def lib_sha1() -> str:
    """sha1 of the product library (tools/pmc_summary.py records it in each profile)."""
    import hashlib
    path = os.path.join(ROOT, "smoothquant-mixedprecision_amd", "smoothquant", "libsqmp_w4a4.so")
    try:
        with open(path, "rb") as f:
            return hashlib.sha1(f.read()).hexdigest()
    except OSError:
        return ""


def pick_traffic(pname: str, live_us: float, tol: float = 0.05, tol_same: float = 0.15):
    """HBM bytes per launch of the timed kernel from a committed counter profile
    (profiles/r0N*_<pname>, tools/pmc_summary.py): a profile of THIS library build (its
    lib_sha1) whose profiled median kernel duration is within `tol_same` of the live HIP-event
    average (counter collection lowers the clock: 1.76-1.94 GHz profiled vs about 2.0-2.1
    live, MI355X_MICROARCH.md "DVFS give-back"), else the newest profile of another build
    within `tol`.  Returns (bytes or None, {file, avg_kernel_us, live, accepted})."""
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*_" + pname)))
    lib = lib_sha1()
    info, rows = None, []
    for prof in reversed(cands):
        try:
            with open(prof) as f:
                j = json.load(f)
        except (OSError, ValueError):
            continue
        us = j.get("avg_kernel_us")
        same = bool(lib) and j.get("lib_sha1") == lib
        ok = bool(us) and abs(us - live_us) <= (tol_same if same else tol) * live_us
        cur = {"file": os.path.relpath(prof, ROOT), "avg_kernel_us": us,
               "live_avg_us": round(live_us, 2), "accepted": ok, "same_library": same}
        if info is None:
            info = cur  # the newest, reported even when rejected
        rows.append((cur, j))
    # a profile of this very library build first, then the newest within the tolerance
    for want_same in (True, False):
        for cur, j in rows:
            if cur["accepted"] and (cur["same_library"] or not want_same):
                return j.get("hbm_bytes_per_launch"), cur
    if info is not None:
        info["note"] = (f"no committed profile of this build within {tol_same:.0%} (or of another "
                        f"build within {tol:.0%}) of the live kernel time: traffic null")
    return None, info


# ------------------------------------------------------------------ Llama-2-7B layer
# BASELINE config 4's linears (the north star's end-to-end workload): one decoder layer of
# Llama-2-7B at 2048 tokens (one prefill window), G=64, 5 % salient, max-sorted per_group
# weights and activations, fp16.  The 7 linears run in the order a LlamaDecoderLayer calls
# them, q/k/v on one input object and gate/up on another, so k, v and up reuse the column
# statistics of their sibling (fake_quant.py:479-561 swaps them one by one; the reference
# recomputes the identical sort per layer).
LLAMA_LINEARS = [  # name, K, N, input
    ("q_proj", 4096, 4096, "attn"), ("k_proj", 4096, 4096, "attn"),
    ("v_proj", 4096, 4096, "attn"), ("o_proj", 4096, 4096, "o"),
    ("gate_proj", 4096, 11008, "mlp"), ("up_proj", 4096, 11008, "mlp"),
    ("down_proj", 11008, 4096, "down"),
]
LLAMA_T, LLAMA_G, LLAMA_P = 2048, 64, 0.05


def llama_layer(dev, iters=40, flow="experiments"):
    """Per-linear and whole-layer time of the W4A4 layer against the same 7 unquantized
    F.linear calls (hipBLASLt), HIP events on the launch stream.  flow "experiments": config 4
    (fp16, per_group sorted W and A, G 64, 5 % salient; run_experiments.py); "ppl_eval": the
    reference's SmoothQuant baseline evaluation (smoothquant/ppl_eval.py:69-83: bf16,
    quantize_model with per_channel W, per_token A, quantize_bmm_input=True, no salient
    channels -- each linear quantizes its input in place, q/k/v their outputs); "token":
    quantize_llama_like's defaults (fp16, per_channel W, per_token A in place, no salient
    channels, no output quantization)."""
    from smoothquant.fake_quant import W4A4Linear, link_siblings
    gen = torch.Generator(device=dev).manual_seed(7)
    ppl = flow in ("ppl_eval", "token")
    dt = torch.bfloat16 if flow == "ppl_eval" else torch.float16
    xs = {}
    for name, K in (("attn", 4096), ("o", 4096), ("mlp", 4096), ("down", 11008)):
        x = torch.randn(LLAMA_T, K, generator=gen, device=dev)
        x[:, torch.randperm(K, generator=gen, device=dev)[: K // 100]] *= 30.0
        xs[name] = x.to(dt)
    layers = []
    for name, K, N, src in LLAMA_LINEARS:
        lin = torch.nn.Linear(K, N, bias=False).to(dev, dt)
        with torch.no_grad():
            lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).to(dt))
        if ppl:
            q = W4A4Linear.from_float(lin, weight_quant="per_channel", act_quant="per_token",
                                      quantize_output=(flow == "ppl_eval" and
                                                       name in ("q_proj", "k_proj", "v_proj")))
        else:
            imp = xs[src][:512].float().abs().mean(0).cpu()
            q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                                      importance=imp, salient_prop=LLAMA_P, group_size=LLAMA_G)
        layers.append((name, q, lin.weight.detach(), src))
    # the sibling groups quantize_llama_like links (q/k/v, gate/up: fake_quant.SiblingGroup)
    link_siblings(*[layers[i][1] for i in (0, 1, 2)])
    link_siblings(*[layers[i][1] for i in (4, 5)])
    stream = torch.cuda.current_stream(dev)
    # per_token without salient channels quantizes its input in place (as the reference): the
    # W4A4 passes start from fresh copies of the unquantized inputs (restored before the pass's
    # first event, outside the timed span), and the unquantized F.linear calls always read the
    # originals -- a GEMM on already-quantized activations draws less power and runs faster
    work = {k: v.clone() for k, v in xs.items()} if ppl else xs

    def run(fp16, ev=None):
        if ppl and not fp16:
            for k, v in xs.items():
                work[k].copy_(v)
        if ev is not None:
            ev[0].record(stream)
        for i, (_, q, w, src) in enumerate(layers):
            if fp16:
                torch.nn.functional.linear(xs[src], w)
            else:
                q(work[src])
            if ev is not None:
                ev[i + 1].record(stream)

    out = {}
    for kind in (False, True, False, True):  # interleaved rounds, best of each
        for _ in range(5):
            run(kind)
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(len(layers) + 1)]
               for _ in range(iters)]
        for ev in evs:
            run(kind, ev)
        evs[-1][-1].synchronize()
        per = [sorted(ev[i].elapsed_time(ev[i + 1]) for ev in evs)[iters // 2]
               for i in range(len(layers))]
        tot = sorted(ev[0].elapsed_time(ev[-1]) for ev in evs)[iters // 2]
        key = "fp16" if kind else "w4a4"  # ("fp16": the unquantized model dtype)
        if key not in out or tot < out[key][1]:
            out[key] = (per, tot)
    flops = sum(2.0 * LLAMA_T * K * N for _, K, N, _ in LLAMA_LINEARS)
    (pw4, tw4), (pf16, tf16) = out["w4a4"], out["fp16"]
    if ppl:
        u = "bf16" if flow == "ppl_eval" else "fp16"
        return {
            "workload": (f"Llama-2-7B decoder layer linears, {LLAMA_T} tokens, the reference's "
                         "ppl_eval flow: bf16, W4 per_channel, A4 per_token (in place), q/k/v "
                         "outputs quantized per_token, no salient channels"
                         if flow == "ppl_eval" else
                         f"Llama-2-7B decoder layer linears, {LLAMA_T} tokens, "
                         "quantize_llama_like's defaults: fp16, W4 per_channel, A4 per_token (in "
                         "place), no salient channels, no output quantization"),
            "w4a4_ms": round(tw4, 4), f"{u}_linear_ms": round(tf16, 4),
            f"w4a4_over_{u}_speed": round(tf16 / tw4, 4),
            "w4a4_TFLOP_per_s": round(flops / (tw4 * 1e-3) / 1e12, 1),
            "per_linear": {name: {"w4a4_ms": round(a, 4), f"{u}_ms": round(b, 4),
                                  f"{u}_over_w4a4": round(b / a, 3)}
                           for (name, _, _, _), a, b in zip(LLAMA_LINEARS, pw4, pf16)},
            "note": "median of 40 layer passes, best of 2 interleaved rounds; every input is "
                    "quantized in place by its layer, as in the reference: each W4A4 pass starts "
                    "from fresh copies of the unquantized inputs (copied before the pass's first "
                    "event), the unquantized F.linear calls read the originals",
        }
    return {
        "workload": (f"Llama-2-7B decoder layer linears, {LLAMA_T} tokens, W4A4 G={LLAMA_G}, "
                     f"{int(LLAMA_P * 100)}% salient, per_group(sorted) W and A, fp16; "
                     "q/k/v and gate/up share their input (sibling statistics reuse)"),
        "w4a4_ms": round(tw4, 4), "fp16_linear_ms": round(tf16, 4),
        "w4a4_over_fp16_speed": round(tf16 / tw4, 4),
        "w4a4_TFLOP_per_s": round(flops / (tw4 * 1e-3) / 1e12, 1),
        "per_linear": {name: {"w4a4_ms": round(a, 4), "fp16_ms": round(b, 4),
                              "fp16_over_w4a4": round(b / a, 3)}
                       for (name, _, _, _), a, b in zip(LLAMA_LINEARS, pw4, pf16)},
        # the sibling groups as units (their first member's time covers the whole group)
        "per_group": {g: {"w4a4_ms": round(sum(pw4[i] for i in ix), 4),
                          "fp16_ms": round(sum(pf16[i] for i in ix), 4),
                          "fp16_over_w4a4": round(sum(pf16[i] for i in ix) / sum(pw4[i] for i in ix), 3)}
                      for g, ix in (("qkv", (0, 1, 2)), ("o", (3,)), ("gate_up", (4, 5)),
                                    ("down", (6,)))},
        "note": "median of 40 layer passes, best of 2 interleaved rounds; q/k/v and gate/up are "
                "linked sibling groups (as quantize_llama_like links them): the first member's "
                "time covers the group's one quantizer pass and one GEMM launch, the others "
                "return the outputs it computed",
    }


def per_token_leg(dev, iters=200):
    """The per_token act mode of the same config-2 layer (BASELINE configs' per_token rows; the
    reference's per_token path, fake_quant.py:64-90): W4A4Linear.forward on the auto kernel
    (e4m3 codes on the block-scaled FP8 MFMA, sqmp_gemm_f8), step and GEMM timed with HIP
    events on the launch stream; frac against the dense FP8 MFMA peak."""
    from smoothquant import ops
    q, x, lin = make_layer(dev, "per_token", seed=4321)
    pw = q.packed()
    stream = torch.cuda.current_stream(dev)
    flops = 2.0 * M * N * K
    use_f8 = ops.f8_auto(pw, "per_token", 4)
    if use_f8:
        a8, sa, xs = ops.quant_act_f8(x, pw, "per_token", 4)
        gemm = lambda: ops.gemm_f8(a8, sa, xs, pw, lin.bias)  # noqa: E731
        quant = lambda: ops.quant_act_f8(x, pw, "per_token", 4)  # noqa: E731
        kdt = "f8"
    else:
        a = ops.quant_act_fp(x, pw, "per_token", 4, G)
        gemm = lambda: ops.gemm_fq(a, pw, lin.bias)  # noqa: E731
        quant = lambda: ops.quant_act_fp(x, pw, "per_token", 4, G)  # noqa: E731
        kdt = "f16"
    step = lambda: q(x)  # noqa: E731
    for fn in (gemm, quant, step):
        for _ in range(20):
            fn()
    gemm_ms = time_events(gemm, iters, stream)
    quant_ms = time_events(quant, iters, stream)
    step_ms = time_events(step, iters, stream)
    achieved = flops / (gemm_ms * 1e-3) / 1e12
    return {
        "workload": "the config-2 layer with act per_token (4-bit, per-row absmax), weight "
                    "per_group(sorted), 10% salient",
        "kernel": ("sqmp_gemm_f8 (e4m3 codes, block-scaled FP8 MFMA) + fp16 salient tail"
                   if use_f8 else "sqmp_gemm_fq (fp16 D values)"),
        "ms_per_step": round(step_ms, 4),
        "TFLOP_per_s": round(flops / (step_ms * 1e-3) / 1e12, 1),
        "gemm_avg_ms": round(gemm_ms, 4),
        "gemm_TFLOP_per_s": round(achieved, 1),
        "peak": PEAK_TFLOPS[kdt],
        "frac": round(achieved / PEAK_TFLOPS[kdt], 4),
        "prepass_avg_ms": round(quant_ms, 4),
        "note": "HIP events, 200 back-to-back calls each after 20 warm-up; frac = GEMM "
                "achieved / dense peak of the kernel's MFMA dtype (FP8 5033 TFLOP/s)",
    }


def fp32_leg(dev, iters=100):
    """BASELINE config 3's dtype (the reference runs OPT in fp32, run_experiments.py:152-154) on
    the config-2 layer: W4A4Linear.forward in fp32 (the quantizer writes the two f16 planes,
    sqmp_gemm_h2d runs 3 f16 MFMAs per product); step and GEMM timed with HIP events on the
    launch stream.  floor_frac = the three-product f16 floor (3 x 2MN(Kp + S_pad) / P_f16) /
    GEMM time; traffic from the committed counter profile of the same library."""
    from smoothquant import ops
    q, x, lin = make_layer(dev, "per_group", seed=777, dtype=torch.float32)
    pw = q.packed()
    stream = torch.cuda.current_stream(dev)
    flops = 2.0 * M * N * K
    if not ops.h2_planes_ok(pw, "per_group", M, G):
        return {"note": "the fp32 planes path does not take this layer"}
    a2 = ops.quant_act_fp(x, pw, "per_group", 4, G, h2=True)
    gemm = lambda: ops.gemm_h2_planes(a2, pw, lin.bias)  # noqa: E731
    step = lambda: q(x)  # noqa: E731
    for fn in (gemm, step):
        for _ in range(10):
            fn()
    gemm_ms = time_events(gemm, iters, stream)
    step_ms = time_events(step, iters, stream)
    floor_s = 3 * 2.0 * M * N * (pw.Kp + pw.S_pad) / (PEAK_TFLOPS["f16"] * 1e12)
    traffic, tprof = pick_traffic("pmc_gemm_h2d_fp32.json", gemm_ms * 1e3)
    alg = M * (pw.Kp + pw.S_pad) * 4 + N * (pw.Kp + pw.S_pad) * 4 + M * N * 4
    return {
        "workload": "the config-2 layer in fp32 (weight per_group(sorted) int4 + act per_group "
                    "4-bit, 10% salient), the reference's OPT dtype",
        "kernel": "sqmp::h2d::gemm_h2d_kernel (row-scaled two-piece fp16 planes, 3 f16 MFMAs "
                  "per product, fp32 accumulation)",
        "ms_per_step": round(step_ms, 4),
        "TFLOP_per_s": round(flops / (step_ms * 1e-3) / 1e12, 1),
        "gemm_avg_ms": round(gemm_ms, 4),
        "gemm_TFLOP_per_s": round(flops / (gemm_ms * 1e-3) / 1e12, 1),
        "floor_frac": round(floor_s / (gemm_ms * 1e-3), 4),
        "three_product_floor_ms": round(floor_s * 1e3, 4),
        "algorithmic_bytes": alg,
        "traffic": traffic,
        "traffic_over_algorithmic": None if not traffic else round(traffic / alg, 2),
        "traffic_profile": tprof,
        "note": "HIP events, 100 back-to-back calls each after 10 warm-up",
    }


def e2e_leg(windows=8, cpu=True):
    """BASELINE config 4 end to end (the metric's Llama-2-7B W4A4 tokens/s): bench_e2e.run on
    the Llama-2-7B architecture with random-init fp16 weights on the device, G=64, 5 % salient,
    per_group(sorted) weights and activations (quantize_llama_like), batch 1, `windows` windows
    of 2048 tokens (the reference's Evaluator, run_experiments.py:86-123): W4A4, unquantized
    fp16, the reference's fake-quant forward restated in PyTorch ops on the GPU (fp16 GEMM and
    fp32 GEMM: the PPL noise of its own accumulation order), and the torch-CPU fp32 baseline
    extrapolated from 1 and 2 decoder layers."""
    import bench_e2e
    args = bench_e2e.parse(["--model", "llama2-7b", "--windows", str(windows), "--rounds", "2"]
                           + ([] if cpu else ["--no-cpu"]))
    r = bench_e2e.run(args)
    torch.cuda.empty_cache()
    cpu = r.get("cpu_baseline")
    if cpu is not None:
        cpu = dict(cpu, cores_note=CORES_NOTE)
    return {
        "workload": (f"Llama-2-7B prefill (32 layers, random-init fp16 weights on the device), "
                     f"W4A4 G={r['config']['group_size']}, {int(r['config']['salient_prop'] * 100)}% "
                     f"salient, per_group(sorted) W and A (quantize_llama_like), batch 1, "
                     f"{windows} x {r['config']['seq_len']}-token windows"),
        "w4a4_tokens_per_s": r["value"],
        "fp16_tokens_per_s": r["unquantized_tokens_per_s"],
        "w4a4_over_fp16": r["w4a4_over_unquantized"],
        "reference_fakequant_gpu_tokens_per_s": r.get("reference_fakequant_tokens_per_s"),
        "speedup_vs_reference_fakequant": r.get("speedup_vs_reference_fakequant"),
        "ppl_w4a4": r["ppl_w4a4"], "ppl_fp16": r["ppl_unquantized"],
        "ppl_delta_vs_fp16": round(r["ppl_w4a4"] - r["ppl_unquantized"], 4),
        "ppl_reference_fakequant": r.get("ppl_reference_fakequant"),
        "ppl_delta_vs_reference": r.get("ppl_delta_vs_reference"),
        "reference_gemm_order_noise": r.get("reference_gemm_order_noise"),
        "cpu_baseline": cpu,
        "setup_s": r.get("setup_s"),
        "note": "PPL of a random-init model (~ vocab size): only differences mean anything; the "
                "W4A4 delta vs the reference fake-quant reads against the reference's own "
                "fp16-vs-fp32-GEMM difference (reference_gemm_order_noise)",
    }


# ------------------------------------------------------------------ rehearsal (CPU)
def rehearsal(args, rank, world):
    """The launcher / barrier / max-over-ranks / report path on CPU with gloo: the step is
    the CPU fake-quant layer on a 64-row batch of the config-2 layer."""
    from oracle.torch_cpu import CPUFakeQuantLinear
    gen = torch.Generator().manual_seed(1234 + rank)
    W, b, x, imp = synthetic_layer(gen, "cpu", torch.float32)
    layer = CPUFakeQuantLinear(W[:256], b[:256], "per_group", args.act, 4, G, imp, P)
    xs = x[:64].contiguous()
    for _ in range(args.warmup):
        layer(xs)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        layer(xs)
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, torch.device("cpu"))
    flops = 2.0 * 64 * 256 * K
    return {"metric": "rehearsal (CPU/gloo launcher check; not a measurement)",
            "value": round(job_tflops(world, flops, args.steps, elapsed), 6),
            "unit": "TFLOP/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4)}


# ------------------------------------------------------------------ main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_children(args, argv)
    rank, world, local = setup_dist(args.gpus, "gloo" if args.rehearsal else "nccl")
    if args.rehearsal:
        out = rehearsal(args, rank, world)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return 0

    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from smoothquant import ops

    fp32 = args.dtype == "fp32"
    q, x, lin = make_layer(dev, args.act, seed=1234 + rank,
                           dtype=torch.float32 if fp32 else torch.float16)
    pw = q.packed()
    # what W4A4Linear(kernel="auto") runs for this layer
    use_f8 = ops.f8_auto(pw, args.act, 4)
    use_fqt = not use_f8 and ops.fqt_eligible(pw, args.act, 4, G, M)
    stream = torch.cuda.current_stream(dev)
    flops = 2.0 * M * N * K

    # ---- secondary measurements first, slowest-to-settle last: the reference fake-quant
    # forward (PyTorch ops), the vendor dense GEMM, then ~0.1 s of back-to-back W4A4
    # GEMMs right before the warm-up, so the timed region starts at the clock the chip
    # holds under this load (DVFS, MI355X_MICROARCH.md; a kernel trace of a 20-step run
    # shows the GEMM at 510-680 us in its first milliseconds, 480 us once settled)
    sec_iters = max(200, args.steps)  # ~0.1 s of back-to-back GEMMs, whatever --steps is
    # the reference's own fake-quant forward (PyTorch ops, tools/torch_fakequant.py) on
    # this GPU, same layer and input
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from torch_fakequant import TorchFakeQuantLinear
    ref = TorchFakeQuantLinear(q.weight, lin.bias.detach(), q.salient_indices, args.act, 4, G)
    y_ref, y_ours = ref(x), q(x.clone())
    ref_rel = float((y_ref.float() - y_ours.float()).norm() / y_ref.float().norm())
    del y_ref, y_ours
    ref_ms = time_events(lambda: ref(x), max(20, args.steps // 5), stream)

    # vendor dense fp16 GEMM (hipBLASLt via torch) on the same shape, unquantized: what
    # the reference's F.linear costs on this GPU, without any act-quant
    wd = lin.weight.detach()
    dense = lambda: torch.nn.functional.linear(x, wd, lin.bias)  # noqa: E731
    for _ in range(10):
        dense()
    dense_ms = time_events(dense, sec_iters, stream)
    # dominant kernel: the GEMM, timed alone on the stream it is launched on
    if use_f8:
        a8, sa, xs = ops.quant_act_f8(x, pw, args.act, 4)
        gemm = lambda: ops.gemm_f8(a8, sa, xs, pw, lin.bias)  # noqa: E731
        quant = lambda: ops.quant_act_f8(x, pw, args.act, 4)  # noqa: E731
        kdt = "f8"
        kname = ("sqmp::gemm_f8v2_kernel<F16> (e4m3 on v_mfma_scale_f32_16x16x128_f8f6f4)"
                 if pw.Gw % 128 == 0 else
                 "sqmp::gemm_f8_kernel<F16> (e4m3 on v_mfma_scale_f32_32x32x64_f8f6f4)")
    elif use_fqt:
        c4 = ops.quant_act_c4(x, pw, args.act, 4, G)
        gemm = lambda: ops.gemm_fqt(*c4, pw, lin.bias, G)  # noqa: E731
        quant = lambda: ops.quant_act_c4(x, pw, args.act, 4, G)  # noqa: E731
        kdt = "f16"
        kname = ("sqmp::fq7::gemm_fq7_kernel<F16,1,256,2,0,true,3> (activation order, sqmp_gemm_fqt7)"
                 if c4[1].dim() == 3 else
                 "sqmp::gemm_fq6_kernel<F16,1,256,true> (activation order, sqmp_gemm_fqt)")
    elif fp32 and ops.h2_planes_ok(pw, args.act, M):
        # the forward's fp32 path: the quantizer writes the two f16 planes, sqmp_gemm_h2d
        a2 = ops.quant_act_fp(x, pw, args.act, 4, G, h2=True)
        gemm = lambda: ops.gemm_h2_planes(a2, pw, lin.bias)  # noqa: E731
        quant = lambda: ops.quant_act_fp(x, pw, args.act, 4, G, h2=True)  # noqa: E731
        kdt = "f32"
        kname = ("sqmp::h2d::gemm_h2d_kernel<false,128> (sqmp_gemm_h2d: row-scaled two-piece "
                 "fp16 planes by LDS-DMA, 3 f16 MFMAs per product)")
    else:
        a = ops.quant_act_fp(x, pw, args.act, 4, G)
        gemm = lambda: ops.gemm_fq(a, pw, lin.bias)  # noqa: E731
        quant = lambda: ops.quant_act_fp(x, pw, args.act, 4, G)  # noqa: E731
        kdt, kname = "f16", ("sqmp::fq7::gemm_fq7_kernel<F16,1,256,2> (weights in registers)"
                             if ops.FQ7_AUTO and ops.fq7_eligible(pw)
                             else "sqmp::gemm_fq6_kernel<F16,1,256>")
        if fp32:
            kdt = "f32"
            kname = ("sqmp::gemm_x3_kernel<H=true> (sqmp_gemm_h2: row-scaled two-piece fp16 "
                     "splits, 3 f16 MFMAs per product)")
    quant_ms = time_events(quant, sec_iters, stream)
    for _ in range(10):
        gemm()
    gemm_ms = time_events(gemm, sec_iters, stream)
    # ---- the timed region: W warm-up steps, then exactly K steps
    def step():
        return q(x)

    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        for _ in range(10):
            step()
        torch.cuda.synchronize(dev)
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
    value = job_tflops(world, flops, args.steps, elapsed)

    achieved = flops / (gemm_ms * 1e-3) / 1e12
    t_roof = contract_roofline_s(pw.S)
    # prepass algorithmic bytes: read x (stats) + read x (quantize) + write the operand(s)
    esz = 4 if fp32 else 2
    xbytes = M * K * esz
    if use_f8:
        wbytes = M * pw.Kp + M * 4 + M * pw.S_pad * 2
        reads = 2 if args.act == "per_tensor" else 1
    elif use_fqt:
        Kq = (K - pw.S + 63) // 64 * 64
        # act codes + group scales + exact salient x, then the permuted weight (write) from
        # the packed codes (read)
        wbytes = (M * Kq // 2 + M * (Kq // G) * 2 + M * pw.S_pad * 2
                  + N * (Kq + pw.S_pad) * 2 + N * pw.Kp // 2)
        reads = 2
    else:
        wbytes = M * (pw.Kp + pw.S_pad) * esz
        reads = 2 if args.act in ("per_group", "per_tensor") else 1
    prepass_bytes = reads * xbytes + wbytes

    pname = ("pmc_gemm_f8v2_per_token.json" if kdt == "f8"
             else "pmc_gemm_h2d_fp32.json" if fp32 and "h2d" in kname
             else "pmc_gemm_h2_fp32.json" if fp32
             else "pmc_gemm_fqt7_per_group.json" if use_fqt and "fqt7" in kname
             else "pmc_gemm_fqt_per_group.json" if use_fqt
             else f"pmc_gemm_fq6_{args.act}.json")
    traffic, traffic_prof = pick_traffic(pname, gemm_ms * 1e3)

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
        "dtype": ("e4m3 codes (fp32 accumulate) + fp16 salient tail" if use_f8 else
                  "fp32 (fp32-accurate products from fp16 pieces on the f16 MFMA)" if fp32
                  else "fp16"),
        "data": "synthetic (random-init weights N(0,0.02^2), x N(0,1) with 1% outlier channels x30)",
        "config": {
            "workload": (f"W4A4Linear.forward: weight per_group(sorted) int4 + act {args.act} "
                         f"{'(sorted) ' if args.act == 'per_group' else ''}4-bit, "
                         f"{int(P * 100)}% salient fp16 side-GEMM"),
            "M": M, "K": K, "N": N, "group_size": G, "salient_prop": P,
            "salient_channels": pw.S,
            "kernel": ("gemm_f8" if use_f8 else "gemm_fqt" if use_fqt
                       else "gemm_fq"),
            "parallelism": f"replicas x{world}",
        },
        "roofline": {
            "bound": "mfma",
            "achieved": round(achieved, 1),
            "peak": round(flops / t_roof / 1e12, 1),
            "peak_kind": "int8-MFMA contract roofline: 2MNK / (2MNK'/P_i8 + 2MNS/P_f16)",
            "unit": "TFLOP/s",
            "frac": round(t_roof / (gemm_ms * 1e-3), 4),
            "frac_dtype_peak": round(achieved / PEAK_TFLOPS[kdt], 4),
            "dtype_peak": PEAK_TFLOPS[kdt],
            "traffic": traffic,
            "traffic_profile": traffic_prof,
            "kernel": kname,
            "avg_ms": round(gemm_ms, 4),
            "algorithmic_flops_per_launch": flops,
            "t_roof_contract_us": round(t_roof * 1e6, 2),
            "frac_contract_step": round(t_roof / (ms_per_step * 1e-3), 4),
            "note": ("frac = the fraction of the int8-MFMA roofline (BASELINE.md §2 T_roof = "
                     "2MNK'/P_i8 + 2MNS/P_f16, over the GEMM time; peak = 2MNK / T_roof); "
                     "frac_dtype_peak = achieved / the dense MFMA peak of the kernel's dtype "
                     "(dtype_peak); frac_contract_step = T_roof / step time"
                     + ("; fp32: peak = the f32 MFMA (the dtype's own); the kernel executes "
                        "3 f16 MFMAs per product over Kp + S_pad positions: "
                        f"executed_f16_frac = {3 * achieved * (pw.Kp + pw.S_pad) / K / PEAK_TFLOPS['f16']:.4f}"
                        if fp32 else "")),
        },
        "reference_points": {
            "reference_fakequant_forward_ms": round(ref_ms, 4),
            "reference_fakequant_TFLOP_per_s": round(flops / (ref_ms * 1e-3) / 1e12, 1),
            "speedup_vs_reference_fakequant": round(ref_ms / ms_per_step, 2),
            "reference_vs_ours_rel_err": ref_rel,
            f"torch_{args.dtype}_linear_ms": round(dense_ms, 4),
            f"torch_{args.dtype}_linear_TFLOP_per_s": round(flops / (dense_ms * 1e-3) / 1e12, 1),
            "note": "reference fake-quant forward restated in PyTorch ops (tools/torch_fakequant.py) on "
                    f"this GPU; {args.dtype} F.linear = unquantized hipBLASLt GEMM of the same shape",
        },
        "prepass": {
            "avg_ms": round(quant_ms, 4),
            "algorithmic_bytes": prepass_bytes,
            "GB_per_s": round(prepass_bytes / (quant_ms * 1e-3) / 1e9, 1),
            "hbm_peak_GB_per_s": HBM_PEAK_GBS,
            "in_step_ms": round(ms_per_step - gemm_ms, 4),
            "note": "avg_ms: the prepass kernels timed back to back on their own (x stays in the "
                    "Infinity Cache); in_step_ms = step time - GEMM time (the prepass inside the "
                    "forward, plus launch gaps)",
        },
    }
    if not fp32 and args.act == "per_group" and not args.no_layer:
        out["per_token"] = per_token_leg(dev)
    if not fp32 and not args.no_layer:
        out["llama_layer"] = llama_layer(dev)
        out["llama_layer_pplflow"] = llama_layer(dev, flow="ppl_eval")
        out["llama_layer_token"] = llama_layer(dev, flow="token")
        out["fp32"] = fp32_leg(dev)
    if not fp32 and not args.no_layer and not args.no_e2e and world == 1:
        out["e2e"] = e2e_leg(args.e2e_windows, cpu=rank == 0 and not args.no_cpu)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.act)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
