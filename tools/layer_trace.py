"""One Llama-2-7B decoder layer's 7 W4A4 linears at 2048 tokens (bench.py llama_layer's
shapes), run PASSES times with a device sync between passes -- a target for
`rocprofv3 --kernel-trace`; then `python tools/layer_trace.py --parse TRACE.csv` prints the
last pass's kernels in order with their durations and the gaps between them.

    python tools/layer_trace.py [PASSES]
    python tools/layer_trace.py --parse gpurun_out/.../kernel_trace.csv
"""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]


def parse(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # passes are separated by torch.cuda._sleep's spin kernel: keep the last full pass
    passes, cur = [], []
    for r in rows:
        if "spin" in r[2] or "sleep" in r[2]:
            if cur:
                passes.append(cur)
            cur = []
        else:
            cur.append(r)
    passes.append(cur)
    passes = [p for p in passes if p]
    last = passes[-1]
    t0, prev_end, busy = last[0][0], last[0][0], 0
    # the median duration of each launch position over the passes of the same shape (the
    # first few passes warm the clock and the caches: the second half only)
    full = [p for p in passes if len(p) == len(last)]
    full = full[len(full) // 2:]
    med = [sorted((p[i][1] - p[i][0]) for p in full)[len(full) // 2] for i in range(len(last))]
    for i, (s, e, n) in enumerate(last):
        short = n.split("(")[0].replace("void ", "")[:70]
        print(f"{(s - t0) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:5.1f}  dur {(e - s) / 1e3:6.1f}  "
              f"median {med[i] / 1e3:6.1f}  {short}")
        prev_end, busy = e, busy + (e - s)
    nongemm = sum(m for m, (_, _, n) in zip(med, last) if "gemm" not in n)
    print(f"pass: {(last[-1][1] - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, "
          f"{len(last)} launches ({len(passes)} passes in the trace); medians over {len(full)} "
          f"passes: kernels {sum(med) / 1e3:.1f} us, non-GEMM {nongemm / 1e3:.1f} us")


def run(passes):
    import torch
    import bench
    from smoothquant.fake_quant import W4A4Linear
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(7)
    xs = {}
    for name, K in (("attn", 4096), ("o", 4096), ("mlp", 4096), ("down", 11008)):
        x = torch.randn(bench.LLAMA_T, K, generator=gen, device=dev)
        x[:, torch.randperm(K, generator=gen, device=dev)[: K // 100]] *= 30.0
        xs[name] = x.half()
    layers = []
    for name, K, N, src in bench.LLAMA_LINEARS:
        lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.float16)
        with torch.no_grad():
            lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).half())
        imp = xs[src][:512].float().abs().mean(0).cpu()
        layers.append((W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                                             importance=imp, salient_prop=bench.LLAMA_P,
                                             group_size=bench.LLAMA_G), xs[src]))
    if os.environ.get("SQMP_LINK", "1") == "1":  # the sibling groups quantize_llama_like links
        from smoothquant.fake_quant import link_siblings
        link_siblings(*[layers[i][0] for i in (0, 1, 2)])
        link_siblings(*[layers[i][0] for i in (4, 5)])
    for _ in range(passes):
        for q, x in layers:
            q(x)
        torch.cuda.synchronize()
        torch.cuda._sleep(100_000)  # a separator kernel between passes in the trace
        torch.cuda.synchronize()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
