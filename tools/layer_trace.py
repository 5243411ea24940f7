"""One Llama-2-7B decoder layer's 7 W4A4 linears at 2048 tokens (bench.py llama_layer's
shapes), run PASSES times with a device sync between passes -- a target for
`rocprofv3 --kernel-trace`; then `python tools/layer_trace.py --parse TRACE.csv` prints the
last pass's kernels in order with their durations and the gaps between them.

    python tools/layer_trace.py [PASSES]
    python tools/layer_trace.py --parse gpurun_out/.../kernel_trace.csv

LT_FLOW=ppl_eval: the reference's smoothquant/ppl_eval.py configuration instead (bf16,
per_channel weights, per_token activations, no salient channels, output quantization of
q/k/v as quantize_model(quantize_bmm_input=True) binds it); LT_FLOW=token_fp16: the
quantize_llama_like defaults in fp16 (per_channel W, per_token A, no salient, no output quant); LT_FP16=1 adds the unquantized
F.linear pass of the same shapes after the W4A4 pass (a second separator in between).
"""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]


def _segments(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # passes are separated by torch.cuda._sleep's spin kernel
    segs, cur = [], []
    for r in rows:
        if "spin" in r[2] or "sleep" in r[2]:
            if cur:
                segs.append(cur)
            cur = []
        else:
            cur.append(r)
    segs.append(cur)
    return [p for p in segs if p]


def _report(passes, label):
    last = passes[-1]
    t0, prev_end, busy = last[0][0], last[0][0], 0
    # the median duration of each launch position over the passes of the same shape (the
    # first few passes warm the clock and the caches: the second half only)
    full = passes[len(passes) // 2:]
    med = [sorted((p[i][1] - p[i][0]) for p in full)[len(full) // 2] for i in range(len(last))]
    if label:
        print(f"# {label}")
    for i, (s, e, n) in enumerate(last):
        short = n.split("(")[0].replace("void ", "")[:70]
        print(f"{(s - t0) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:5.1f}  dur {(e - s) / 1e3:6.1f}  "
              f"median {med[i] / 1e3:6.1f}  {short}")
        prev_end, busy = e, busy + (e - s)
    nongemm = sum(m for m, (_, _, n) in zip(med, last) if "gemm" not in n.lower()
                  and "Cijk" not in n)
    print(f"pass: {(last[-1][1] - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, "
          f"{len(last)} launches ({len(passes)} passes in the trace); medians over {len(full)} "
          f"passes: kernels {sum(med) / 1e3:.1f} us, non-GEMM {nongemm / 1e3:.1f} us")


def parse(path):
    """Every distinct pass shape (kernel-name sequence) seen at least 3 times, in order of
    first appearance: the last pass of that shape with per-launch medians."""
    segs = _segments(path)
    shapes = {}
    for sgm in segs:
        shapes.setdefault(tuple(n for _, _, n in sgm), []).append(sgm)
    multi = [v for v in shapes.values() if len(v) >= 3]
    for v in multi:
        _report(v, f"pass shape of {len(v[0])} launches" if len(multi) > 1 else "")


def run(passes):
    import torch
    import bench
    from smoothquant.fake_quant import W4A4Linear
    flow = os.environ.get("LT_FLOW", "")
    ppl_flow = flow in ("ppl_eval", "token_fp16")
    dt = torch.bfloat16 if flow == "ppl_eval" else torch.float16
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(7)
    xs = {}
    for name, K in (("attn", 4096), ("o", 4096), ("mlp", 4096), ("down", 11008)):
        x = torch.randn(bench.LLAMA_T, K, generator=gen, device=dev)
        x[:, torch.randperm(K, generator=gen, device=dev)[: K // 100]] *= 30.0
        xs[name] = x.to(dt)
    layers, dense = [], []
    for name, K, N, src in bench.LLAMA_LINEARS:
        lin = torch.nn.Linear(K, N, bias=False).to(dev, dt)
        with torch.no_grad():
            lin.weight.copy_((torch.randn(N, K, generator=gen, device=dev) * 0.02).to(dt))
        dense.append((lin.weight.detach().clone(), xs[src]))
        if ppl_flow:
            q = W4A4Linear.from_float(lin, weight_quant="per_channel", act_quant="per_token",
                                      quantize_output=(flow == "ppl_eval"
                                                       and name in ("q_proj", "k_proj", "v_proj")))
        else:
            imp = xs[src][:512].float().abs().mean(0).cpu()
            q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                                      importance=imp, salient_prop=bench.LLAMA_P,
                                      group_size=bench.LLAMA_G)
        layers.append((q, xs[src]))
    if os.environ.get("SQMP_LINK", "1") == "1":  # the sibling groups quantize_llama_like links
        from smoothquant.fake_quant import link_siblings
        link_siblings(*[layers[i][0] for i in (0, 1, 2)])
        link_siblings(*[layers[i][0] for i in (4, 5)])
    fp16 = os.environ.get("LT_FP16") == "1"
    for _ in range(passes):
        # (per_token without salient channels quantizes its input in place, as the reference
        # does: fresh copies, made before the separator, keep every pass on the same input)
        ins = [x.clone() if ppl_flow else x for _, x in layers]
        if ppl_flow:
            torch.cuda.synchronize()
            torch.cuda._sleep(100_000)
            torch.cuda.synchronize()
        for (q, _), x in zip(layers, ins):
            q(x)
        torch.cuda.synchronize()
        torch.cuda._sleep(100_000)  # a separator kernel between passes in the trace
        torch.cuda.synchronize()
        if fp16:
            for w, x in dense:
                torch.nn.functional.linear(x, w)
            torch.cuda.synchronize()
            torch.cuda._sleep(100_000)
            torch.cuda.synchronize()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
