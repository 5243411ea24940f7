"""Whether sibling GEMMs (q/k/v: 3 x 2048 x 4096 -> 4096; gate/up: 2 x 2048 x 4096 -> 11008)
gain from running concurrently: one after another on one stream (packed-order OPT 3 and 8)
against one per stream (OPT 8: two workgroups per CU, so a second launch finds free slots).
python tools/sib_concurrency.py [rounds] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda")
main = torch.cuda.current_stream(dev)
side = [torch.cuda.Stream(dev) for _ in range(3)]
for name, M, K, Ns in (("qkv", 2048, 4096, (4096, 4096, 4096)), ("gate_up", 2048, 4096, (11008, 11008))):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, K, generator=g, device=dev).half()
    sal = torch.argsort(x.float().abs().mean(0), descending=True)[: int(0.05 * K)].cpu()
    pws, acts = [], []
    for N in Ns:
        w = (torch.randn(N, K, generator=g, device=dev) * 0.02).half()
        pws.append(ops.pack_weight(w, "per_group", 4, 64, sal))
        acts.append(ops.quant_act_fp(x, pws[-1], "per_group", 4, 64).clone())

    def seq():
        for a, pw in zip(acts, pws):
            ops.gemm_fq(a, pw, None)

    def conc():
        ev = torch.cuda.Event()
        ev.record(main)
        done = []
        for s, a, pw in zip(side, acts, pws):
            s.wait_event(ev)
            with torch.cuda.stream(s):
                ops.gemm_fq(a, pw, None)
                e = torch.cuda.Event()
                e.record(s)
                done.append(e)
        for e in done:
            main.wait_event(e)

    variants = [("seq OPT3", "3", seq), ("seq OPT8", "8", seq), ("streams OPT8", "8", conc),
                ("streams OPT3", "3", conc)]
    res = {v[0]: [] for v in variants}
    for _ in range(rounds):
        for tag, opt, fn in variants:
            os.environ["SQMP_FQ7_OPT"] = opt
            __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
            for _ in range(5):
                fn()
            a0, b0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a0.record(main)
            for _ in range(iters):
                fn()
            b0.record(main)
            b0.synchronize()
            res[tag].append(a0.elapsed_time(b0) / iters * 1e3)
    print(f"{name}: " + " | ".join(f"{t}: {sorted(v)[len(v) // 2]:7.1f} us" for t, v in res.items()),
          flush=True)
