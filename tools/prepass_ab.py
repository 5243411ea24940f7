"""A/B timing of the activation quantizer (prepass): lane-contiguous kernel vs the previous
row kernels (SQMP_DISABLE_LC=1 in a child process), plus bit-exact equality of the two
A operands.  python tools/prepass_ab.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]

SHAPES = [(16384, 4096, 4096, 128, 0.10), (2048, 4096, 4096, 64, 0.05),
          (2048, 4096, 11008, 64, 0.05), (2048, 11008, 4096, 64, 0.05),
          (4096, 2048, 2048, 128, 0.05), (2048, 8192, 2048, 128, 0.05)]


def child(out_path):
    import torch
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    dev = torch.device("cuda")
    res = {}
    for (M, K, N, G, p) in SHAPES:
        for act in ("per_group", "per_token"):
            g = torch.Generator(device=dev).manual_seed(0)
            lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.float16)
            with torch.no_grad():
                lin.weight.copy_(torch.randn(N, K, generator=g, device=dev) * 0.02)
            x = torch.randn(M, K, generator=g, device=dev)
            x[:, torch.randperm(K, generator=g, device=dev)[: K // 100]] *= 30
            x = x.half()
            q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=act,
                                      importance=x.float().abs().mean(0).cpu(), salient_prop=p,
                                      group_size=G)
            pw = q.packed()
            f = lambda: ops.quant_act_fp(x, pw, act, 4, G)  # noqa: E731
            for _ in range(3):
                a = f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            res[f"{M}x{K}->{N} G{G} {act}"] = (ms, a[:, : pw.Kp + pw.S].float().sum().item(),
                                              a.view(torch.int16).long().sum().item())
    import json
    json.dump(res, open(out_path, "w"))


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(sys.argv[1])
        sys.exit(0)
    import json
    outs = {}
    for tag, env in (("lc", {}), ("old", {"SQMP_DISABLE_LC": "1"})):
        path = f"/tmp/prepass_{tag}.json"
        subprocess.run([sys.executable, __file__, path], check=True, env={**os.environ, **env},
                       timeout=300)
        outs[tag] = json.load(open(path))
    for k in outs["lc"]:
        a, b = outs["lc"][k], outs["old"][k]
        same = a[2] == b[2]
        print(f"{k:34s} lc {a[0]*1e3:8.1f} us   old {b[0]*1e3:8.1f} us   x{b[0]/a[0]:5.2f}   "
              f"A-operand checksum {'equal' if same else 'DIFFERENT'}")
