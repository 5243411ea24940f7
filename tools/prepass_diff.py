"""Debug: A operands of the lane-contiguous and the previous quantizer (child processes,
SQMP_DISABLE_LC) compared element-wise and against the CPU oracle.
python tools/prepass_diff.py [M K G act]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
M, K, G = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (2048, 4096, 64)))
ACT = sys.argv[4] if len(sys.argv) > 4 else "per_group"


def child(tag):
    import torch
    from smoothquant import ops
    from smoothquant.fake_quant import W4A4Linear
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    lin = torch.nn.Linear(K, 512, bias=False).to(dev, torch.float16)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(512, K, generator=g, device=dev) * 0.02)
    x = torch.randn(M, K, generator=g, device=dev)
    x[:, torch.randperm(K, generator=g, device=dev)[: K // 100]] *= 30
    x = x.half()
    q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant=ACT,
                              importance=x.float().abs().mean(0).cpu(), salient_prop=0.05,
                              group_size=G)
    pw = q.packed()
    a = ops.quant_act_fp(x, pw, ACT, 4, G)
    torch.cuda.synchronize()
    np.save(f"/tmp/pd_{tag}_a.npy", a.view(torch.int16).cpu().numpy())
    np.save(f"/tmp/pd_x.npy", x.float().cpu().numpy())
    np.save(f"/tmp/pd_amap.npy", pw.amap.cpu().numpy())
    np.save(f"/tmp/pd_sal.npy", pw.salient.cpu().numpy())
    print(tag, "Kp", pw.Kp, "S", pw.S, "S_pad", pw.S_pad)


if __name__ == "__main__":
    if len(sys.argv) > 5:
        child(sys.argv[5])
        sys.exit(0)
    for tag, env in (("lc", {}), ("old", {"SQMP_DISABLE_LC": "1"})):
        subprocess.run([sys.executable, __file__, str(M), str(K), str(G), ACT, tag], check=True,
                       env={**os.environ, **env}, timeout=300)
    a_lc, a_old = np.load("/tmp/pd_lc_a.npy"), np.load("/tmp/pd_old_a.npy")
    x, amap, sal = np.load("/tmp/pd_x.npy"), np.load("/tmp/pd_amap.npy"), np.load("/tmp/pd_sal.npy")
    d = np.argwhere(a_lc != a_old)
    print("differing elements:", len(d), "of", a_lc.size)
    from oracle import fake_quant_oracle as O
    dt = O.DT("fp16")
    qx = O.quantize_input(x.astype(np.float16), ACT, 4, G, sal.astype(np.int64), dt)
    want = np.zeros_like(a_lc)
    Kp = len(amap)
    valid = amap >= 0
    want[:, :Kp][:, valid] = qx[:, amap[valid]].astype(np.float16).view(np.int16)
    want[:, Kp:Kp + len(sal)] = qx[:, sal].astype(np.float16).view(np.int16)
    h = lambda v: np.asarray(v, np.int16).view(np.float16)  # noqa: E731
    for tag, a in (("lc", a_lc), ("old", a_old)):
        bad = (h(a).astype(np.float32) != h(want).astype(np.float32))
        print(tag, "value mismatches vs oracle:", int(bad.sum()))
        idx = np.argwhere(bad)[:8]
        for m, p in idx:
            print(f"   row {m} pos {p} col {amap[p] if p < Kp else 'sal'}: got {h(a[m, p])} want {h(want[m, p])}")
