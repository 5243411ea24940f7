"""Host (CPU) time per W4A4 call vs GPU time per call at a small M: shows whether the
forward is launch-bound.  python tools/host_overhead.py [M] [K] [N]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

from smoothquant import ops  # noqa: E402
from smoothquant.fake_quant import W4A4Linear  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
N = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
dev = torch.device("cuda")
lin = torch.nn.Linear(K, N, bias=False).to(dev, torch.float16)
x = torch.randn(M, K, device=dev).half()
q = W4A4Linear.from_float(lin, weight_quant="per_group", act_quant="per_group",
                          importance=x.float().abs().mean(0).cpu(), salient_prop=0.05,
                          group_size=64)
pw = q.packed()
a_op = ops.quant_act_fp(x, pw, "per_group", 4, 64)
for name, fn in [("quant_act_fp", lambda: ops.quant_act_fp(x, pw, "per_group", 4, 64)),
                 ("gemm_fq", lambda: ops.gemm_fq(a_op, pw, None)),
                 ("forward", lambda: q(x)),
                 ("F.linear", lambda: torch.nn.functional.linear(x, lin.weight)),
                 ("packed()", lambda: q.packed())]:
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t_host = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / n
    print(f"{name:14s} host {t_host*1e6:7.1f} us/call   host+drain {t_all*1e6:7.1f} us/call")
