"""In-process A/B of the activation-order GEMM's variants at config 2 (sqmp_gemm_fqt7,
SQMP_FQT7_OPT read per launch): interleaved rounds, HIP events, y bit-identical across
variants.  python tools/ab_fqt7.py [variants, comma-separated] [rounds] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4,5").split(",")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
dev = torch.device("cuda")
q, x, lin = bench.make_layer(dev, "per_group", seed=1)
pw = q.packed()
c4 = ops.quant_act_c4(x, pw, "per_group", 4, bench.G)
stream = torch.cuda.current_stream(dev)
run = lambda: ops.gemm_fqt(*c4, pw, lin.bias, bench.G)  # noqa: E731
ref = None
for v in variants:
    os.environ["SQMP_FQT7_OPT"] = v
    y = run()
    torch.cuda.synchronize()
    if ref is None:
        ref = y.clone()
    assert torch.equal(y.view(torch.int16), ref.view(torch.int16)), f"variant {v} changed y"
t_end = __import__("time").perf_counter() + 2.0
while __import__("time").perf_counter() < t_end:
    for _ in range(10):
        run()
    torch.cuda.synchronize()
res = {v: [] for v in variants}
flops = 2.0 * bench.M * bench.N * bench.K
for r in range(rounds):
    for v in variants:
        os.environ["SQMP_FQT7_OPT"] = v
        for _ in range(10):
            run()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(iters):
            run()
        b.record(stream)
        b.synchronize()
        res[v].append(a.elapsed_time(b) / iters * 1e3)
for v in variants:
    t = sorted(res[v])
    print(f"OPT={v}: median {t[len(t) // 2]:7.1f} us  min {t[0]:7.1f} us  "
          f"({flops / t[len(t) // 2] / 1e6:7.1f} TFLOP/s)  all {[round(u, 1) for u in res[v]]}")
