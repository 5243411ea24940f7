"""In-process A/B of the activation-order GEMM's variants at config 2 (sqmp_gemm_fqt7,
SQMP_FQT7_OPT read per launch): interleaved rounds, HIP events, y bit-identical across
variants.  python tools/ab_fqt7.py [variants, "+"- or comma-separated] [rounds] [iters] [ENV]
ENV (default SQMP_FQT7_OPT) names the per-launch variable; SQMP_FQ7_DIAG selects the timing
diagnostics of a SQMP_DIAG=1 build (wrong results by design: no equality check then).  A
variant "J4:3" runs the 64-row-block operands (ops.FQT7_J = 4) with value 3; "P..." times the
prepass (quant_act_c4) of that variant instead of the GEMM.  (The one-wave-per-SIMD fqt8 /
fqt9 variants were removed in round 5, profiles/r04_ab_fqt8.txt, r04_ab_fqt9.txt; the fqa
variant in round 6, profiles/r05_ab_fqa_dense_core.txt.)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from smoothquant import ops  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else "0+1+2+3+4+5").replace(",", "+").split("+")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
ENV = sys.argv[4] if len(sys.argv) > 4 else "SQMP_FQT7_OPT"
dev = torch.device("cuda")
q, x, lin = bench.make_layer(dev, "per_group", seed=1)
pw = q.packed()
stream = torch.cuda.current_stream(dev)


def parse(v):
    pre = v.startswith("P")
    v = v[1:] if pre else v
    j, val = (int(v[1:v.index(":")]), v[v.index(":") + 1:]) if v.startswith("J") else (2, v)
    return pre, j, val


def use(j):
    ops.FQT7_J = j if j in (2, 4) else 2


ops_c4 = {}
for v in variants:
    _, j, _ = parse(v)
    if j not in ops_c4:
        use(j)
        ops_c4[j] = ops.quant_act_c4(x, pw, "per_group", 4, bench.G)


def runner(v):
    pre, j, _ = parse(v)
    if pre:
        def f():
            use(j)
            return ops.quant_act_c4(x, pw, "per_group", 4, bench.G)[0]
        return f
    def g():
        use(j)
        return ops.gemm_fqt(*ops_c4[j], pw, lin.bias, bench.G)
    return g


ref = None
for v in variants:
    os.environ[ENV] = parse(v)[2]
    __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
    run = runner(v)
    y = run()
    if parse(v)[0]:
        continue
    torch.cuda.synchronize()
    if ref is None:
        ref = y.clone()
    assert ENV.endswith("_DIAG") or torch.equal(y.view(torch.int16), ref.view(torch.int16)), f"variant {v} changed y"
t_end = __import__("time").perf_counter() + 2.0
while __import__("time").perf_counter() < t_end:
    for _ in range(10):
        runner(variants[0])()
    torch.cuda.synchronize()
res = {v: [] for v in variants}
flops = 2.0 * bench.M * bench.N * bench.K
for r in range(rounds):
    for v in variants:
        os.environ[ENV] = parse(v)[2]
        __import__("smoothquant._lib", fromlist=["_lib"]).reload_knobs()  # (knobs are read once at load)
        run = runner(v)
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
    print(f"{ENV}={v}: median {t[len(t) // 2]:7.1f} us  min {t[0]:7.1f} us  "
          f"({flops / t[len(t) // 2] / 1e6:7.1f} TFLOP/s)  all {[round(u, 1) for u in res[v]]}")
