"""Per-token in-place quantizer (token_rows_kernel) timing probe: fp16 vs bf16 at the Llama
shapes, alone and after the F8 quantizer reads the same x (HIP events, median of 50)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "smoothquant-mixedprecision_amd")]

import torch  # noqa: E402


def t_us(fn, n=50):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for _ in range(5):
        fn()
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in evs)[n // 2] * 1e3


def main():
    from smoothquant import ops
    from smoothquant.fake_quant import _fq_act, W4A4Linear
    dev = torch.device("cuda")
    for dt in (torch.float16, torch.bfloat16):
        for K in (4096, 11008):
            x0 = torch.randn(2048, K, device=dev).to(dt)
            xs = [x0.clone() for _ in range(60)]
            it = iter(range(10 ** 9))
            print(f"{dt} K={K}: fresh rows {t_us(lambda: _fq_act(xs[next(it) % 60], 'per_token', 4)):.1f} us, "
                  f"same rows again {t_us(lambda: _fq_act(x0, 'per_token', 4)):.1f} us")
            if dt == torch.float16:
                lin = torch.nn.Linear(K, 4096, bias=False).to(dev, dt)
                q = W4A4Linear.from_float(lin, weight_quant="per_channel", act_quant="per_token")
                pw = q.packed()
                def both():
                    ops.quant_act_f8(x0, pw, "per_token", 4)
                    _fq_act(x0, "per_token", 4)
                print(f"   F8 quantizer {t_us(lambda: ops.quant_act_f8(x0, pw, 'per_token', 4)):.1f} us, "
                      f"F8 quantizer + in-place {t_us(both):.1f} us")


if __name__ == "__main__":
    main()
