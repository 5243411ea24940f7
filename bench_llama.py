"""Config 4 of BASELINE.json (Llama-2-7B W4A4 prefill tokens/s on 1 MI355X): bench_e2e.py
with --model llama2-7b.  python bench_llama.py [bench_e2e options]"""
import sys

import bench_e2e

if __name__ == "__main__":
    bench_e2e.main(["--model", "llama2-7b"] + sys.argv[1:])
