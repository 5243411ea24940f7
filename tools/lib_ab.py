"""Same-box A/B of two builds of libsqmp_w4a4.so (the C ABI is the same; SQMP_LIB_PATH
selects the library): interleaved rounds of tools/gemm_time.py KIND, one process per run,
and the y of each build checked equal on the first round.

    python tools/lib_ab.py BASE.so NEW.so [kinds, comma-separated: fqt,f8] [rounds] [iters]

Prints the per-run averages and the median per (kind, build)."""
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = {"base": os.path.abspath(sys.argv[1]), "new": os.path.abspath(sys.argv[2])}
kinds = (sys.argv[3] if len(sys.argv) > 3 else "fqt,f8").split(",")
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 4
iters = sys.argv[5] if len(sys.argv) > 5 else "200"

res = {(k, n): [] for k in kinds for n in libs}
for r in range(rounds):
    for k in kinds:
        for n, path in (libs.items() if r % 2 == 0 else reversed(list(libs.items()))):
            env = dict(os.environ, SQMP_LIB_PATH=path)
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gemm_time.py"), k, iters],
                                 env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stdout, out.stderr)
                raise SystemExit(f"{k} {n} failed")
            line = out.stdout.strip().splitlines()[-1]
            ms = float(line.split("avg_ms=")[1].split()[0])
            res[(k, n)].append(ms)
            print(f"round {r} {k:4s} {n:4s} {ms * 1e3:8.1f} us", flush=True)
for k in kinds:
    b, v = statistics.median(res[(k, "base")]), statistics.median(res[(k, "new")])
    print(f"{k}: base {b * 1e3:.1f} us  new {v * 1e3:.1f} us  ({(v / b - 1) * 100:+.1f} %)")
