"""Kernel breakdown of ONE request's prefill from a rocprofv3 kernel trace (rocpd SQLite).

  python tools/ttft_breakdown.py gpurun_out/prof_ttft/run_results.db [--gap-us 500] [--which -1]

The trace of tools/vlm_bench.py --batch 0 holds several single-request TTFTs separated by idle
gaps; kernels are split into bursts at gaps > --gap-us and burst --which (default: the last one
with the most kernels) is summarised: span, GPU-busy time, idle gaps, and per kernel name the
count, total time and the idle time before its launches.
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    gap_us = float(sys.argv[sys.argv.index("--gap-us") + 1]) if "--gap-us" in sys.argv else 500.0
    which = int(sys.argv[sys.argv.index("--which") + 1]) if "--which" in sys.argv else None
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    bursts, cur = [], []
    for r in rows:
        if cur and (r[1] - cur[-1][2]) / 1000.0 > gap_us:
            bursts.append(cur)
            cur = []
        cur.append(r)
    if cur:
        bursts.append(cur)
    if which is None:
        big = max(len(b) for b in bursts)
        cand = [i for i, b in enumerate(bursts) if len(b) >= 0.9 * big]
        which = cand[-1]
    b = bursts[which]
    span = (b[-1][2] - b[0][1]) / 1000.0
    busy = sum(e - s for _, s, e in b) / 1000.0
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    prev_end = None
    for n, s, e in b:
        a = agg[n]
        a[0] += 1
        a[1] += (e - s) / 1000.0
        if prev_end is not None:
            a[2] += max(0.0, (s - prev_end) / 1000.0)
        prev_end = e
    print(f"bursts {len(bursts)} (sizes {[len(x) for x in bursts]}), showing #{which}")
    print(f"kernels {len(b)} span us {span:.1f}")
    print(f"busy us {busy:.1f}")
    print(f"gaps us {span - busy:.1f}")
    for n, (k, t, g) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:5d} {t:10.1f}us gap {g:7.1f} {n[:90]}")


if __name__ == "__main__":
    main()
