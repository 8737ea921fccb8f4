"""Kernel statistics from a rocprofv3 SQLite (rocpd) database, as the CSV the older
``--stats`` output used: Name, Calls, TotalDurationNs, AverageNs, Percentage.

  python tools/rocpd_stats.py gpurun_out/prof_bench/run_results.db [out.csv] [--top N] [--ar-share]

``--pmc`` prints per-kernel sums of the collected PMC counters (pmc_events view) instead, with
derived MFMA / LDS-conflict / VALU ratios; ``--kernels a,b`` filters by name substring.
``--ar-share`` also prints the all-reduce share of GPU kernel time (IPC one-shot ``custom_ar``
kernels + RCCL collectives) — BASELINE row 5's "all-reduce share of decode step time".
"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start) from kernels group by name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(n, k, t, t / k, 100.0 * t / tot) for n, k, t in rows]


def _flag_values():
    return [sys.argv[i + 1] for i, a in enumerate(sys.argv[:-1]) if a in ("--top", "--kernels")]


def pmc(db, kernels=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, counter_name, sum(counter_value), count(distinct dispatch_id) from pmc_events "
                     "group by name, counter_name").fetchall()
    out: dict = {}
    for n, cn, v, k in rows:
        if kernels and not any(x in n for x in kernels):
            continue
        d = out.setdefault(n, {"dispatches": k})
        d[cn] = v
    for d in out.values():
        if d.get("SQ_INSTS_LDS"):
            d["lds_bank_conflict_cycles_per_lds_inst"] = d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_INSTS_LDS"]
        tot = sum(d.get(k, 0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"))
        if tot:
            d["mfma_inst_fraction"] = d.get("SQ_INSTS_MFMA", 0) / tot
        if d.get("SQ_WAVE_CYCLES"):
            d["wait_inst_fraction"] = d.get("SQ_WAIT_INST_ANY", 0) / d["SQ_WAVE_CYCLES"]
    try:   # kernel time under the profiler -> effective clock from GRBM_GUI_ACTIVE
        dur = dict(c.execute("select name, sum(end - start) from kernels group by name").fetchall())
    except sqlite3.Error:
        dur = {}
    for n, d in out.items():
        if n in dur:
            d["kernel_ns"] = dur[n]
        if d.get("GRBM_GUI_ACTIVE") and d.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            # MFMA-busy share of every SIMD's cycles over the dispatches (1,024 SIMDs; the GRBM counter
            # is summed over the 8 XCDs, so per-XCD active cycles = GRBM_GUI_ACTIVE / 8)
            d["mfma_busy_per_simd"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 1024)
            if n in dur:
                d["clock_ghz_grbm"] = d["GRBM_GUI_ACTIVE"] / 8 / dur[n]
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    if "--pmc" in sys.argv:
        import json

        ks = sys.argv[sys.argv.index("--kernels") + 1].split(",") if "--kernels" in sys.argv else None
        for n, d in sorted(pmc(args[0], ks).items()):
            print(json.dumps({"kernel": n[:120], **{k: (round(v, 4) if isinstance(v, float) else v)
                                                   for k, v in d.items()}}))
        return
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 15
    rows = stats(args[0])
    if len(args) > 1:
        with open(args[1], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for r in rows:
                w.writerow([r[0], r[1], r[2], round(r[3], 1), round(r[4], 3)])
    for n, k, t, a, p in rows[:top]:
        print(f"{p:6.2f}%  {k:6d}  {a / 1e3:9.2f} us  {n[:110]}")
    if "--ar-share" in sys.argv:
        keys = ("custom_ar", "allreduce", "AllReduce", "ncclDevKernel", "rccl")
        ar = [r for r in rows if any(k in r[0] for k in keys)]
        tot = sum(r[2] for r in rows) or 1
        import json

        print(json.dumps({"all_reduce_share_of_kernel_time": sum(r[2] for r in ar) / tot,
                          "all_reduce_calls": sum(r[1] for r in ar),
                          "all_reduce_avg_us": (sum(r[2] for r in ar) / max(sum(r[1] for r in ar), 1)) / 1e3,
                          "kernels": [r[0][:80] for r in ar]}))


if __name__ == "__main__":
    main()
