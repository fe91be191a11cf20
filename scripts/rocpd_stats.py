"""Per-kernel (name, grid) duration summary of a rocprofv3 rocpd database
(rocprofv3 -d DIR -o NAME writes NAME_results.db): calls, avg / min / max us.
usage: python scripts/rocpd_stats.py DB [name-filter] [--seq]  (--seq: the dispatch sequence with gaps)"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    c = sqlite3.connect(db)
    t = {r[0].split("_0000")[0]: r[0] for r in c.execute("select name from sqlite_master where type='table'")}
    q = (f"select s.display_name, d.grid_size_x, d.grid_size_y, d.start, d.end, s.arch_vgpr_count, s.accum_vgpr_count "
         f"from {t['rocpd_kernel_dispatch']} d join {t['rocpd_info_kernel_symbol']} s on d.kernel_id = s.id "
         f"order by d.start")
    rows = [r for r in c.execute(q) if filt in r[0]]
    if "--seq" in sys.argv:
        prev = None
        for r in rows:
            gap = (r[3] - prev) / 1e3 if prev is not None else 0.0
            print(f"{r[0][:70]:70s} grid=({r[1]},{r[2]}) {(r[4] - r[3]) / 1e3:9.1f} us  gap {gap:8.1f} us")
            prev = r[4]
        return
    agg = defaultdict(list)
    for r in rows:
        agg[(r[0][:90], r[1], r[2], r[5], r[6])].append((r[4] - r[3]) / 1e3)
    for (n, gx, gy, av, acc), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n:90s} grid=({gx},{gy}) vgpr={av}/{acc} calls={len(d):5d} avg={sum(d) / len(d):9.1f} "
              f"min={min(d):9.1f} max={max(d):9.1f} us")


if __name__ == "__main__":
    main()
