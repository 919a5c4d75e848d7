#!/usr/bin/env python3
"""Summarise rocprofv3 --stats / --kernel-trace CSV output into a short text table."""
import csv
import glob
import sys
from collections import defaultdict


def main(root, out=None, top=30):
    stats = glob.glob(f"{root}/**/*kernel_stats.csv", recursive=True)
    dbs = glob.glob(f"{root}/**/*results.db", recursive=True)
    lines = []
    if not stats and dbs:   # rocprofv3's default rocpd SQLite output (ROCm 7.x)
        import sqlite3
        con = sqlite3.connect(dbs[0])
        # the rocpd top_kernels view reports durations in MICROseconds (a round-2 summary printed
        # them as ns and came out 1000x small): scale to ns so the arithmetic below is uniform
        rows = [(n, c, t * 1e3, a * 1e3) for n, c, t, a in
                con.execute("select name, total_calls, total_duration, average from top_kernels").fetchall()]
        tot = sum(r[2] for r in rows) or 1
        lines.append(f"# {dbs[0]}\n# total kernel time {tot/1e6:.1f} ms over {sum(r[1] for r in rows)} dispatches")
        lines.append(f"{'pct':>6} {'total_ms':>10} {'calls':>7} {'avg_us':>9}  kernel")
        for name, calls, total, avg in sorted(rows, key=lambda r: -r[2])[:top]:
            lines.append(f"{100*total/tot:6.2f} {total/1e6:10.2f} {calls:7d} {avg/1e3:9.1f}  {name[:150]}")
    elif stats:
        rows = list(csv.DictReader(open(stats[0])))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        lines.append(f"# {stats[0]}\n# total kernel time {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
        if dbs:   # the same run in rocpd form: its top_kernels total, read as microseconds
            import sqlite3
            t_db = sum(r[0] for r in sqlite3.connect(dbs[0]).execute("select total_duration from top_kernels"))
            lines.append(f"# rocpd top_kernels total of the same run: {t_db / 1e3:.1f} ms if read as us "
                         f"({t_db / 1e6:.3f} ms if read as ns)")
        lines.append(f"{'pct':>6} {'total_ms':>10} {'calls':>7} {'avg_us':>9}  kernel")
        for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
            lines.append(f"{100*float(r['TotalDurationNs'])/tot:6.2f} {float(r['TotalDurationNs'])/1e6:10.2f} "
                         f"{int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.1f}  {r['Name'][:150]}")
    else:
        traces = glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)
        agg = defaultdict(lambda: [0, 0.0])
        for t in traces:
            for r in csv.DictReader(open(t)):
                d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                a = agg[r["Kernel_Name"]]
                a[0] += 1
                a[1] += d
        tot = sum(v[1] for v in agg.values()) or 1
        lines.append(f"{'pct':>6} {'total_ms':>10} {'calls':>7} {'avg_us':>9}  kernel")
        for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
            lines.append(f"{100*d/tot:6.2f} {d/1e6:10.2f} {n:7d} {d/n/1e3:9.1f}  {k[:150]}")
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
