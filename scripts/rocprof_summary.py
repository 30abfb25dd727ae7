"""Summarise a rocprofv3 SQLite (.db) kernel trace: per-kernel total/avg time and share.

    python scripts/rocprof_summary.py gpurun_out/prof/bench_results.db [--out profiles/x.md]
"""
import argparse
import sqlite3
import sys


def summarize(db, top=40, by_grid=False, last_frac=1.0):
    con = sqlite3.connect(db)
    cur = con.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = cur.execute(f"select {name_col}, start, end, grid_x from kernels order by start").fetchall()
    rows = rows[int(len(rows) * (1.0 - last_frac)):]    # steady state: skip setup / tuning dispatches
    agg = {}
    for name, s, e, gx in rows:
        d = (e - s) / 1e3  # ns -> us
        name = f"{name} [grid {gx}]" if by_grid else name
        n, tot = agg.get(name, (0, 0.0))
        agg[name] = (n + 1, tot + d)
    total = sum(t for _, t in agg.values())
    out = [f"| kernel | calls | total us | avg us | % |", "|---|---|---|---|---|"]
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        short = name if len(name) < 90 else name[:87] + "..."
        out.append(f"| `{short}` | {n} | {t:.1f} | {t / n:.2f} | {100 * t / total:.1f} |")
    out.append(f"\ntotal kernel time: {total / 1e3:.3f} ms over {len(rows)} dispatches")
    return "\n".join(out)


def sequence(db, last=80):
    """The last ``last`` dispatches in launch order with their durations (one forward of an
    in-order single-stream trace: isolated per-kernel times, attributable to layers)."""
    con = sqlite3.connect(db)
    cur = con.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = cur.execute(f"select {name_col}, start, end, grid_x from kernels order by start").fetchall()[-last:]
    out = ["| # | kernel | grid | us |", "|---|---|---|---|"]
    tot = 0.0
    for i, (name, s, e, gx) in enumerate(rows):
        d = (e - s) / 1e3
        tot += d
        short = name if len(name) < 80 else name[:77] + "..."
        out.append(f"| {i} | `{short}` | {gx} | {d:.1f} |")
    span = (rows[-1][2] - rows[0][1]) / 1e3 if rows else 0.0
    out.append(f"\nsum {tot:.1f} us, span {span:.1f} us over {len(rows)} dispatches")
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--out")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--by-grid", action="store_true", help="split kernels by grid size (layer shapes)")
    ap.add_argument("--sequence", type=int, default=0, help="list the last N dispatches in order instead")
    ap.add_argument("--last-frac", type=float, default=1.0, help="summarise only the last fraction of dispatches")
    a = ap.parse_args()
    s = sequence(a.db, a.sequence) if a.sequence else summarize(a.db, a.top, a.by_grid, a.last_frac)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
