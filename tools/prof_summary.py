"""Summarise a rocprofv3 kernel-trace database (.db) or kernel_stats.csv into a per-kernel table (markdown)."""
import csv
import sqlite3
import sys


def from_db(path):
    con = sqlite3.connect(path)
    q = """select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start),
                  max(d.end - d.start)
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by s.kernel_name order by 3 desc"""
    return [(r[0], r[1], r[2], r[3], r[4], r[5]) for r in con.execute(q)]


def from_csv(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                         float(r["MinNs"]), float(r["MaxNs"])))
    return sorted(rows, key=lambda r: -r[2])


def probe_rows(path, name_like="conv_fwd_direct_poolILi48E", grid=(8192, 1, 1)):
    """Dispatches of a bench roofline probe kernel by name and grid (workgroups x, y, z) — the per-launch average to
    compare with bench.py's roofline avg_us. Probe replays after the timed steps are included."""
    con = sqlite3.connect(path)
    q = """select d.end - d.start from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           where s.kernel_name like ? and d.grid_size_x / d.workgroup_size_x = ? and d.grid_size_y = ?
           and d.grid_size_z = ?"""
    try:
        return [r[0] for r in con.execute(q, (f"%{name_like}%",) + tuple(grid))]
    except sqlite3.OperationalError:
        return []


def main(path, top=40, per=1):
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    if path.endswith(".db"):
        for label, pat, grid in (("roofline kernel k_lin<32, 32> x3 (imagination, grid 8x32x3)", "k_linILi32ELi32E",
                                  (8, 32, 3)),
                                 ("secondary conv_fwd_direct_pool<48> (encoder stage 2, 8192 workgroups)",
                                  "conv_fwd_direct_poolILi48E", (8192, 1, 1))):
            pr = probe_rows(path, pat, grid)
            if pr:
                print(f"{label}: {len(pr)} dispatches, avg {sum(pr) / len(pr) / 1e3:.1f} us, "
                      f"min {min(pr) / 1e3:.1f} us\n")
    tot = sum(r[2] for r in rows)
    print(f"total kernel time {tot / 1e6:.2f} ms over the profiled run ({tot / 1e6 / per:.2f} ms per step, {per} steps)")
    print("| share | total ms | calls | avg us | kernel |")
    print("|---:|---:|---:|---:|---|")
    for name, n, t, avg, mn, mx in rows[:top]:
        print(f"| {100 * t / tot:5.1f}% | {t / 1e6:8.2f} | {n} | {avg / 1e3:8.1f} | `{name[:110]}` |")


if __name__ == "__main__":
    main(sys.argv[1], per=int(sys.argv[2]) if len(sys.argv) > 2 else 1)
