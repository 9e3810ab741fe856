"""Dump a rocprofv3 --pmc results db as a compact per-dispatch CSV (kernel, grid, workgroup, counters...)."""
import collections
import csv
import glob
import sqlite3
import sys


def main(root, out):
    db = sqlite3.connect(glob.glob(root + "/**/*.db", recursive=True)[0])
    rows = db.execute("select dispatch_id, kernel_name, grid_size_x, grid_size_y, workgroup_size_x, counter_name, "
                      "value from counters_collection").fetchall()
    disp = collections.OrderedDict()
    names = set()
    for did, kn, gx, gy, wx, cn, v in rows:
        d = disp.setdefault(did, {"kernel": kn.replace("(anonymous namespace)::", "")[:150], "grid": f"{gx}x{gy}",
                                  "wg": wx})
        d[cn] = d.get(cn, 0) + v
        names.add(cn)
    cols = ["kernel", "grid", "wg"] + sorted(names)
    with open(out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for d in disp.values():
            w.writerow(d)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
