"""Per-kernel averages of every PMC counter in one or more rocprofv3 --pmc result directories (markdown).

Usage: python tools/pmc_kernel_avg.py <filter-substring> <pmc_dir>...   (kernels whose short name contains the filter)
Rows: (kernel, grid); columns: per-dispatch average of each counter (raw units: SQ cycle counters in quad-cycles,
see MI355X_MICROARCH.md 's_memtime tick vs SQ PMC units')."""
import collections
import sys

from pmc_table import _db, counters


def main(filt, *dirs):
    rows = collections.defaultdict(dict)
    names = []
    for d in dirs:
        if _db(d) is None:
            continue
        for k, cs in counters(d).items():
            if filt not in k[0]:
                continue
            for cn, vals in cs.items():
                rows[k][cn] = sum(vals) / len(vals)
                if cn not in names:
                    names.append(cn)
    for k in sorted(rows):
        print(f"### `{k[0]}` grid {k[1]}x{k[2]}x{k[3]}")
        for cn in names:
            if cn in rows[k]:
                print(f"- {cn}: {rows[k][cn]:.4g}")
        print()


if __name__ == "__main__":
    main(*sys.argv[1:])
