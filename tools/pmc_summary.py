"""Per-kernel PMC summary from a rocprofv3 --pmc results db: sums each counter over a kernel's dispatches and
prints the SQ cycle breakdown (WAIT_ANY = parked on s_waitcnt / barrier, WAIT_INST_ANY = issue stall,
ACTIVE_INST_ANY = issuing; quad-cycles) and MFMA busy share."""
import collections
import sqlite3
import sys


def main(path, pattern=""):
    db = sqlite3.connect(path)
    rows = db.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection").fetchall()
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for name, did, cn, v in rows:
        if pattern and pattern not in name:
            continue
        short = name.replace("void ", "").replace("(anonymous namespace)::", "")
        short = short.split("(")[0][:60] or name[:60]
        agg[short][cn] += v
        disp[short].add(did)
    items = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
    print(f"{'kernel':60s} {'disp':>5s} {'wait%':>6s} {'stall%':>7s} {'active%':>8s} {'mfma%busy':>9s} {'ldsconf%':>8s}")
    for k, c in items[:25]:
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        busy = c.get("SQ_BUSY_CYCLES", 0) or 1
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0) or 1
        print(f"{k:60s} {len(disp[k]):5d} {100 * c.get('SQ_WAIT_ANY', 0) / wc:6.1f} "
              f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:7.1f} {100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc:8.1f} "
              f"{100 * c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (busy * 4 * 4):9.1f} "
              f"{100 * c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
