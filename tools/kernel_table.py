"""Per-update kernel table of bench.py's timed steps: every (kernel, launch grid) pair ranked by its time per update,
joined with the per-dispatch PMC counters of the round's separate --pmc passes.

Usage: python tools/kernel_table.py <trace_dir> <steps> <out.json> [<pmc_dir> ...]  (prints markdown)

bench.py brackets its K timed steps with two empty dispatches (sd_trace_mark: k_trace_mark with 1 and 2 workgroups),
so warm-up updates, graph captures, the probes' re-launches and the per-phase re-runs after the timed steps are all
outside the window. Per (kernel, grid): launches per update and ms per update (trace durations inside the window,
divided by K), the average launch, and from the PMC passes (per-dispatch averages over every dispatch of the same
kernel and grid — the counters cannot be windowed, a shape's dispatches are the same work wherever they run):
  HBM bytes = 2 x FETCH_SIZE (gfx950: FETCH_SIZE reports half of wide coalesced reads) + WRITE_SIZE (KB -> B)
  clock GHz = the in-kernel clock probe of the profiled bench line (KT_BENCH_LOG: sd_clock_probe, s_memtime over
              s_memrealtime), else GRBM_GUI_ACTIVE / 8 XCDs / duration for >= 0.3 ms dispatches,
  mfma util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clk x dur),
  L2 hit %  = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum).
bench.py reads the JSON (its kernel_table path is explicit, not the newest file) to name the top launch shapes it
probes live and to attach their counter traffic."""
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_table import _db, counters, short  # noqa: E402

MARK_US = []
LONG_US = 300.0  # dispatches at least this long carry their own GRBM-derived clock


def probe_clock(log):
    """mean of the bench line's clock_ghz_mfma_load (in-kernel sd_clock_probe), or None"""
    if not log or not os.path.exists(log):
        return None
    for line in open(log):
        if line.startswith("{") and "clock_ghz_mfma_load" in line:
            v = [c for c in json.loads(line).get("clock_ghz_mfma_load") or [] if c]
            return sum(v) / len(v) if v else None
    return None


def window(tdir):
    con = _db(tdir)
    q = """select s.kernel_name, d.grid_size_x, d.grid_size_y, d.grid_size_z, d.workgroup_size_x, d.start, d.end
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"""
    rows = [(short(kn), gx // max(wx, 1), gy, gz, st, en) for kn, gx, gy, gz, wx, st, en in con.execute(q)]
    marks = [(r[1], r[4], r[5]) for r in rows if r[0].startswith("k_trace_mark")]
    b = [m for m in marks if m[0] == 1]
    e = [m for m in marks if m[0] == 2]
    if not b or not e:
        raise SystemExit("no k_trace_mark window in the trace (bench.py too old?)")
    t0, t1 = b[-1][2], e[-1][1]
    global MARK_US
    MARK_US = [(m[2] - m[1]) / 1e3 for m in (b[-1], e[-1])]  # durations of the two empty dispatches
    out = collections.defaultdict(list)
    for k, gx, gy, gz, st, en in rows:
        if t0 <= st and en <= t1 and not k.startswith("k_trace_mark"):
            out[(k, gx, gy, gz)].append(en - st)
    return out, (t1 - t0)


def main(tdir, steps, out_json, *pdirs):
    steps = int(steps)
    tr, span = window(tdir)
    cs = collections.defaultdict(dict)
    for p in pdirs:
        if _db(p) is None:
            continue
        for k, d in counters(p).items():
            for cn, vals in d.items():
                cs[k][cn] = sum(vals) / len(vals)
    total = sum(sum(v) for v in tr.values())
    rows = []
    for key, durs in sorted(tr.items(), key=lambda kv: -sum(kv[1])):
        k, gx, gy, gz = key
        avg = sum(durs) / len(durs)
        c = cs.get(key, {})
        r = {"kernel": k, "grid": [gx, gy, gz], "launches_per_update": len(durs) / steps,
             "ms_per_update": sum(durs) / steps / 1e6, "avg_us": avg / 1e3, "share": sum(durs) / total}
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            r["hbm_bytes"] = 1024.0 * (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0))
        if "GRBM_GUI_ACTIVE" in c:
            r["_grbm_clk"] = c["GRBM_GUI_ACTIVE"] / 8 / avg  # cycles per ns = GHz (trustworthy >= 0.3 ms only)
            r["_mfma_busy"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if "TCC_HIT_sum" in c:
            h, m = c["TCC_HIT_sum"], c.get("TCC_MISS_sum", 0.0)
            r["l2_hit"] = h / (h + m) if h + m else None
        rows.append(r)
    # GRBM_GUI_ACTIVE / duration reads high (4-6 GHz) on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md); those
    # rows take the median clock of this run's >= 0.3 ms dispatches (same run, same DVFS state), and MFMA utilisation
    # is derived from whichever clock the row carries
    long_clk = sorted(r["_grbm_clk"] for r in rows if "_grbm_clk" in r and r["avg_us"] >= LONG_US)
    ref_clk = long_clk[len(long_clk) // 2] if long_clk else None
    # the PMC pass that holds GRBM_GUI_ACTIVE runs the dispatches serialised while the durations come from the
    # two-stream trace, so even a long dispatch's GRBM / duration can read above the part's clock (2.56 GHz measured).
    # When the profiled bench line carries the in-kernel clock probe (sd_clock_probe: s_memtime over s_memrealtime
    # under an MFMA load, before and after the timed steps), every row uses it; GRBM stays a diagnostic column.
    probe = probe_clock(os.environ.get("KT_BENCH_LOG"))
    if probe is not None:
        ref_clk = probe
    for r in rows:
        g = r.pop("_grbm_clk", None)
        busy = r.pop("_mfma_busy", None)
        if g is None:
            continue
        if probe is not None:
            clk, r["clock_source"] = probe, "sd_clock_probe (bench line clock_ghz_mfma_load, mean)"
            if r["avg_us"] >= LONG_US:
                r["grbm_clock_ghz"] = g
        elif r["avg_us"] >= LONG_US or ref_clk is None:
            clk, r["clock_source"] = g, "GRBM_GUI_ACTIVE / duration"
        else:
            clk, r["clock_source"] = ref_clk, f"median of the >= {LONG_US:.0f} us dispatches"
        r["clock_ghz"] = clk
        if busy is not None:
            r["mfma_util"] = busy / (1024 * clk * r["avg_us"] * 1e3)
    res = {"empty_dispatch_us": MARK_US, "reference_clock_ghz": ref_clk, "steps": steps, "window_ms_per_update": span / steps / 1e6, "kernel_ms_per_update": total / steps / 1e6,
           "trace_dir": os.path.basename(os.path.normpath(tdir)), "rows": rows}
    json.dump(res, open(out_json, "w"), indent=1)
    print(f"timed window: {span / steps / 1e6:.3f} ms per update ({steps} updates); kernel time "
          f"{total / steps / 1e6:.3f} ms per update (two streams overlap); an empty dispatch (k_trace_mark) lasts "
          f"{MARK_US[0]:.2f} / {MARK_US[1]:.2f} us in this trace\n")
    print("| rank | ms/update | share | launches/update | avg us | kernel | grid | HBM MB/launch | clock GHz | "
          "mfma util | L2 hit |")
    print("|---:|---:|---:|---:|---:|---|---|---:|---:|---:|---:|")
    for i, r in enumerate(rows[:40]):
        f = lambda x, fmt: (fmt % x) if x is not None else "—"  # noqa: E731
        print(f"| {i + 1} | {r['ms_per_update']:.3f} | {100 * r['share']:.1f}% | {r['launches_per_update']:g} | "
              f"{r['avg_us']:.1f} | `{r['kernel']}` | {'x'.join(map(str, r['grid']))} | "
              f"{f(r.get('hbm_bytes', None) and r['hbm_bytes'] / 1e6, '%.1f')} | {f(r.get('clock_ghz'), '%.2f')} | "
              f"{f(r.get('mfma_util'), '%.2f')} | {f(r.get('l2_hit'), '%.2f')} |")


if __name__ == "__main__":
    main(*sys.argv[1:])
