"""Join a rocprofv3 kernel-trace db with PMC-pass dbs into one per-kernel table (markdown).

Usage: python tools/pmc_table.py <trace_dir> <pmc_dir>...   (directories holding rocprofv3 .db results)

Per (kernel, grid) group: dispatches, average duration (trace pass), and per-dispatch averages of every counter
found in the PMC passes, with derived columns:
  clock GHz   = GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md 'DVFS give-back': reads high below ~0.3 ms)
  mfma util   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clock x duration)
  waves/CU    = 4 x SQ_WAVE_CYCLES (quad-cycles summed over waves) / (256 CUs x clock x duration): mean resident waves
  wait/stall/active % of SQ_WAVE_CYCLES (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY)
  HBM bytes   = 2 x FETCH_SIZE (gfx950: FETCH_SIZE reports half of wide coalesced reads) + WRITE_SIZE, KB -> B
  L2 hit %    = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
Durations come from a separate un-instrumented pass, so the derived clock / utilisation mix two runs (stated)."""
import collections
import glob
import sqlite3
import sys


def _db(d):
    fs = glob.glob(d + "/**/*.db", recursive=True)
    return sqlite3.connect(fs[0]) if fs else None


_DEM = {}


def short(name):
    """demangled base name with template arguments (trace dbs hold mangled names, PMC dbs demangled ones)"""
    if name not in _DEM:
        s = name
        if s.startswith("_Z"):
            import subprocess
            s = subprocess.run(["c++filt"], input=s.replace(".kd", ""), capture_output=True, text=True).stdout.strip()
        s = s.replace("void ", "").replace("(anonymous namespace)::", "").replace("sdg::", "").replace("sdb::", "")
        _DEM[name] = s.split("(")[0][:70]
    return _DEM[name]


def trace(d):
    con = _db(d)
    q = """select s.kernel_name, d.grid_size_x, d.grid_size_y, d.grid_size_z, d.workgroup_size_x, d.end - d.start
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id"""
    out = collections.defaultdict(list)
    for kn, gx, gy, gz, wx, dt in con.execute(q):
        out[(short(kn), gx // max(wx, 1), gy, gz)].append(dt)
    return out


def counters(d):
    con = _db(d)
    cols = [r[1] for r in con.execute("pragma table_info(counters_collection)")]
    gz = "grid_size_z" if "grid_size_z" in cols else "1"
    q = f"""select kernel_name, dispatch_id, grid_size_x, grid_size_y, {gz}, workgroup_size_x, counter_name, value
            from counters_collection"""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    key_of = {}
    for kn, did, gx, gy, gzv, wx, cn, v in con.execute(q):
        key_of[did] = (short(kn), gx // max(wx, 1), gy, gzv)
        per[did][cn] += v
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for did, cs in per.items():
        for cn, v in cs.items():
            out[key_of[did]][cn].append(v)
    return out


def main(tdir, *pdirs):
    tr = trace(tdir)
    cs = collections.defaultdict(dict)
    for p in pdirs:
        if _db(p) is None:
            continue
        for k, d in counters(p).items():
            for cn, vals in d.items():
                cs[k][cn] = sum(vals) / len(vals)
    rows = sorted(tr.items(), key=lambda kv: -sum(kv[1]))
    tot = sum(sum(v) for v in tr.values())
    print(f"kernel trace: {sum(len(v) for v in tr.values())} dispatches, {tot / 1e6:.2f} ms of kernel time\n")
    print("| share | kernel | grid (wg x, y, z) | n | avg us | clock GHz | mfma util | waves/CU | wait % | stall % | "
          "active % | HBM MB/disp | L2 hit % |")
    print("|---:|---|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, ts in rows[:45]:
        avg = sum(ts) / len(ts)
        c = cs.get(k, {})
        gui, mf, wc = c.get("GRBM_GUI_ACTIVE"), c.get("SQ_VALU_MFMA_BUSY_CYCLES"), c.get("SQ_WAVE_CYCLES")
        clk = gui / 8 / (avg * 1e-9) / 1e9 if gui else None
        util = mf / (1024 * clk * 1e9 * avg * 1e-9) if (mf is not None and clk) else None
        wpc = 4 * wc / (256 * clk * 1e9 * avg * 1e-9) if (wc and clk) else None
        f, w = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
        hbm = (2 * f + w) * 1024 / 1e6 if (f is not None and w is not None) else None
        h, m = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        hit = 100 * h / (h + m) if (h is not None and m is not None and h + m > 0) else None

        def fmt(x, s="{:.2f}"):
            return s.format(x) if x is not None else "-"
        pct = (lambda n: fmt(100 * c[n] / wc, "{:.0f}") if (wc and n in c) else "-")
        print(f"| {100 * sum(ts) / tot:.1f}% | `{k[0]}` | {k[1]}x{k[2]}x{k[3]} | {len(ts)} | {avg / 1e3:.1f} | "
              f"{fmt(clk)} | {fmt(util)} | {fmt(wpc, '{:.1f}')} | {pct('SQ_WAIT_ANY')} | {pct('SQ_WAIT_INST_ANY')} | "
              f"{pct('SQ_ACTIVE_INST_ANY')} | {fmt(hbm, '{:.1f}')} | {fmt(hit, '{:.0f}')} |")
    import os
    for k, ts in rows[:int(os.environ.get("PMC_RAW", "0"))]:  # every counter of the top kernels, per dispatch
        print(f"\n### `{k[0]}` {k[1]}x{k[2]}x{k[3]} ({sum(ts) / len(ts) / 1e3:.1f} us)")
        for cn, v in sorted(cs.get(k, {}).items()):
            print(f"- {cn}: {v:.4g}")


if __name__ == "__main__":
    main(*sys.argv[1:])
