"""HBM traffic per launch of the roofline probe kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Selects the dispatches of the probe kernel by name and grid (encoder conv2 fwd: 1M pixels / 128-row tiles = 8192
workgroups), averages per dispatch, applies the gfx950 correction from MI355X_MICROARCH.md (FETCH_SIZE reports half
of the bytes of wide coalesced reads: x2), converts KB -> bytes, and writes a small JSON that bench.py reports as
roofline.traffic."""
import json
import sqlite3
import sys


def per_launch(path, counter, name_like, grid_wgs):
    db = sqlite3.connect(path)
    rows = db.execute("select grid_size_x, workgroup_size_x, value, description from counters_collection "
                      "where counter_name = ? and kernel_name like ?", (counter, f"%{name_like}%")).fetchall()
    vals = [v for gx, wx, v, _ in rows if gx // max(wx, 1) == grid_wgs]
    desc = rows[0][3] if rows else ""
    return (sum(vals) / len(vals) if vals else None), len(vals), desc


# algorithmic bytes per launch: the conv input read once + the stage's outputs written once
ALGO = {
    "conv_fwd16<48>": 4.0 * 1024 * 32 * 32 * (32 + 48),  # NHWC input, full-resolution conv output
    # input + pooled (f32) + y (f32) + argmax (u8) + rstd (f32 per pooled pixel)
    "conv_fwd16_pool<48>": 4.0 * 1024 * 32 * 32 * 32 + 1024 * 16 * 16 * (48 * (4 + 4 + 1) + 4),
    "conv_fwd_direct_pool<48>": 4.0 * 1024 * 32 * 32 * 32 + 1024 * 16 * 16 * (48 * (4 + 4 + 1) + 4),
}


def main(fetch_db, write_db, out, name="conv_fwd_direct_pool<48>"):
    wgs = 8192
    pat = name.rstrip(">")  # demangled names carry further template arguments (e.g. conv_fwd16_pool<48, true>)
    f, nf, fdesc = per_launch(fetch_db, "FETCH_SIZE", pat, wgs)
    w, nw, wdesc = per_launch(write_db, "WRITE_SIZE", pat, wgs)
    kb = 1024.0  # rocprofv3 FETCH_SIZE / WRITE_SIZE are in kilobytes
    res = {"kernel": name, "grid_workgroups": wgs, "algorithmic_bytes": ALGO[name], "dispatches": [nf, nw],
           "fetch_bytes_raw": f * kb if f is not None else None,
           "fetch_bytes": 2 * f * kb if f is not None else None,  # gfx950: FETCH_SIZE = 1/2 of wide reads
           "write_bytes": w * kb if w is not None else None,
           "fetch_desc": fdesc[:160], "write_desc": wdesc[:160]}
    res["traffic_bytes"] = (res["fetch_bytes"] or 0) + (res["write_bytes"] or 0)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
