"""Per-phase kernel list of one graph-replayed update from a rocprofv3 kernel-trace database of tools/timeline.py
(SDREAMER_MARKS=1): the device marks (mark_kernel dispatches) split each queue's dispatches into phases; prints, per
phase of the LAST update, the kernels in order with their durations, and a per-phase summary.
Usage: python tools/phase_kernels.py run.db [kernels listed per phase]"""
import sqlite3
import sys
from collections import defaultdict


def main(path, top=12):
    con = sqlite3.connect(path)
    cols = [r[1] for r in con.execute("pragma table_info(rocpd_kernel_dispatch)")]
    qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    q = f"""select s.kernel_name, d.start, d.end, {('d.' + qcol) if qcol else '0'} from rocpd_kernel_dispatch d
            join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"""
    rows = list(con.execute(q))
    marks = [r for r in rows if "mark_kernel" in r[0]]
    # the last update: from the last "start" mark (first mark of an update on the main queue) to the end
    starts = [i for i, r in enumerate(rows) if "mark_kernel" in r[0]]
    if not starts:
        print("no marks in trace")
        return
    # group marks per update: an update begins where the gap between consecutive marks on the main queue is largest
    main_q = marks[0][3]
    mq = [r for r in marks if r[3] == main_q]
    n_upd = max(1, len(mq) // max(1, len(set(1 for _ in mq))))
    t0 = mq[-(len(mq) // 8 if len(mq) >= 8 else len(mq))][1] if False else None
    # simplest robust choice: the last 30 ms of the trace
    tend = rows[-1][2]
    last = [r for r in rows if r[1] >= tend - 30e6]
    byq = defaultdict(list)
    for r in last:
        byq[r[3]].append(r)
    for qid, rs in byq.items():
        print(f"== queue {qid}: {len(rs)} dispatches")
        phase, pt, acc = 0, None, defaultdict(float)
        seg = []
        for name, s, e, _ in rs:
            if "mark_kernel" in name:
                if seg:
                    tot = sum(x[1] for x in seg)
                    span = (seg[-1][2] - seg[0][3]) / 1e3
                    agg = defaultdict(lambda: [0, 0.0])
                    for n, d, _, _ in seg:
                        agg[n][0] += 1
                        agg[n][1] += d
                    print(f"  phase {phase}: {len(seg)} kernels, busy {tot / 1e3:.1f} us, span {span:.1f} us")
                    for n, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
                        print(f"      {d / 1e3:8.1f} us {c:4d}x  {n[:100]}")
                phase += 1
                seg = []
                continue
            seg.append((name, e - s, e, s))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
