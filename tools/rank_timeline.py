"""Timeline of one steady-state step from a rocprofv3 --kernel-trace database (rocpd SQLite, the
`rankprof` session step: tools/c4_rank_cost.py --variants block,rccl under rocprofv3): the step's
sub-cycle and glue spans, the kernel sums per family, the idle time, and a window of stage launches
with their start/end (B on the high-priority stream, I, the RCCL transport).
Usage: python tools/rank_timeline.py <rp_results.db>"""
import collections
import sqlite3
import sys


def load(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, queue_id, start, end, grid_x from kernels order by start"))
    return [(r[0].split("(")[0].replace("void ", "").replace("hnumo::", "")[:28],) + r[1:] for r in rows]


def step(rows, a, b, label):
    seg = rows[a:b]
    t0, t1 = seg[0][2], seg[-1][3]
    iv = sorted((r[2], r[3]) for r in seg)
    busy, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            busy, cs, ce = busy + ce - cs, s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"{label}: step span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f}, idle {(t1 - t0 - busy) / 1e3:.1f}")
    st = [i for i, r in enumerate(seg) if r[0].startswith("btp_stage")]
    groups, cur = [], [st[0]]
    for i in st[1:]:
        if all(seg[j][0].startswith("nccl") for j in range(cur[-1] + 1, i)):
            cur.append(i)
        else:
            groups.append(cur)
            cur = [i]
    groups.append(cur)
    prev = t0
    for g in groups:
        s, e = seg[g[0]][2], max(seg[j][3] for j in g)
        print(f"  glue {(s - prev) / 1e3:8.1f} us | sub-cycle {(e - s) / 1e3:8.1f} us ({len(g)} stage launches)")
        prev = e
    print(f"  glue {(t1 - prev) / 1e3:8.1f} us")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        agg[r[0]][0] += 1
        agg[r[0]][1] += (r[3] - r[2]) / 1e3
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:8]:
        print(f"  {v[0]:4d} x {k:28s} {v[1]:10.1f} us (sum of durations)")
    mid = [r for r in seg if r[0].startswith(("btp_stage", "nccl"))]
    mid = mid[len(mid) // 2: len(mid) // 2 + 9]
    for r in mid:
        print(f"    {r[0]:28s} queue {r[1]} grid {r[4]:8d} start {(r[2] - t0) / 1e3:9.1f} end {(r[3] - t0) / 1e3:9.1f}")


def main():
    rows = load(sys.argv[1])
    me = [i for i, r in enumerate(rows) if r[0].startswith("mom_elem")]
    # c4_rank_cost runs block then rccl, 2 warm-up + timed steps each, 2 mom_elem launches a step
    half = len(me) // 2
    step(rows, me[half - 3] + 1, me[half - 1] + 1, "block (single-rank 79x158, graph)")
    step(rows, me[-3] + 1, me[-1] + 1, "rccl (self-neighbour rank, two streams)")


if __name__ == "__main__":
    main()
