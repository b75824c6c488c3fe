"""Timeline of a pipelined bench run from a rocprofv3 kernel trace (tools/ab_timeline.sh).

For the dispatches of the intra row kernel: how long each runs, how much of the wall time has
0 / 1 / 2+ of them running, and what else runs beside them (per kernel: busy time while an
intra kernel runs vs. while none does).  Usage: python tools/timeline.py <kernel_trace.csv>
"""
import csv
import sys
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name):
    n = name.replace("void ", "").replace("p265r::", "")
    return n.split("(")[0]


def segment(rows):
    """The pipelined stretch: from the first intra dispatch that overlaps another intra dispatch
    to the last one that does (the bench's timed + warmup steps)."""
    intra = [(s, e) for s, e, n in rows if "intra_rows_kernel" in n]
    ov = [i for i in range(len(intra)) if (i > 0 and intra[i][0] < intra[i - 1][1]) or
          (i + 1 < len(intra) and intra[i + 1][0] < intra[i][1])]
    if not ov:
        return None
    return intra[ov[0]][0], intra[ov[-1]][1]


def main(path):
    rows = load(path)
    seg = segment(rows)
    if seg is None:
        print("no overlapping intra dispatches")
        return
    t0, t1 = seg
    rows = [(max(s, t0), min(e, t1), n) for s, e, n in rows if e > t0 and s < t1]
    events = []
    for s, e, n in rows:
        events.append((s, 1, n))
        events.append((e, -1, n))
    events.sort(key=lambda x: (x[0], x[1]))
    run = defaultdict(int)
    by_intra = defaultdict(float)          # wall time with k intra kernels running
    busy = defaultdict(lambda: [0.0, 0.0])   # kernel -> [time running beside intra, without]
    prev = t0
    for t, d, n in events:
        dt = (t - prev) * 1e-6
        k = sum(v for name, v in run.items() if "intra_rows_kernel" in name)
        by_intra[min(k, 2)] += dt
        for name, v in run.items():
            if v > 0 and "intra_rows_kernel" not in name:
                busy[short(name)][0 if k else 1] += dt
        run[n] += d
        prev = t
    wall = (t1 - t0) * 1e-6
    durs = defaultdict(list)
    for s, e, n in rows:
        durs[short(n)].append((e - s) * 1e-6)
    print(f"pipelined stretch {wall:.2f} ms")
    for k in (0, 1, 2):
        print(f"  {k}{'+' if k == 2 else ''} intra kernels running: {by_intra[k]:8.2f} ms ({100 * by_intra[k] / wall:5.1f} %)")
    print("kernel                                   n    avg ms   beside-intra ms  alone ms")
    for name, d in sorted(durs.items(), key=lambda x: -sum(x[1])):
        b = busy.get(name, [0.0, 0.0])
        print(f"  {name:36s} {len(d):5d} {sum(d) / len(d):9.3f} {b[0]:12.2f} {b[1]:12.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
