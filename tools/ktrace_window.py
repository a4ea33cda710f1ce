"""Per-kernel summary of the timed steps only: reads a rocprofv3 kernel_trace.csv, keeps the kernels
between the two marker kernels bench.py launches when AVSE_PROFILE_MARK=1 (torch.cuda._sleep -> spin_kernel), and
prints / writes the same columns as rocprofv3's kernel_stats.csv.
usage: ktrace_window.py TRACE.csv STEPS OUT_STATS.csv [OUT_POST.csv [OUT_ROOF.csv]]
OUT_POST.csv: the same summary for the kernels after the second marker -- bench.py's isolated roofline /
roofline_hip measurements, which run after the timed steps (their averages are the live numbers' counterpart;
the whole-run rocprof average mixes them with the in-step calls, which overlap the avse1 lip stream).
OUT_ROOF.csv: with the avse1 workload's in-step roofline (bench.py Avse1Step.roofline brackets its 3 eager train
steps with markers 3 and 4), the summary of those steps: the kernel averages the line's `roofline.avg_ms` is."""
import csv
import sys
from collections import defaultdict

trace, steps, out = sys.argv[1], float(sys.argv[2]), sys.argv[3]
post_out = sys.argv[4] if len(sys.argv) > 4 else None
rows = []
queue_of = {}
with open(trace) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
        q = r.get("Stream_Id") or r.get("Queue_Id")
        if q is not None:
            queue_of[rows[-1]] = q
rows.sort()
marks = [i for i, r in enumerate(rows) if "spin_kernel" in r[2]]
if len(marks) < 2:
    sys.exit(f"expected 2 marker kernels, found {len(marks)}")
win = rows[marks[0] + 1:marks[1]]


def write_stats(sel, path):
    agg = defaultdict(list)
    for s, e, n in sel:
        agg[n].append(e - s)
    tot = sum(sum(v) for v in agg.values())
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([n, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / max(1, tot), min(v), max(v)])
    return tot


tot = write_stats(win, out)
span = win[-1][1] - win[0][0]
if post_out:
    write_stats(rows[marks[1] + 1:], post_out)
roof_out = sys.argv[5] if len(sys.argv) > 5 else None
if roof_out and len(marks) >= 4:
    write_stats(rows[marks[2] + 1:marks[3]], roof_out)
print(f"timed window: {span / 1e6:.2f} ms wall, {tot / 1e6:.2f} ms kernel busy "
      f"({tot / 1e6 / steps:.2f} ms/step over {steps:g} steps, {len(win)} launches)")


def union_ns(iv):
    """total length of the union of [s, e) intervals"""
    tot, cur_s, cur_e = 0, None, None
    for s_, e_ in sorted(iv):
        if cur_e is None or s_ > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s_, e_
        else:
            cur_e = max(cur_e, e_)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


if queue_of:
    # per stream / queue: the union of its kernels' intervals in the timed window (the branch with the most busy time
    # bounds the step when the branches overlap); all streams together: the GPU's busy union
    per = defaultdict(list)
    for r in win:
        per[queue_of.get(r, "?")].append((r[0], r[1]))
    allb = union_ns([(r[0], r[1]) for r in win])
    print(f"busy union of all streams: {allb / 1e6 / steps:.2f} ms/step (wall {span / 1e6 / steps:.2f})")
    for q, iv in sorted(per.items(), key=lambda kv: -union_ns(kv[1])):
        print(f"  stream/queue {q}: {union_ns(iv) / 1e6 / steps:.2f} ms/step busy, {len(iv) / steps:.0f} launches/step")
