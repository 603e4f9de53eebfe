#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of scripts/headline_trace.py: the dispatches after the
largest start-time gap (the timed steps), their per-kernel durations, how many kernels overlap
(time-weighted), per-queue busy fractions and the idle gaps of the device.
    python scripts/regime_summary.py DIR/.../run_kernel_trace.csv [steps] > profiles/regime_<tag>.json"""
import collections, csv, json, sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "rocclr" not in r["Kernel_Name"]]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [int(r["Start_Timestamp"]) for r in rows]
# the timed steps follow the LAST idle gap of >= 50 ms (headline_trace.py sleeps 100 ms)
big = [i + 1 for i in range(len(st) - 1) if st[i + 1] - st[i] >= 50_000_000]
cut = big[-1] if big else 0
rows = rows[cut:]


def short(n):
    n = n.replace("void ", "").replace("tq::(anonymous namespace)::", "").replace("tq::", "")
    d, o = 0, ""
    for ch in n:
        if ch == "(" and d == 0:
            break
        d += ch == "<"
        d -= ch == ">"
        o += ch
    return o


iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
       r.get("Queue_Id") or r.get("Stream_Id") or "?") for r in rows]
t0 = min(a for a, _, _, _ in iv)
t1 = max(b for _, b, _, _ in iv)
ev = sorted([(a, 1) for a, _, _, _ in iv] + [(b, -1) for _, b, _, _ in iv])
hist = collections.Counter()
cur, last = 0, t0
for t, d in ev:
    hist[cur] += t - last
    cur += d
    last = t
span = t1 - t0
busy = span - hist.get(0, 0)
per = collections.defaultdict(lambda: [0, 0])
for a, b, n, _ in iv:
    per[n][0] += 1
    per[n][1] += b - a
q = collections.defaultdict(int)
for a, b, _, qq in iv:
    q[qq] += b - a
idle = []
cur, last = 0, None
for t, d in ev:
    if cur == 0 and last is not None and t > last:
        idle.append(t - last)
    cur += d
    if cur == 0:
        last = t
out = {
    "dispatches": len(iv), "span_us": span / 1e3, "device_busy_frac": busy / span,
    "ms_per_block_trace": (span / 1e6 / steps) if steps else None,
    "kernel_time_over_span": sum(b - a for a, b, _, _ in iv) / span,
    "overlap_time_frac": {str(k): round(v / span, 4) for k, v in sorted(hist.items())},
    "idle_gaps": {"count": len(idle), "total_us": sum(idle) / 1e3,
                  "max_us": max(idle) / 1e3 if idle else 0.0},
    "queues": {str(k): {"kernel_us": v / 1e3, "frac_of_span": round(v / span, 4)} for k, v in q.items()},
    "kernels": {n: {"count": c, "avg_us": round(t / c / 1e3, 3), "total_us": round(t / 1e3, 1),
                    "frac_of_kernel_time": round(t / sum(x[1] for x in per.values()), 4)}
                for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])},
}
print(json.dumps(out, indent=1))
