#!/usr/bin/env python3
"""Where a VO run's wall time goes, from a rocprofv3 kernel trace (run_kernel_trace.csv):
  python tools/vo_timeline.py TRACE.csv [last_ms]
Per stream (the VO schedule puts each chain on its own stream, the frame->next chunks on a side
stream): kernels in start order, busy time by kernel name, and the gaps between one kernel's end
and the next one's start on the same stream (launch latency or an event wait).  Over the whole
device: the time with 0, 1, 2, 3+ kernels running.  Only the last `last_ms` of the trace is read
(default: everything), so a timed region at the end of a run can be isolated."""
import collections
import csv
import sys


def short(name):
    for key in ("picp_match_mfma", "picp_block_kernel", "vo_append", "vo_gather", "picp_match_prep",
                "picp_persistent", "picp_round", "fillBuffer", "copyBuffer"):
        if key in name:
            return key
    return name[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id") or r.get("Queue_Id"),
           short(r["Kernel_Name"])) for r in rows]
    ks.sort()
    if len(sys.argv) > 2:
        t_end = max(k[1] for k in ks)
        ks = [k for k in ks if k[0] >= t_end - float(sys.argv[2]) * 1e6]
    t0, t1 = min(k[0] for k in ks), max(k[1] for k in ks)
    print("window %.3f ms, %d kernels" % ((t1 - t0) / 1e6, len(ks)))
    by_stream = collections.defaultdict(list)
    for k in ks:
        by_stream[k[2]].append(k)
    for s, lst in sorted(by_stream.items(), key=lambda kv: kv[1][0][0]):
        busy = collections.Counter()
        cnt = collections.Counter()
        gaps = []
        for i, (a, b, _, n) in enumerate(lst):
            busy[n] += b - a
            cnt[n] += 1
            if i:
                gaps.append(max(0, a - lst[i - 1][1]))
        span = lst[-1][1] - lst[0][0]
        gsum = sum(gaps)
        print("stream %s: %d kernels, span %.3f ms, busy %.3f ms, gaps %.3f ms (median gap %.1f us)" % (
            s, len(lst), span / 1e6, sum(busy.values()) / 1e6, gsum / 1e6,
            sorted(gaps)[len(gaps) // 2] / 1e3 if gaps else 0.0))
        for n, v in busy.most_common():
            print("    %-20s %5d launches  %8.3f ms  %7.1f us each" % (n, cnt[n], v / 1e6, v / 1e3 / cnt[n]))
    # device concurrency profile
    ev = []
    for a, b, _, _ in ks:
        ev.append((a, 1))
        ev.append((b, -1))
    ev.sort()
    level, last, hist = 0, ev[0][0], collections.Counter()
    for t, d in ev:
        hist[min(level, 3)] += t - last
        level += d
        last = t
    tot = sum(hist.values())
    print("device: " + ", ".join("%s running %.1f %%" % ("3+" if l == 3 else l, 100.0 * hist[l] / tot)
                                 for l in range(4)))


if __name__ == "__main__":
    main()
