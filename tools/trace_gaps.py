"""Idle gaps between consecutive kernels in a rocprofv3 --kernel-trace CSV (one stream's dispatch gaps: how much of
the wall clock the GPU is NOT running a kernel while the host keeps it fed).

usage: python tools/trace_gaps.py KERNEL_TRACE_CSV [--max-gap-us 200]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--max-gap-us", type=float, default=200.0, help="larger gaps count as host phases, not dispatch")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    busy = 0
    gaps = []
    end = iv[0][0]
    for s, e, _ in iv:
        if s > end:
            gaps.append((s - end) / 1e3)
        busy += max(0, e - max(s, end))
        end = max(end, e)
    span = (iv[-1][1] - iv[0][0]) / 1e3
    small = [g for g in gaps if g <= a.max_gap_us]
    print(f"kernels {len(iv)}  span {span / 1e3:.1f} ms  busy {busy / 1e6:.1f} ms ({busy / 1e3 / span:.3f})")
    print(f"gaps <= {a.max_gap_us:.0f} us: {len(small)}, total {sum(small) / 1e3:.2f} ms, "
          f"mean {sum(small) / max(1, len(small)):.2f} us; larger gaps: {len(gaps) - len(small)}, "
          f"total {(sum(gaps) - sum(small)) / 1e3:.1f} ms")
    for lo, hi in [(0, 1), (1, 2), (2, 4), (4, 8), (8, 16), (16, 50), (50, a.max_gap_us)]:
        sel = [g for g in small if lo <= g < hi]
        print(f"  [{lo:5.0f},{hi:5.0f}) us: {len(sel):7d} gaps, {sum(sel) / 1e3:8.2f} ms")


if __name__ == "__main__":
    main()
