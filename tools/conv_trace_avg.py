"""Average duration of the sdmoe_conv3x3 launches in a rocprofv3 kernel trace, for cross-checking bench.py's
HIP-event roofline timing: conv launches are gemm_kernel instances with MODE (5th template argument) 1 or 2;
a split-K reduce dispatched right after one belongs to that launch.

usage: python tools/conv_trace_avg.py gpurun_out/<dir>/run_kernel_trace.csv"""
import csv
import re
import sys

PAT = re.compile(r"gemm_kernel<\d+, \d+, \d+, \d+, (\d+), \d+, \d+>")


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    n = tot = red = 0
    prev_conv = False
    for r in rows:
        name = r["Kernel_Name"]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        m = PAT.search(name)
        if m and m.group(1) in ("1", "2"):
            n += 1
            tot += d
            prev_conv = True
        elif "splitk_reduce" in name and prev_conv:
            red += d
            prev_conv = False
        else:
            prev_conv = False
    print(f"conv launches {n}: gemm avg {tot / n / 1e3:.1f} us, incl. split-K reduce {(tot + red) / n / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
