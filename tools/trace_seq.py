"""One U-Net evaluation's dispatch sequence from a rocprofv3 --kernel-trace CSV: every kernel between the last two
cfg_ddim_kernel dispatches (one denoising step), with its duration, the idle gap before it, grid and workgroup size.

usage: python tools/trace_seq.py kernel_trace.csv [--out seq.txt]
"""
import argparse
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)
    name = re.sub(r"\((GemmParams|AttnParams)\)$", "", name)
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    if not rows:
        sys.exit("empty trace")
    k = rows[0].keys()
    gx = next((c for c in ("Grid_Size_X", "Grid_Size", "Grid_X") if c in k), None)
    wx = next((c for c in ("Workgroup_Size_X", "Workgroup_Size", "Workgroup_X") if c in k), None)
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                  r.get(gx, "?") if gx else "?", r.get(wx, "?") if wx else "?") for r in rows))
    cut = [i for i, e in enumerate(ev) if "cfg_ddim_kernel" in e[2]]
    if len(cut) < 2:
        sys.exit("need two cfg_ddim_kernel dispatches, found %d" % len(cut))
    seq = ev[cut[-2] + 1:cut[-1] + 1]
    out = []
    busy = sum(e[1] - e[0] for e in seq)
    span = seq[-1][1] - ev[cut[-2]][1]
    out.append("# one denoising step: %d dispatches, span %.1f us, busy %.1f us (%.1f%%)"
               % (len(seq), span / 1e3, busy / 1e3, 100.0 * busy / span))
    out.append("# idx   dur_us  gap_us   grid  wg  kernel")
    prev = ev[cut[-2]][1]
    for i, (s, e, n, g, w) in enumerate(seq):
        out.append("%5d %8.1f %7.1f %6s %3s  %s" % (i, (e - s) / 1e3, (s - prev) / 1e3, g, w, short(n)))
        prev = e
    txt = "\n".join(out) + "\n"
    if a.out:
        open(a.out, "w").write(txt)
    print(txt[:4000])


if __name__ == "__main__":
    main()
