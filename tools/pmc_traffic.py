"""HBM traffic per launch of a kernel family from rocprofv3 --pmc counter CSVs.

usage: python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv \
           --kernel 'gemm_kernel<' --mode 1 --out profiles/traffic.json

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports exactly half of the bytes of wide
coalesced streaming reads (16 B/lane loads and LDS-DMA alike) -> doubled; WRITE_SIZE (KiB) is exact for
16-B-per-lane stores. Counters are collected in separate passes (one counter group per run).

A split-K launch is two dispatches (the fp32 partial slabs, then splitk_reduce_kernel): a reduce dispatch that directly
follows a kept gemm dispatch is charged to that launch, so bytes_per_launch is per conv op, as bench.py times it."""
import argparse
import csv
import json
import re
from collections import defaultdict


def load(path, counter):
    per = defaultdict(float)
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[d] += float(r["Counter_Value"])
            names[d] = r.get("Kernel_Name", "")
    return per, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--kernel", default="gemm_kernel<")
    ap.add_argument("--mode", default="1,2,9,10,11,12,13,14",
                    help="comma list of gemm_kernel MODE values (5th template arg: 1 = conv, 2 = conv with fused "
                    "upsample, 9-11 halo conv, 12-14 halo conv with fused upsample); '' = any")
    ap.add_argument("--out", default=None)
    ap.add_argument("--build", default="", help="git revision of the measured build (recorded in the json)")
    # the bench workload the PMC passes profiled: bench.py attaches roofline.traffic only to a line of the same
    # model / prompts per GPU / mask (a B = 8 figure on a --batch 1 line would be mislabelled evidence)
    ap.add_argument("--model", default="sd14")
    ap.add_argument("--batch", type=int, required=True, help="bench.py --batch of the profiled run (prompts per GPU)")
    ap.add_argument("--mask", default="remove")
    a = ap.parse_args()
    fetch, names = load(a.fetch_csv, "FETCH_SIZE")
    write, wnames = load(a.write_csv, "WRITE_SIZE")
    pat = re.compile(r"gemm_kernel<\d+, \d+, \d+, \d+, (\d+), \d+, \d+>")
    modes = set(a.mode.split(",")) if a.mode else set()

    def keep(n):
        if a.kernel not in n:
            return False
        if a.mode == "":
            return True
        m = pat.search(n)
        return bool(m) and m.group(1) in modes
    def select(per, nm):
        """per-launch sums: kept gemm dispatches plus the splitk_reduce dispatch right after each one"""
        out, last, nred = [], None, 0
        for d in sorted(per, key=lambda x: int(x)):
            n = nm[d]
            if keep(n):
                out.append(per[d])
                last = len(out) - 1
            elif "splitk_reduce" in n and last is not None:
                out[last] += per[d]
                nred += 1
                last = None
            else:
                last = None
        return out, nred
    f_sel, f_red = select(fetch, names)
    w_sel, w_red = select(write, wnames)
    if not f_sel or not w_sel:
        raise SystemExit("no matching dispatches")
    fetch_b = 2.0 * 1024 * sum(f_sel) / len(f_sel)   # gfx950: FETCH_SIZE counts half of wide reads
    write_b = 1024 * sum(w_sel) / len(w_sel)
    res = {"kernel": a.kernel, "mode": a.mode, "launches_fetch": len(f_sel), "launches_write": len(w_sel),
           "splitk_reduce_dispatches": f_red,
           "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
           "bytes_per_launch": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1; KiB -> bytes",
           "build": a.build, "model": a.model, "batch": a.batch, "mask": a.mask}
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
