#!/bin/bash
# B = 1 (nimg 2) split-K sweep of the conv / linear shapes: knob 9 forced split factor (0 = auto)
set -u
O=gpurun_out/b1_split; mkdir -p $O
for k in 0 4 8 12 16 20 32; do
  SDMOE_TUNE=9=$k timeout -k 10 200 python tools/gemm_bench.py --nimg 2 --iters 50 > $O/k$k.log 2>&1 || { echo "FAILED $k"; tail -5 $O/k$k.log; exit 1; }
done
python3 - <<'PY'
import re
rows = {}
ks = [0, 4, 8, 12, 16, 20, 32]
for k in ks:
    for l in open(f"gpurun_out/b1_split/k{k}.log"):
        m = re.match(r"(\S.*?)\s+([\d.]+) us", l)
        if m and (m.group(1).startswith("conv") or m.group(1).startswith("linear")):
            rows.setdefault(m.group(1).strip(), {})[k] = float(m.group(2))
print("shape".ljust(40) + "".join(f"{'9=' + str(k):>9s}" for k in ks))
for name, v in rows.items():
    print(name.ljust(40) + "".join(f"{v.get(k, 0):9.1f}" for k in ks))
PY
