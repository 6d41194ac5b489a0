#!/bin/bash
# Round-5 first GPU pass: full -m gpu suite, metric bench, hipBLASLt yardstick, attention kernel A/B, SDXL expert union.
set -u
O=gpurun_out/r05a
mkdir -p $O
export SDMOE_PARITY_REPORT=$O/parity_report.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 400 --timeout-method thread \
  > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -3 $O/gputests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python tools/blas_yardstick.py > $O/yardstick.txt 2>&1 || { tail -20 $O/yardstick.txt; exit 1; }
cat $O/yardstick.txt
timeout -k 10 300 python tools/micro_ab.py attn --tune "" --tune "4=1" --tune "4=9" > $O/attn_ab.txt 2>&1 || { tail -20 $O/attn_ab.txt; exit 1; }
cat $O/attn_ab.txt
timeout -k 10 400 python tools/expert_union.py --model sdxl --out $O/expert_union_sdxl.json > $O/expert_union_sdxl.log 2>&1 || { tail -20 $O/expert_union_sdxl.log; exit 1; }
tail -30 $O/expert_union_sdxl.log
