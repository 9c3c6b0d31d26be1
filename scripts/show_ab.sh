#!/bin/bash
# print gpurun_out/ab.txt (kernel_bench lines) and the stock-decode legs of each variant
cd "$(dirname "$0")/.."
grep -v "^$\|amdgpu.ids" gpurun_out/ab.txt | python3 -c "
import sys, json
cur = None
for l in sys.stdin:
    if l.startswith('=='):
        cur = l.split()[1]; continue
    d = json.loads(l); print(cur, d['kind'], d['ratio'], d['compress_ms'], d['decompress_ms'])
"
for v in ${VARIANTS:-base cur}; do
  [ -f gpurun_out/bst_$v.json ] && python3 -c "
import json; d = json.load(open('gpurun_out/bst_$v.json'))
print('$v', {k: v['avg_launch_ms'] for k, v in d['stock_decode'].items()})"
done
[ -f gpurun_out/ss.txt ] && grep -v amdgpu gpurun_out/ss.txt
true
