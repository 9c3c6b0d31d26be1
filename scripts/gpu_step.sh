set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lz4.py tests/test_gpu_fullsize.py tests/test_gpu_mutations.py > gpurun_out/gpu_tests.txt 2>&1 && tail -2 gpurun_out/gpu_tests.txt && \
VARIANTS="split0 cur" CODEC=lz4 KINDS=0,1,2,5,6 ROUNDS=3 bash scripts/ab.sh > gpurun_out/ab_k.txt 2>&1 && \
python3 - <<'PY'
import json,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/ab_k.txt'):
    if l.startswith('=='): cur=l.split()[1]; continue
    if l.startswith('{'):
        j=json.loads(l); d[(j['codec'],j['kind'],cur)].append(j['decompress_ms'])
for k,v in sorted(d.items()): print(k, [round(x,3) for x in v])
PY
