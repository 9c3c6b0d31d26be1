set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_zstd.py tests/test_gpu_collisions.py tests/test_gpu_fullsize.py > gpurun_out/gpu_tests.txt 2>&1 && tail -2 gpurun_out/gpu_tests.txt && \
VARIANTS="zm0 cur" CODEC=zstd KINDS=1,2,5,6 ROUNDS=2 bash scripts/ab.sh > gpurun_out/ab_zm.txt 2>&1 && \
python3 - <<'PY'
import json,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/ab_zm.txt'):
    if l.startswith('=='): cur=l.split()[1]; continue
    if l.startswith('{'):
        j=json.loads(l); d[(j['codec'],j['kind'],cur)].append(j['compress_ms'])
for k,v in sorted(d.items()): print(k, [round(x,3) for x in v])
PY
