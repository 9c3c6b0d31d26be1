set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VARIANTS="cur zl_ilp zl_def zd_ilp" CODEC=zstd KINDS=1,2,5 ROUNDS=2 bash scripts/ab.sh > gpurun_out/ab_zsched.txt 2>&1 && \
python3 - <<'PY'
import json,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/ab_zsched.txt'):
    if l.startswith('=='): cur=l.split()[1]; continue
    if l.startswith('{'):
        j=json.loads(l); d[(j['kind'],cur)].append(j['decompress_ms'])
for k,v in sorted(d.items()): print(k, [round(x,3) for x in v])
PY
